"""Multi-level Haar (BASELINE config 5's 2-level DWT) on the GPU: against
PyWavelets' wavedecn/waverecn golden vectors (the reference's tap source,
tests/golden/pywt_haar3d_wavedec2.npz from oracle/gen_pywt_wavedec_golden.py),
bit-exact composition with the single-level kernel, perfect reconstruction."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"
HIGH = ("LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")


@pytest.mark.parametrize("n", [0, 1, 2])
def test_wavedec2_matches_pywt_golden(n):
    from DWT_IDWT.DWT_IDWT_layer import DWT_3D_Multilevel, IDWT_3D_Multilevel
    g = np.load(os.path.join(GOLDEN, "pywt_haar3d_wavedec2.npz"), allow_pickle=False)
    x = torch.from_numpy(g[f"x{n}"]).float().view(1, 1, *g[f"x{n}"].shape)
    co = DWT_3D_Multilevel("haar", level=2)(x.to(DEV))
    assert np.allclose(co[0].cpu().double().numpy()[0, 0], g[f"x{n}_L2_LLL"], atol=1e-5)
    for lev, d in ((2, co[1]), (1, co[2])):
        for b in HIGH:
            assert np.allclose(d[b].cpu().double().numpy()[0, 0], g[f"x{n}_L{lev}_{b}"], atol=1e-5), (lev, b)
    rec = IDWT_3D_Multilevel("haar")(co).cpu()
    assert np.allclose(rec.double().numpy()[0, 0], g[f"x{n}_rec"], atol=1e-5)


def test_wavedec3_composes_single_level_bitexact_and_roundtrips():
    from cwdm_hip import ops
    x = torch.rand(2, 3, 16, 24, 32, generator=torch.Generator().manual_seed(2)).to(DEV)
    co = ops.wavedec3(x, 3)
    assert len(co) == 4 and co[0].shape == (2, 3, 2, 3, 4) and co[3]["HHH"].shape == (2, 3, 8, 12, 16)
    b1 = ops.dwt3d(x)
    b2 = ops.dwt3d(b1[0].contiguous())
    for i, k in enumerate(HIGH):
        assert torch.equal(co[3][k], b1[1 + i]) and torch.equal(co[2][k], b2[1 + i])
    rec = ops.waverec3(co)
    assert float((rec - x).abs().max()) < 1e-5
    with pytest.raises(AssertionError):
        ops.wavedec3(torch.rand(1, 1, 12, 8, 8, device=DEV), 3)
