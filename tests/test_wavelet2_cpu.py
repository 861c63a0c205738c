"""Config 5's two-level block representation, CPU side: the oracle
(oracle/wavelet2.py) pinned to PyWavelets' wavedecn(level=2) golden vectors
(tests/golden/pywt_haar3d_wavedec2.npz), and the per-subband FATS tables of
GaussianDiffusion(wavelet_levels=2) against the oracle's."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import diffusion as od, wavelet2 as w2

HIGH = ("LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")


@pytest.mark.parametrize("n", [0, 1, 2])
def test_oracle_analysis2_matches_pywt_wavedecn(n):
    """Channels 0..7 = level-2 bands of LLL1 / 3 (LLL2 again / 3), channels
    8.. = level-1 details folded 2x2x2 (phase 4 pz + 2 py + px)."""
    g = np.load(os.path.join(GOLDEN, "pywt_haar3d_wavedec2.npz"), allow_pickle=False)
    x = torch.from_numpy(g[f"x{n}"]).view(1, 1, *g[f"x{n}"].shape)
    c = w2.analysis2(x)[0].numpy()
    assert np.allclose(c[0], g[f"x{n}_L2_LLL"] / 9.0, atol=1e-12)
    for k, b in enumerate(HIGH):
        assert np.allclose(c[1 + k], g[f"x{n}_L2_{b}"] / 3.0, atol=1e-12)
        det = g[f"x{n}_L1_{b}"]
        for ph in range(8):
            pz, py, px = ph >> 2, (ph >> 1) & 1, ph & 1
            assert np.allclose(c[8 + 8 * k + ph], det[pz::2, py::2, px::2], atol=1e-12), (b, ph)
    assert np.allclose(w2.synthesis2(w2.analysis2(x))[0, 0].numpy(), g[f"x{n}_rec"], atol=1e-6)


def test_process_xstart2_is_a_projection():
    x = torch.rand(1, 1, 8, 8, 8, dtype=torch.float64)
    c = w2.analysis2(x)
    assert torch.allclose(w2.process_xstart2(c), c, atol=1e-12)       # already in [0, 1]
    c2 = w2.process_xstart2(c * 3.0)
    assert torch.allclose(w2.process_xstart2(c2), c2, atol=1e-12)
    img = w2.synthesis2(c2)
    assert img.min() >= -1e-12 and img.max() <= 1 + 1e-12


def test_band_of_channel():
    assert [w2.band_of_channel(j) for j in (0, 7, 8, 15, 16, 63)] == [0, 7, 8, 8, 9, 14]


def test_per_subband_tables_match_oracle():
    from guided_diffusion import script_util
    shift = np.linspace(-1.0, 1.5, 15)
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i", timestep_respacing="ddim50",
                                              band_log_snr_shift=shift, wavelet_levels=2)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), use_timesteps=od.space_timesteps(1000, "ddim50"),
                    band_shift=w2.channel_shift(shift))
    assert d.subband_channels == 64 and d.alphas_cumprod.shape == (50, 64)
    assert np.array_equal(d.alphas_cumprod, tab.alphas_cumprod)
    assert np.array_equal(d.posterior_mean_coef1, tab.posterior_mean_coef1)
    assert tuple(d.coef_table("cpu").shape) == (50, 64, 8)
    with pytest.raises(ValueError):
        script_util.create_gaussian_diffusion(steps=1000, mode="i2i", band_log_snr_shift=np.zeros(8), wavelet_levels=2)


@pytest.mark.parametrize("n", [0, 1])
def test_oracle_unscaled_analysis2_is_pywt_wavedecn(n):
    """The noise image's transform in the config-5 training front end
    (analysis2(scale=False): no LLL / 3, as the reference's noise DWT) is the
    plain orthonormal wavedecn(level=2) in the same channel layout, so unit
    Gaussian noise stays unit Gaussian."""
    g = np.load(os.path.join(GOLDEN, "pywt_haar3d_wavedec2.npz"), allow_pickle=False)
    x = torch.from_numpy(g[f"x{n}"]).view(1, 1, *g[f"x{n}"].shape)
    c = w2.analysis2(x, scale=False)[0].numpy()
    assert np.allclose(c[0], g[f"x{n}_L2_LLL"], atol=1e-12)
    for k, b in enumerate(HIGH):
        assert np.allclose(c[1 + k], g[f"x{n}_L2_{b}"], atol=1e-12)
    assert np.isclose(float((c.astype(np.float64) ** 2).sum()), float((g[f"x{n}"].astype(np.float64) ** 2).sum()),
                      rtol=1e-6)   # the oracle Haar runs in fp32 like the reference
