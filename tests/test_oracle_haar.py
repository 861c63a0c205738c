"""Pin the oracle's Haar restatement: PyWavelets fixtures + analytic KATs."""
import math
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import haar

BANDS = haar.BAND_NAMES


def _golden():
    return np.load(os.path.join(GOLDEN, "pywt_haar3d.npz"), allow_pickle=False)


def test_pywt_taps_match_reference_filters():
    g = _golden()
    np.testing.assert_allclose(g["rec_lo"], haar.HAAR_LO, rtol=0, atol=0)
    np.testing.assert_allclose(g["rec_hi"], haar.HAAR_HI, rtol=0, atol=0)
    # IDWT_3D uses dec_* reversed (DWT_IDWT_layer.py:553-557): identical for Haar
    np.testing.assert_allclose(g["dec_lo"][::-1], haar.HAAR_LO, rtol=0, atol=0)
    np.testing.assert_allclose(g["dec_hi"][::-1], haar.HAAR_HI, rtol=0, atol=0)


@pytest.mark.parametrize("n", range(5))
@pytest.mark.parametrize("form", ["closed", "matrix"])
def test_dwt_matches_pywt(n, form):
    g = _golden()
    x = torch.from_numpy(g[f"x{n}"]).float()[None, None]
    D, H, W = x.shape[-3:]
    if form == "matrix" and D > max(H, W):
        pytest.skip("reference matrix form rejects depth > max(H, W)")
    fn = haar.dwt3d if form == "closed" else haar.dwt3d_matrix
    bands = fn(x)
    for name, b in zip(BANDS, bands):
        np.testing.assert_allclose(b[0, 0].double().numpy(), g[f"x{n}_{name}"], rtol=2e-6, atol=2e-6)


@pytest.mark.parametrize("n", range(5))
def test_idwt_matches_pywt(n):
    g = _golden()
    bands = [torch.from_numpy(g[f"x{n}_{b}"]).float()[None, None] for b in BANDS]
    rec = haar.idwt3d(*bands)
    np.testing.assert_allclose(rec[0, 0].double().numpy(), g[f"x{n}_rec"], rtol=2e-6, atol=2e-6)
    np.testing.assert_allclose(rec[0, 0].double().numpy(), g[f"x{n}"], rtol=2e-6, atol=2e-6)


def test_constant_volume():
    c = 0.37
    x = torch.full((1, 1, 4, 4, 4), c)
    b = haar.dwt3d(x)
    assert torch.allclose(b[0], torch.full_like(b[0], 2 * math.sqrt(2) * c), atol=1e-6)
    for k in range(1, 8):
        assert torch.count_nonzero(b[k]) == 0


def test_impulse_sign_pattern():
    # impulse at (1, 0, 1): band pqr sign = s_p(1) s_q(0) s_r(1), s_L = +, s_H = (+, -)
    x = torch.zeros(1, 1, 2, 2, 2)
    x[0, 0, 1, 0, 1] = 1.0
    b = haar.dwt3d(x)
    mag = 1 / (2 * math.sqrt(2))
    for k, name in enumerate(BANDS):
        sign = 1
        for letter, bit in zip(name, (1, 0, 1)):
            if letter == "H" and bit == 1:
                sign = -sign
        assert abs(float(b[k]) - sign * mag) < 1e-6, name


def test_perfect_reconstruction_parseval_adjoint():
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 6, 8, 10, generator=gen)
    b = haar.dwt3d(x)
    assert torch.allclose(haar.idwt3d(*b), x, atol=1e-5)
    assert abs(sum(float((t ** 2).sum()) for t in b) - float((x ** 2).sum())) < 1e-3
    y = [torch.randn(t.shape, generator=gen) for t in b]
    lhs = sum(float((bb * yy).sum()) for bb, yy in zip(b, y))
    rhs = float((x * haar.idwt3d(*y)).sum())
    assert abs(lhs - rhs) < 1e-3


def test_matrix_form_agrees_with_closed_form():
    x = torch.rand(1, 2, 8, 12, 10)
    for a, b in zip(haar.dwt3d_matrix(x), haar.dwt3d(x)):
        assert torch.allclose(a, b, atol=5e-7)
    bands = haar.dwt3d(x)
    assert torch.allclose(haar.idwt3d_matrix(*bands), haar.idwt3d(*bands), atol=5e-7)


def test_matrix_form_depth_quirk():
    # DWT_IDWT_layer.py:465 sizes the matrices by max(H, W): deeper volumes fail
    with pytest.raises(RuntimeError):
        haar.dwt3d_matrix(torch.rand(1, 1, 8, 4, 4))


def test_odd_sizes_rejected():
    with pytest.raises(AssertionError):
        haar.dwt3d(torch.rand(1, 1, 3, 4, 4))


def test_oracle_two_level_matches_pywt_wavedecn_golden():
    """The oracle's single-level restatement applied twice to the LLL band is
    pywt.wavedecn(level=2) (the multi-level DWT of BASELINE config 5)."""
    import os
    import numpy as np
    from conftest import GOLDEN
    from oracle import haar as oh
    g = np.load(os.path.join(GOLDEN, "pywt_haar3d_wavedec2.npz"), allow_pickle=False)
    for n in range(3):
        x = torch.from_numpy(g[f"x{n}"]).view(1, 1, *g[f"x{n}"].shape)
        b1 = oh.dwt3d(x)
        b2 = oh.dwt3d(b1[0])
        assert np.allclose(b2[0].numpy()[0, 0], g[f"x{n}_L2_LLL"], atol=1e-12)
        for i, b in enumerate(("LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")):
            assert np.allclose(b1[1 + i].numpy()[0, 0], g[f"x{n}_L1_{b}"], atol=1e-12)
            assert np.allclose(b2[1 + i].numpy()[0, 0], g[f"x{n}_L2_{b}"], atol=1e-12)
