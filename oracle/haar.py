"""Oracle: single-level 3D Haar analysis/synthesis (TEST INFRASTRUCTURE ONLY).

Two independent restatements of the reference's wavelet layer:

* ``dwt3d_matrix`` / ``idwt3d_matrix`` follow the reference literally: banded
  filter matrices built like ``DWT_3D.get_matrix`` (DWT_IDWT/DWT_IDWT_layer.py:459-518,
  IDWT_3D.get_matrix :563-622) and contracted with ``torch.matmul`` in the same
  stage order as ``DWTFunction_3D.forward`` (DWT_IDWT/DWT_IDWT_Functions.py:117-136)
  and ``IDWTFunction_3D.forward`` (:161-181).
* ``dwt3d`` / ``idwt3d`` are the closed (block-local) form of the same maps:
  band_pqr[i,j,k] = c^3 * sum_{a,b,e} s_p(a) s_q(b) s_r(e) x[2i+a, 2j+b, 2k+e]
  with c = 1/sqrt(2) rounded to fp32, s_L = +1, s_H = (+1, -1), and the band
  letters indexing the (D, H, W) axes.

pywt is absent from this interpreter, so the taps are the pywt Haar values
(rec_lo = [c, c], rec_hi = [c, -c]; dec_* reversed are the same), pinned by
``tests/golden/pywt_haar3d.npz``.
"""
import math

import numpy as np
import torch

BAND_NAMES = ("LLL", "LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")
# pywt.Wavelet('haar').rec_lo / rec_hi, literally (pinned by tests/golden/pywt_haar3d.npz)
HAAR_LO = [0.7071067811865476, 0.7071067811865476]
HAAR_HI = [0.7071067811865476, -0.7071067811865476]


def _band_matrices(n_max, n_axis, lo, hi):
    """Banded analysis matrices for one axis (DWT_IDWT_layer.py:465-503).

    Returns (low, high) of shape (n_axis//2, n_axis), row i holding the taps
    at columns 2i, 2i+1.  ``n_max`` mirrors the reference's L1 = max(H, W)
    sizing quirk (:465) which makes depth > max(H, W) a shape error.
    """
    if n_axis > n_max + len(lo) - 2 + 0:
        # reference slices matrix_h[:, 0:(n + band_length - 2)] of a matrix
        # sized by max(H, W); a deeper depth cannot be sliced out of it.
        raise RuntimeError(
            f"DWT_3D: depth {n_axis} exceeds max(H, W) = {n_max} (reference get_matrix sizing)")
    half = n_max // 2
    band = len(lo)
    mh = np.zeros((half, n_max + band - 2))
    mg = np.zeros((n_max - half, n_max + band - 2))
    for i in range(half):
        mh[i, 2 * i:2 * i + band] = lo
    for i in range(n_max - half):
        mg[i, 2 * i:2 * i + band] = hi
    low = mh[: n_axis // 2, : n_axis + band - 2]
    high = mg[: n_axis - n_axis // 2, : n_axis + band - 2]
    return low, high


def haar_matrices(d, h, w):
    """The six fp32 matrices the reference passes to DWTFunction_3D."""
    n_max = max(h, w)
    l0, h0 = _band_matrices(n_max, h, HAAR_LO, HAAR_HI)
    l1, h1 = _band_matrices(n_max, w, HAAR_LO, HAAR_HI)
    l2, h2 = _band_matrices(n_max, d, HAAR_LO, HAAR_HI)
    f = lambda a: torch.tensor(a, dtype=torch.float32)
    # W-axis matrices are stored transposed (DWT_IDWT_layer.py:497, :502)
    return f(l0), f(l1.T.copy()), f(l2), f(h0), f(h1.T.copy()), f(h2)


def dwt3d_matrix(x):
    """Matrix-form DWT (DWTFunction_3D.forward, DWT_IDWT_Functions.py:117-136)."""
    assert x.dim() == 5
    l0, l1, l2, h0, h1, h2 = haar_matrices(*x.shape[-3:])
    lo_h = torch.matmul(l0, x)            # contract H
    hi_h = torch.matmul(h0, x)
    out = []
    for first in (lo_h, hi_h):
        for wm in (l1, h1):
            hw = torch.matmul(first, wm).transpose(2, 3)   # contract W, D <-> H
            out.append(hw)
    ll, lh, hl, hh = out
    bands = []
    for dm in (l2, h2):
        for hw in (ll, lh, hl, hh):
            bands.append(torch.matmul(dm, hw).transpose(2, 3))  # contract D
    return tuple(bands)  # LLL, LLH, LHL, LHH, HLL, HLH, HHL, HHH


def idwt3d_matrix(*bands):
    """Matrix-form IDWT (IDWTFunction_3D.forward, DWT_IDWT_Functions.py:161-181)."""
    assert len(bands) == 8
    d = bands[0].shape[-3] + bands[7].shape[-3]
    h = bands[0].shape[-2] + bands[7].shape[-2]
    w = bands[0].shape[-1] + bands[7].shape[-1]
    l0, l1, l2, h0, h1, h2 = haar_matrices(d, h, w)
    lll, llh, lhl, lhh, hll, hlh, hhl, hhh = bands

    def dstage(lo_b, hi_b):  # undo the D contraction
        return (torch.matmul(l2.t(), lo_b.transpose(2, 3))
                + torch.matmul(h2.t(), hi_b.transpose(2, 3))).transpose(2, 3)

    ll = dstage(lll, hll)
    lh = dstage(llh, hlh)
    hl = dstage(lhl, hhl)
    hh = dstage(lhh, hhh)
    lo_h = torch.matmul(ll, l1.t()) + torch.matmul(lh, h1.t())
    hi_h = torch.matmul(hl, l1.t()) + torch.matmul(hh, h1.t())
    return torch.matmul(l0.t(), lo_h) + torch.matmul(h0.t(), hi_h)


_C32 = float(np.float32(HAAR_LO[0]))


def dwt3d(x):
    """Closed-form DWT: same stage order (H, then W, then D) as the matrices."""
    assert x.dim() == 5
    D, H, W = x.shape[-3:]
    if D % 2 or H % 2 or W % 2:
        raise AssertionError("Haar DWT_3D needs even D, H, W")
    c = torch.tensor(_C32, dtype=x.dtype)
    e_h, o_h = x[..., 0::2, :], x[..., 1::2, :]
    lo = c * e_h + c * o_h
    hi = c * e_h - c * o_h
    res = {}
    for a, t in (("L", lo), ("H", hi)):
        e_w, o_w = t[..., 0::2], t[..., 1::2]
        for b, u in (("L", c * e_w + c * o_w), ("H", c * e_w - c * o_w)):
            e_d, o_d = u[..., 0::2, :, :], u[..., 1::2, :, :]
            res["L" + a + b] = c * e_d + c * o_d
            res["H" + a + b] = c * e_d - c * o_d
    return tuple(res[n] for n in BAND_NAMES)


def idwt3d(*bands):
    """Closed-form IDWT: D, then W, then H (reverse of dwt3d)."""
    assert len(bands) == 8
    named = dict(zip(BAND_NAMES, bands))
    c = torch.tensor(_C32, dtype=bands[0].dtype)
    B, C, d, h, w = bands[0].shape

    def inter(even, odd, dim):
        shape = list(even.shape)
        shape[dim] *= 2
        out = torch.empty(shape, dtype=even.dtype)
        idx_e = [slice(None)] * len(shape)
        idx_o = [slice(None)] * len(shape)
        idx_e[dim] = slice(0, None, 2)
        idx_o[dim] = slice(1, None, 2)
        out[tuple(idx_e)] = even
        out[tuple(idx_o)] = odd
        return out

    stage_d = {}
    for hw in ("LL", "LH", "HL", "HH"):
        lo_b, hi_b = named["L" + hw], named["H" + hw]
        stage_d[hw] = inter(c * lo_b + c * hi_b, c * lo_b - c * hi_b, 2)
    stage_w = {}
    for a in ("L", "H"):
        lo_b, hi_b = stage_d[a + "L"], stage_d[a + "H"]
        stage_w[a] = inter(c * lo_b + c * hi_b, c * lo_b - c * hi_b, 4)
    lo_b, hi_b = stage_w["L"], stage_w["H"]
    return inter(c * lo_b + c * hi_b, c * lo_b - c * hi_b, 3)


def dwt_cat(x, lll_scale=1.0 / 3.0):
    """DWT of a 1-channel volume, concatenated as the reference does
    (``th.cat([LLL / 3., LLH, ...], dim=1)``, gaussian_diffusion.py:1131-1140)."""
    b = dwt3d(x)
    return torch.cat([b[0] / 3.0 if lll_scale == 1.0 / 3.0 else b[0] * lll_scale] + list(b[1:]), dim=1)


def idwt_split(xw):
    """IDWT of an 8-channel subband tensor with LLL x 3 (sample.py:113-121)."""
    B, _, D, H, W = xw.shape
    parts = [xw[:, i].view(B, 1, D, H, W) for i in range(8)]
    parts[0] = parts[0] * 3.0
    return idwt3d(*parts)
