"""Torch-tensor wrappers over the libcwdm C ABI (device memory + current stream).

PyTorch is plumbing here: it owns device buffers and streams; every compute
step is a libcwdm kernel.  Inputs must live on a ROCm device -- there is no CPU
path (``_need_cuda`` raises).
"""
import ctypes
import math

import torch

from . import _lib
from ._lib import CWDM_BF16, CWDM_F16, CWDM_F32, CWDM_F64, check, lib, strides

DT = {torch.float32: CWDM_F32, torch.bfloat16: CWDM_BF16, torch.float16: CWDM_F16}


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("fast-cwdm_amd: HIP kernels need tensors on a ROCm device "
                               "(no CPU fallback in the product path)")


def check_device_status(where):
    """Raise if a kernel flagged a condition it could not return (cwdm_device_status,
    e.g. an apply-ahead counter wait that ran out: that conv's output is invalid).
    Synchronises the device: call once per sampling loop, not per step."""
    st = lib().cwdm_device_status(1)
    if st < 0:
        check(st, where)
    if st:
        raise RuntimeError(f"{where}: device error word {st:#x} (CWDM_DEV_E_AA_TIMEOUT = 1: a persistent conv's "
                           f"workgroups were not all resident; results of this call are invalid)")


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def dwt3d(x, lll_div3=False, out=None, out_strides=None, out_dtype=None):
    """Haar DWT of an NCDHW fp32 volume.  Returns (8, B, C, d, h, w) unless
    ``out``/``out_strides`` (band, b, c, voxel) are given."""
    _need_cuda(x)
    if x.dim() != 5:
        raise AssertionError("DWT_3D expects a 5-D (N, C, D, H, W) tensor")
    x = x.contiguous()
    if x.dtype != torch.float32:
        raise TypeError("DWT_3D: fp32 input expected (the reference's filter matrices are fp32)")
    B, C, D, H, W = x.shape
    if out is None:
        out = torch.empty((8, B, C, D // 2, H // 2, W // 2), device=x.device,
                          dtype=out_dtype or torch.float32)
        v = (D // 2) * (H // 2) * (W // 2)
        out_strides = (B * C * v, C * v, v, 1)
    check(lib().cwdm_haar_dwt3d(_p(x), B, C, D, H, W, _p(out), DT[out.dtype], strides(*out_strides),
                                1 if lll_div3 else 0, _stream()), "DWT_3D")
    return out


def idwt3d(bands, band_strides, B, C, d, h, w, lll_mul3=False, clamp01=False, out=None):
    """Haar IDWT.  ``bands`` is a tensor holding all 8 subbands addressed by
    ``band_strides`` (band, b, c, voxel); returns an NCDHW fp32 volume."""
    _need_cuda(bands)
    if out is None:
        out = torch.empty((B, C, 2 * d, 2 * h, 2 * w), device=bands.device, dtype=torch.float32)
    check(lib().cwdm_haar_idwt3d(_p(bands), DT[bands.dtype], strides(*band_strides), B, C, d, h, w, _p(out),
                                 1 if lll_mul3 else 0, 1 if clamp01 else 0, _stream()), "IDWT_3D")
    return out


def idwt3d_planes(bands, lll_mul3=False):
    """IDWT of 8 separate (B, C, d, h, w) band tensors (same dtype, same strides
    up to the base pointer) without stacking them."""
    _need_cuda(*bands)
    if len(bands) != 8:
        raise AssertionError("IDWT_3D takes the 8 subbands")
    b0 = bands[0]
    if lll_mul3:
        raise NotImplementedError("lll_mul3 on separate planes")
    bands = [b.contiguous() if b.dtype in DT else b.float().contiguous() for b in bands]
    dt = bands[0].dtype
    bands = [b if b.dtype == dt else b.to(dt) for b in bands]
    for b in bands:
        if b.shape != b0.shape:
            raise AssertionError("IDWT_3D: all subbands must have one shape")
    B, C, d, h, w = b0.shape
    out = torch.empty((B, C, 2 * d, 2 * h, 2 * w), device=b0.device, dtype=torch.float32)
    v = d * h * w
    arr = (ctypes.c_void_p * 8)(*[b.data_ptr() for b in bands])
    check(lib().cwdm_haar_idwt3d_planes(arr, DT[dt], strides(C * v, v, 1), B, C, d, h, w, _p(out), _stream()),
          "IDWT_3D")
    return out


def prepare_batch(target, c1, c2, c3, eps_img, coef, t, T, per_band=False):
    """training_losses front end in one kernel (cwdm_prepare_batch): returns
    (x_in (B, 32, d, h, w) = [q_sample | 3 condition DWTs], x0 (B, 8, d, h, w)).
    per_band: coef is [T][8][2] (FATS per-band schedules)."""
    vols = [v.contiguous().float() for v in (target, c1, c2, c3, eps_img)]
    _need_cuda(*vols, coef, t)
    for v in vols:
        if v.dim() != 5 or v.shape[1] != 1 or v.shape != vols[0].shape:
            raise AssertionError("prepare_batch: five (B, 1, D, H, W) volumes of one shape")
    B, _, D, H, W = vols[0].shape
    x_in = torch.empty((B, 32, D // 2, H // 2, W // 2), device=vols[0].device, dtype=torch.float32)
    x0 = torch.empty((B, 8, D // 2, H // 2, W // 2), device=vols[0].device, dtype=torch.float32)
    t = t.to(dtype=torch.int64).contiguous()
    check(lib().cwdm_prepare_batch(*[_p(v) for v in vols], B, D, H, W, _p(coef), 1 if per_band else 0, _p(t), T,
                                   _p(x_in), _p(x0), _stream()), "training_losses")
    return x_in, x0


def prepare_batch2(target, c1, c2, c3, eps_img, coef, t, T, per_band=False):
    """The 2-level (config 5) training front end in one kernel
    (cwdm_prepare_batch2): returns (x_in (B, 256, d, h, w) = [q_sample |
    3 condition analyses], x0 (B, 64, d, h, w)), d = D / 4.  per_band: coef
    is [T][64][2] (per-channel FATS rows)."""
    vols = [v.contiguous().float() for v in (target, c1, c2, c3, eps_img)]
    _need_cuda(*vols, coef, t)
    for v in vols:
        if v.dim() != 5 or v.shape[1] != 1 or v.shape != vols[0].shape:
            raise AssertionError("prepare_batch2: five (B, 1, D, H, W) volumes of one shape")
    B, _, D, H, W = vols[0].shape
    if D % 4 or H % 4 or W % 4:
        raise AssertionError(f"prepare_batch2: edges must be multiples of 4 (got {D}x{H}x{W})")
    x_in = torch.empty((B, 256, D // 4, H // 4, W // 4), device=vols[0].device, dtype=torch.float32)
    x0 = torch.empty((B, 64, D // 4, H // 4, W // 4), device=vols[0].device, dtype=torch.float32)
    t = t.to(dtype=torch.int64).contiguous()
    check(lib().cwdm_prepare_batch2(*[_p(v) for v in vols], B, D, H, W, _p(coef), 1 if per_band else 0, _p(t), T,
                                    _p(x_in), _p(x0), _stream()), "training_losses")
    return x_in, x0


def copy3(src, src_strides, dst, dst_strides, B, C, V):
    _need_cuda(src, dst)
    check(lib().cwdm_copy3(_p(src), DT[src.dtype], strides(*src_strides), _p(dst), DT[dst.dtype],
                           strides(*dst_strides), B, C, V, _stream()), "copy3")
    return dst


def ncdhw_strides(t):
    """(b, c, voxel) element strides of a contiguous NCDHW tensor."""
    B, C = t.shape[:2]
    v = t[0, 0].numel()
    return (C * v, v, 1)


def ndhwc_strides(B, C, V, c_total=None):
    ct = C if c_total is None else c_total
    return (V * ct, 1, ct)


def sampler_args(model_out, mo_s, x_t, xt_s, x_prev, xp_s, noise, nz_s, coef, t, T, B, d, h, w,
                 clip_denoised=True, pred_xstart=None, px_s=(0, 0, 0), mirror=None, mr_s=(0, 0, 0),
                 mean_type=0, update=0, per_band=False, levels=1, noise_seed=None):
    """The cwdm_sampler_args of one step.  noise_seed (with noise None): draw
    the noise in the kernel (Philox, keyed by the seed, counter = voxel,
    batch, device timestep, channel group)."""
    _need_cuda(model_out, x_t, x_prev, noise, coef, t, pred_xstart, mirror)
    a = _lib.SamplerArgs()
    a.model_out, a.mo_s = model_out.data_ptr(), _lib.I64x3(*mo_s)
    a.x_t, a.xt_s = x_t.data_ptr(), _lib.I64x3(*xt_s)
    a.x_prev, a.xp_s = x_prev.data_ptr(), _lib.I64x3(*xp_s)
    a.noise = noise.data_ptr() if noise is not None else None
    a.nz_s = _lib.I64x3(*nz_s)
    a.pred_xstart = pred_xstart.data_ptr() if pred_xstart is not None else None
    a.px_s = _lib.I64x3(*px_s)
    a.mirror = mirror.data_ptr() if mirror is not None else None
    a.mirror_dtype = DT[mirror.dtype] if mirror is not None else CWDM_F32
    a.mr_s = _lib.I64x3(*mr_s)
    a.coef, a.t = coef.data_ptr(), t.data_ptr()
    a.T, a.B, a.d, a.h, a.w = T, B, d, h, w
    a.clip_denoised = 1 if clip_denoised else 0
    a.mean_type = int(mean_type)
    a.update = int(update)
    a.per_band = 1 if per_band else 0
    a.levels = int(levels)
    a.noise_philox = 1 if (noise is None and noise_seed is not None) else 0
    a.noise_seed = int(noise_seed or 0) & ((1 << 64) - 1)
    return a


def sampler_step(model_out, mo_s, x_t, xt_s, x_prev, xp_s, noise, nz_s, coef, t, T, B, d, h, w,
                 clip_denoised=True, pred_xstart=None, px_s=(0, 0, 0), mirror=None, mr_s=(0, 0, 0),
                 mean_type=0, update=0, per_band=False, levels=1, noise_seed=None):
    """Fused process_xstart + posterior mean + noise (cwdm_sampler_step);
    update=1: the DDIM step instead of the posterior mean + noise; levels=2:
    the 64-channel two-level block representation (config 5, wavelet2_*);
    noise_seed: in-kernel Philox noise instead of a noise tensor."""
    a = sampler_args(model_out, mo_s, x_t, xt_s, x_prev, xp_s, noise, nz_s, coef, t, T, B, d, h, w,
                     clip_denoised, pred_xstart, px_s, mirror, mr_s, mean_type, update, per_band, levels,
                     noise_seed)
    check(lib().cwdm_sampler_step(ctypes.byref(a), _stream()), "sampler_step")


# ---- two-level block representation (config 5; specification oracle/wavelet2.py) ----
def wavelet2_analysis(x, out=None, c0=0, dtype=None):
    """(B, 1, D, H, W) fp32 image (edges multiples of 4) -> 64 coefficient
    channels per voxel of the (D/4, H/4, W/4) grid, channels-last.  ``out``:
    an existing channels-last (B, d, h, w, C) buffer (fp32 or bf16) written at
    channels [c0, c0 + 64), e.g. a slice of the U-Net input; else a new fp32
    (B, d, h, w, 64) tensor."""
    _need_cuda(x, out)
    if x.dim() != 5 or x.shape[1] != 1:
        raise AssertionError("wavelet2_analysis expects a (B, 1, D, H, W) image")
    B, _, D, H, W = x.shape
    if D % 4 or H % 4 or W % 4:
        raise AssertionError(f"wavelet2_analysis: edges must be multiples of 4 (got {D}x{H}x{W})")
    x = x.contiguous().float()
    d, h, w = D // 4, H // 4, W // 4
    if out is None:
        out = torch.empty((B, d, h, w, 64), dtype=dtype or torch.float32, device=x.device)
    if tuple(out.shape[:4]) != (B, d, h, w) or out.shape[4] < c0 + 64 or not out.is_contiguous():
        raise AssertionError("wavelet2_analysis: out must be a contiguous (B, d, h, w, >= c0 + 64) tensor")
    C = out.shape[4]
    check(lib().cwdm_wavelet2_analysis(x.data_ptr(), B, D, H, W, out.data_ptr(), DT[out.dtype], d * h * w * C, C,
                                       c0, _stream()), "wavelet2_analysis")
    return out


def wavelet2_synthesis(coef, c0=0):
    """Inverse of wavelet2_analysis: channels-last fp32 (B, d, h, w, C >= c0 + 64)
    -> (B, 1, 4d, 4h, 4w) fp32 image."""
    _need_cuda(coef)
    if coef.dim() != 5 or coef.shape[4] < c0 + 64 or coef.dtype != torch.float32 or not coef.is_contiguous():
        raise AssertionError("wavelet2_synthesis expects contiguous fp32 (B, d, h, w, >= c0 + 64) coefficients")
    B, d, h, w, C = coef.shape
    out = torch.empty((B, 1, 4 * d, 4 * h, 4 * w), dtype=torch.float32, device=coef.device)
    check(lib().cwdm_wavelet2_synthesis(coef.data_ptr(), B, d, h, w, d * h * w * C, C, c0, out.data_ptr(), _stream()),
          "wavelet2_synthesis")
    return out


# ---- multi-level Haar (BASELINE config 5) ---------------
HIGH_BANDS = ("LLH", "LHL", "LHH", "HLL", "HLH", "HHL", "HHH")


def wavedec3(x, level):
    """J-level 3D Haar analysis (pywt.wavedecn(x, 'haar', level=J) with the
    reference's single-level kernel applied to the LLL band J times): returns
    [LLL_J, {band: tensor} of level J, ..., of level 1], every tensor
    (B, C, D / 2^j, H / 2^j, W / 2^j) fp32, band letters in (D, H, W) order."""
    _need_cuda(x)
    if x.dim() != 5:
        raise AssertionError("wavedec3 expects a 5-D (N, C, D, H, W) tensor")
    if level < 1:
        raise ValueError("level must be >= 1")
    for s in x.shape[2:]:
        if s % (1 << level):
            raise AssertionError(f"every spatial size must be divisible by 2^level = {1 << level}")
    details = []
    cur = x.contiguous().float()
    for _ in range(level):
        b = dwt3d(cur)
        details.append({k: b[1 + i] for i, k in enumerate(HIGH_BANDS)})
        cur = b[0].contiguous()
    return [cur] + details[::-1]


def waverec3(coeffs):
    """Inverse of wavedec3 (pywt.waverecn)."""
    cur = coeffs[0]
    _need_cuda(cur)
    for d in coeffs[1:]:
        cur = idwt3d_planes([cur] + [d[k] for k in HIGH_BANDS])
    return cur


# ---- volume I/O either side of the path ----------------
_VOL_DT = {torch.float64: CWDM_F64, torch.float32: CWDM_F32}


def quantile_ranks(n, qs):
    """numpy 'linear' quantile bookkeeping (numpy/lib/_function_base_impl.py
    _quantile): virtual index (n - 1) q in float64, its floor and floor + 1
    (clamped to n - 1) as the two order statistics, gamma = index - floor."""
    ranks, gammas = [], []
    for q in qs:
        q = float(q)
        if not 0.0 <= q <= 1.0:
            raise ValueError("Quantiles must be in the range [0, 1]")
        vi = (n - 1) * q
        lo = min(int(math.floor(vi)), n - 1)
        ranks += [lo, min(lo + 1, n - 1)]
        gammas.append(vi - lo if vi < n - 1 else 0.0)
    return ranks, gammas


def quantiles(x, qs, out=None):
    """numpy.quantile(x, qs) (default 'linear') of a device fp64/fp32 tensor,
    as a float64 device tensor of len(qs) <= 2 values."""
    _need_cuda(x)
    if x.dtype not in _VOL_DT:
        raise TypeError("quantiles: float64 or float32 input")
    x = x.contiguous()
    qs = list(qs)
    if not 1 <= len(qs) <= 2:
        raise ValueError("quantiles: one or two quantiles per call")
    n = x.numel()
    if n == 0:
        raise IndexError("cannot compute quantiles of an empty array")
    ranks, gammas = quantile_ranks(n, qs)
    if out is None:
        out = torch.empty(len(qs), dtype=torch.float64, device=x.device)
    ws = torch.empty(int(lib().cwdm_quantile_workspace_bytes()), dtype=torch.uint8, device=x.device)
    rk = (ctypes.c_int64 * len(ranks))(*ranks)
    gm = (ctypes.c_double * len(gammas))(*gammas)
    check(lib().cwdm_quantiles(_p(x), _VOL_DT[x.dtype], n, rk, len(ranks), gm, _p(out), _p(ws), ws.numel(),
                               _stream()), "quantile")
    return out


def volume_prepare(x, lohi, crop=0, out_z=None, out_dtype=torch.float32):
    """(clip(x, lo, hi) - lo) / (hi - lo) in float64 over x[crop:-crop, crop:-crop, :],
    zero-padded in z to out_z, cast to out_dtype."""
    _need_cuda(x, lohi)
    if x.dim() != 3:
        raise AssertionError("volume_prepare expects an (X, Y, Z) volume")
    x = x.contiguous()
    X, Y, Z = x.shape
    out_z = Z if out_z is None else out_z
    out = torch.empty((X - 2 * crop, Y - 2 * crop, out_z), dtype=out_dtype, device=x.device)
    check(lib().cwdm_volume_prepare(_p(x), _VOL_DT[x.dtype], X, Y, Z, _p(lohi.contiguous()), crop, out_z, _p(out),
                                    _VOL_DT[out_dtype], _stream()), "volume_prepare")
    return out


def sample_finish(sample, mask=None, keep_z=None):
    """sample (B, 8, d, h, w) fp32 subbands -> (B, 2d, 2h, keep_z) image:
    IDWT(3 LLL, ...), clamp to [0, 1], zero where mask == 0, z cropped."""
    _need_cuda(sample, mask)
    if sample.dim() != 5 or sample.shape[1] != 8:
        raise AssertionError("sample_finish expects (B, 8, d, h, w) subbands")
    s = sample.contiguous().float()
    B, _, d, h, w = s.shape
    keep_z = 2 * w if keep_z is None else keep_z
    m = None
    if mask is not None:
        m = mask.contiguous().float()
        if m.numel() != B * 8 * d * h * w:
            raise AssertionError("mask must have the image shape (B, 1, 2d, 2h, 2w)")
    out = torch.empty((B, 2 * d, 2 * h, keep_z), dtype=torch.float32, device=s.device)
    check(lib().cwdm_sample_finish(_p(s), B, d, h, w, _p(m), keep_z, _p(out), _stream()), "sample_finish")
    return out
