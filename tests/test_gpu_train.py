"""Training path on the GPU: backward kernels against PyTorch-CPU fp32
autograd of the same op, and the whole native U-Net backward against autograd
through the oracle (fp32 within 1e-3 rel)."""
import ctypes
import math
import os

import pytest
import torch
import torch.nn.functional as F

from oracle import cases, unet as ou

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _nd(x):
    return x.permute(0, 2, 3, 4, 1).contiguous()


def _nc(x):
    return x.permute(0, 4, 1, 2, 3).contiguous()


def _dt(name):
    from cwdm_hip import _lib
    return {"fp32": (_lib.CWDM_F32, torch.float32), "bf16": (_lib.CWDM_BF16, torch.bfloat16),
            "fp16": (_lib.CWDM_F16, torch.float16)}[name]


# --------------------------------------------------------------------------- wgrad
WG_CASES = [
    # name, B, grid(conv), c0, c1, cout, umode, gn, ksize, dy_cs
    ("gn_64_64", 1, (8, 8, 16), 64, 0, 64, 0, True, 3, 64),
    ("concat_odd", 2, (4, 6, 20), 32, 32, 32, 0, True, 3, 32),
    ("up", 1, (8, 8, 16), 32, 0, 64, 1, True, 3, 64),
    ("plain_in32", 1, (8, 4, 16), 32, 0, 64, 0, False, 3, 64),
    ("head_cout8", 1, (8, 8, 8), 64, 0, 8, 0, True, 3, 16),
    # the output head's weight-gradient kernel (16-bit, W % 16, H % 4, D % 4; cout <= 8, cin 64):
    # two batches over several bricks, a cout below 8, no GroupNorm prologue
    ("head_hw_b2", 2, (8, 8, 32), 64, 0, 8, 0, True, 3, 16),
    ("head_hw_cout3", 1, (4, 12, 16), 64, 0, 3, 0, True, 3, 16),
    ("head_hw_nogn", 1, (8, 4, 16), 64, 0, 8, 0, False, 3, 16),
    # > 512 bricks (two per workgroup) with an odd count per batch entry: a workgroup's
    # range straddles the batch boundary (its GroupNorm coefficients reload mid-range)
    ("head_hw_straddle", 2, (100, 44, 16), 64, 0, 8, 0, True, 3, 16),
    ("skip1x1", 2, (4, 8, 16), 64, 32, 64, 0, False, 1, 64),
    ("tiny_grid", 1, (2, 2, 2), 64, 64, 128, 0, True, 3, 128),
    # 1x1 streaming kernel (wgrad1_kernel): R0-like concat 128 + 64 -> 64 over two
    # batches with a partial last 64-row stage, and a 512 -> 256 tile grid
    ("skip1x1_r0", 2, (6, 10, 34), 128, 64, 64, 0, False, 1, 64),
    ("skip1x1_wide", 1, (4, 8, 8), 256, 256, 256, 0, False, 1, 256),
    ("skip1x1_cout40", 1, (3, 5, 7), 48, 16, 40, 0, False, 1, 48),
]


@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", WG_CASES, ids=[c[0] for c in WG_CASES])
def test_conv3d_wgrad_vs_torch(case, dtype_name):
    _run_wgrad_case(case, dtype_name)


def _random_wgrad_cases(n, seed):
    """Seeded wgrad shapes: odd extents, concat inputs, upsampled inputs, 1x1 and 3x3, padded dy rows."""
    import random
    r = random.Random(seed)
    out = []
    for i in range(n):
        umode = r.choice([0, 0, 1])
        k = 3 if umode else r.choice([3, 3, 1])     # upsampled / GN prologues exist for 3x3 only
        ext = tuple(r.randint(1, 9) * (2 if umode else 1) for _ in range(2)) + (r.randint(2, 40) * (2 if umode else 1),)
        cout = r.choice([8, 16, 32, 64, 96, 128])
        dy_cs = (cout + 15) // 16 * 16 + r.choice([0, 16])
        c0 = 16 * r.randint(1, 6)
        c1 = r.choice([0, 32]) + (16 if c0 % 32 else 0)   # cin a multiple of 32
        out.append((f"rand{i}", r.randint(1, 2), ext, c0, c1, cout, umode, k == 3 and r.random() < 0.7, k, dy_cs))
    return out


RANDOM_WG_CASES = _random_wgrad_cases(12, 20261016)


@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", RANDOM_WG_CASES, ids=[c[0] for c in RANDOM_WG_CASES])
def test_conv3d_wgrad_random_shapes_vs_torch(case, dtype_name):
    _run_wgrad_case(case, dtype_name)


CM_CASES = [c for c in WG_CASES + RANDOM_WG_CASES if c[8] == 3] + [
    # grids with interior bricks (halo inside the volume: the DMA kernel's
    # precomputed-offset issue), two batches (brick counters cross a batch),
    # the upsampling source, a ragged x edge and dY rows with spare channels
    ("cm_interior", 2, (12, 12, 48), 64, 0, 64, 0, False, 3, 64),
    ("cm_interior_up", 1, (16, 16, 48), 32, 0, 64, 1, False, 3, 64),
    ("cm_interior_ragged", 1, (12, 16, 40), 32, 0, 32, 0, True, 3, 48),
    ("cm_interior_cs_short", 2, (12, 12, 48), 32, 0, 40, 0, False, 3, 48),
    # cin <= cout: the warp-specialised form (32-output tiles, DMA waves); cin > cout: the
    # 64-output tiles with the DMA issued by the MFMA waves (r05)
    ("cm_ws_square", 1, (12, 12, 48), 64, 0, 64, 0, False, 3, 64),
    ("cm_ws_up_wide", 1, (16, 16, 32), 64, 0, 128, 1, False, 3, 128),
    ("cm_mc2_cin_gt_cout", 1, (12, 12, 48), 128, 0, 64, 0, False, 3, 64),
]


@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("case", CM_CASES, ids=[c[0] for c in CM_CASES])
def test_conv3d_wgrad_kept_activation_vs_torch(case, dtype_name):
    """u_cm: U handed over as the forward kept it (activated, chunk-major
    [B][cin/16][SV][16]) and staged by LDS-DMA -- the exact staged input, so
    only the fp32 summation order differs from torch (1e-4)."""
    _run_wgrad_case(case, dtype_name, cm=True)


def _run_wgrad_case(case, dtype_name, cm=False):
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    name, B, grid, c0, c1, cout, umode, use_gn, k, dy_cs = case
    dtype, tdt = _dt(dtype_name)
    if dtype_name == "fp32" and dy_cs == 16:
        dy_cs = 8
    g = torch.Generator().manual_seed(3)
    D, H, W = grid
    sD, sH, sW = (D // 2, H // 2, W // 2) if umode == 1 else (D, H, W)
    cin = c0 + c1
    x = torch.randn(B, cin, sD, sH, sW, generator=g).to(tdt).float()
    dy = torch.randn(B, cout, D, H, W, generator=g).to(tdt).float()
    gn = None
    h = x
    if use_gn:
        scale = 1 + 0.2 * torch.randn(B, cin, generator=g)
        shift = 0.2 * torch.randn(B, cin, generator=g)
        gn = torch.stack([scale, shift], -1).contiguous()
        h = F.silu(x * scale[:, :, None, None, None] + shift[:, :, None, None, None])
    if dtype_name != "fp32":
        h = h.to(tdt).float()   # staged in bf16 / fp16 like the forward
    h_src = h
    if umode == 1:
        h = F.interpolate(h, scale_factor=2, mode="nearest")
    ref = torch.nn.grad.conv3d_weight(h, (cout, cin, k, k, k), dy, padding=(k // 2))
    xd = _nd(x).to(DEV, tdt)
    x0 = xd[..., :c0].contiguous()
    x1 = xd[..., c0:].contiguous() if c1 else None
    dyd = torch.zeros(B, D, H, W, dy_cs, device=DEV, dtype=tdt)
    dyd[..., :cout] = _nd(dy).to(DEV, tdt)
    dw = torch.zeros(cout, cin, k, k, k, device=DEV)
    d = _lib.WgradDesc()
    d.dtype, d.B, d.D, d.H, d.W, d.ksize = dtype, B, D, H, W, k
    d.u0, d.u_c0 = x0.data_ptr(), c0
    d.u1, d.u_c1 = (x1.data_ptr(), c1) if c1 else (None, 0)
    d.u_mode = umode
    gnd = gn.to(DEV) if gn is not None else None
    d.u_gn = gnd.data_ptr() if gnd is not None else None
    d.dy, d.dy_cs, d.cout = dyd.data_ptr(), dy_cs, cout
    dw0 = torch.randn(cout, cin, k, k, k, generator=g).to(DEV)
    dw.copy_(dw0)   # accumulated into: dw += dW
    d.dw = dw.data_ptr()
    if cm:
        sv = sD * sH * sW
        act = _nd(h_src).reshape(B, sv, cin // 16, 16).permute(0, 2, 1, 3).contiguous().to(DEV, tdt)
        d.u0, d.u_c0, d.u1, d.u_c1, d.u_gn, d.u_cm = act.data_ptr(), cin, None, 0, None, 1
    wsw = torch.empty(lib().cwdm_conv3d_wgrad_workspace_bytes(cout, cin, k), dtype=torch.uint8, device=DEV)
    d.workspace, d.ws_bytes = wsw.data_ptr(), wsw.numel()
    check(lib().cwdm_conv3d_wgrad(ctypes.byref(d), None))
    tol = 1e-4 if (dtype_name == "fp32" or cm) else 1e-2
    assert rel_err(dw - dw0, ref) < tol, name
    # partial tiles meet in per-range slabs added in range order: a second call
    # (workspace left dirty by the first) is bitwise identical
    dw2 = dw0.clone()
    d.dw = dw2.data_ptr()
    check(lib().cwdm_conv3d_wgrad(ctypes.byref(d), None))
    assert torch.equal(dw, dw2), name


# --------------------------------------------------------------------------- dgrad
@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("cfg", [(64, 64, (8, 8, 16)), (192, 64, (4, 8, 8)), (64, 8, (8, 8, 8)), (128, 256, (2, 2, 2))])
def test_conv3d_dgrad_packing_vs_torch(cfg, dtype_name):
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    cin, cout, grid = cfg
    dtype, tdt = _dt(dtype_name)
    ck = 8 if dtype_name == "fp32" else 16
    cpad = (cout + ck - 1) // ck * ck
    g = torch.Generator().manual_seed(4)
    B = 1
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)).to(tdt).float()
    dy = torch.randn(B, cout, *grid, generator=g).to(tdt).float()
    ref = torch.nn.grad.conv3d_input((B, cin, *grid), w, dy, padding=1)
    L = lib()
    pk = torch.empty(L.cwdm_conv3d_packed_bytes(cin, cpad, 3, dtype), dtype=torch.uint8, device=DEV)
    wd = w.to(DEV).contiguous()
    check(L.cwdm_conv3d_pack_dgrad(ctypes.c_void_p(wd.data_ptr()), cout, cin, 3, dtype,
                                   ctypes.c_void_p(pk.data_ptr()), None))
    a = torch.zeros(B, *grid, cpad, device=DEV, dtype=tdt)
    a[..., :cout] = _nd(dy).to(DEV, tdt)
    out = torch.empty(B, *grid, cin, device=DEV, dtype=tdt)
    d = _lib.ConvDesc()
    d.dtype, d.B, (d.D, d.H, d.W), d.cout = dtype, B, grid, cin
    d.a0, d.a_c0, d.a_w = a.data_ptr(), cpad, pk.data_ptr()
    d.res_mode = -1
    d.out, d.out_dtype = out.data_ptr(), dtype
    nws = L.cwdm_conv3d_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=DEV)
    d.workspace, d.ws_bytes = ws.data_ptr(), nws
    check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    tol = 2e-5 if dtype_name == "fp32" else 2e-2
    assert rel_err(_nc(out.float().cpu()), ref) < tol


@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("shape", [(1, (4, 8, 16), 32, 40, 56), (2, (4, 4, 40), 64, 24, 48),
                                   (1, (4, 4, 64), 128, 128, 64), (1, (3, 5, 7), 16, 8, 24),
                                   (2, (3, 4, 22), 64, 128, 64), (1, (2, 3, 40), 64, 64, 64),
                                   (1, (2, 4, 12), 32, 20, 28)])
@pytest.mark.parametrize("acc", [1, 0])
def test_conv3d_b_only_dual_output_accumulate(shape, dtype_name, acc):
    """1x1 skip dgrad: B-only conv writing channel slices to two buffers,
    accumulating (16-bit: the pointwise MFMA kernel, pointwise.hip; partial
    channel and voxel blocks, batch 2, odd grids)."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    dtype, tdt = _dt(dtype_name)
    g = torch.Generator().manual_seed(8)
    B, grid, cout, c0, c1 = shape
    if dtype_name == "fp32" and (c0 + c1) % 32 and c0 + c1 > 32:
        pytest.skip("fp32 brick kernels: output channels a multiple of 32 or below 32")
    cin = c0 + c1
    w = (torch.randn(cout, cin, 1, 1, 1, generator=g) / math.sqrt(cin)).to(tdt).float()
    dy = torch.randn(B, cout, *grid, generator=g).to(tdt).float()
    ref = torch.nn.grad.conv3d_input((B, cin, *grid), w, dy)
    L = lib()
    pk = torch.empty(L.cwdm_conv3d_packed_bytes(cin, cout, 1, dtype), dtype=torch.uint8, device=DEV)
    wd = w.to(DEV).contiguous()
    check(L.cwdm_conv3d_pack_dgrad(ctypes.c_void_p(wd.data_ptr()), cout, cin, 1, dtype,
                                   ctypes.c_void_p(pk.data_ptr()), None))
    base0 = torch.randn(B, *grid, c0, generator=g).to(tdt)
    base1 = torch.randn(B, *grid, c1, generator=g).to(tdt)
    o0, o1 = base0.to(DEV).clone(), base1.to(DEV).clone()
    a = _nd(dy).to(DEV, tdt)
    d = _lib.ConvDesc()
    d.dtype, d.B, (d.D, d.H, d.W), d.cout = dtype, B, grid, cin
    d.b0, d.b_c0, d.b_w = a.data_ptr(), cout, pk.data_ptr()
    d.res_mode = -1
    d.out, d.out_dtype, d.out1, d.out_c0, d.accumulate = o0.data_ptr(), dtype, o1.data_ptr(), c0, acc
    nws = L.cwdm_conv3d_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=DEV)
    d.workspace, d.ws_bytes = ws.data_ptr(), nws
    check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    got = torch.cat([o0.float().cpu() - acc * base0.float(), o1.float().cpu() - acc * base1.float()], -1)
    tol = 2e-5 if dtype_name == "fp32" else 3e-2
    assert rel_err(_nc(got), ref) < tol


@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
def test_conv3d_pointwise_two_sources_bias_vs_torch(dtype_name):
    """A pure 1x1 conv of a concatenated input (two channels-last sources) with
    a per-batch bias, the forward skip product's shape: pointwise kernel vs F.conv3d."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    dtype, tdt = _dt(dtype_name)
    g = torch.Generator().manual_seed(9)
    B, grid, k0, k1, cout = 2, (4, 6, 36), 48, 16, 96
    x = torch.randn(B, k0 + k1, *grid, generator=g).to(tdt).float()
    w = (torch.randn(cout, k0 + k1, 1, 1, 1, generator=g) / 8).to(tdt).float()
    bias = torch.randn(B, cout, generator=g)
    ref = F.conv3d(x, w) + bias[:, :, None, None, None]
    L = lib()
    pk = torch.empty(L.cwdm_conv3d_packed_bytes(cout, k0 + k1, 1, dtype), dtype=torch.uint8, device=DEV)
    wd = w.to(DEV).contiguous()
    check(L.cwdm_conv3d_pack(ctypes.c_void_p(wd.data_ptr()), cout, k0 + k1, 1, dtype,
                             ctypes.c_void_p(pk.data_ptr()), None))
    xd = _nd(x).to(DEV, tdt)
    x0, x1 = xd[..., :k0].contiguous(), xd[..., k0:].contiguous()
    bd = bias.to(DEV).contiguous()
    out = torch.empty(B, *grid, cout, device=DEV, dtype=tdt)
    d = _lib.ConvDesc()
    d.dtype, d.B, (d.D, d.H, d.W), d.cout = dtype, B, grid, cout
    d.b0, d.b_c0, d.b1, d.b_c1, d.b_w = x0.data_ptr(), k0, x1.data_ptr(), k1, pk.data_ptr()
    d.bias, d.bias_bstride = bd.data_ptr(), cout
    d.res_mode = -1
    d.out, d.out_dtype = out.data_ptr(), dtype
    check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    assert rel_err(_nc(out.float().cpu()), ref) < {"bf16": 2e-2, "fp16": 3e-3}[dtype_name]


# --------------------------------------------------------------------------- GN/SiLU backward
@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("chans", [(64, 0), (32, 32)])
def test_gn_silu_bwd_vs_autograd(chans, mode, dtype_name):
    _gn_silu_bwd_case(chans, mode, dtype_name, (4, 8, 6), 2, 8)


# grids with 384-1024 reduce blocks (the wide levels' finalize loads), 8 and 32 groups,
# a concat and a pooled source; two seeds per case
@pytest.mark.parametrize("chans,mode,dtype_name,grid,B,G", [
    ((64, 0), 0, "fp32", (32, 32, 48), 2, 8), ((64, 64), 0, "bf16", (32, 32, 32), 1, 32),
    ((128, 0), 2, "fp32", (32, 64, 64), 1, 32), ((64, 0), 0, "bf16", (64, 64, 32), 1, 32)])
def test_gn_silu_bwd_two_level_finalize_vs_autograd(chans, mode, dtype_name, grid, B, G):
    _gn_silu_bwd_case(chans, mode, dtype_name, grid, B, G)
    _gn_silu_bwd_case(chans, mode, dtype_name, grid, B, G, seed=10)


def _gn_silu_bwd_case(chans, mode, dtype_name, grid, B, G, seed=9):
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    dtype, tdt = _dt(dtype_name)
    c0, c1 = chans
    C = c0 + c1
    g = torch.Generator().manual_seed(seed)
    x = (1.5 * torch.randn(B, C, *grid, generator=g) + 0.3).to(tdt).float()
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    ugrid = {0: grid, 1: tuple(2 * s for s in grid), 2: tuple(s // 2 for s in grid)}[mode]
    du = torch.randn(B, C, *ugrid, generator=g).to(tdt).float()
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    y = F.silu(F.group_norm(xr, G, gr, br, eps=1e-5))
    if mode == 1:
        y = F.interpolate(y, scale_factor=2, mode="nearest")
    elif mode == 2:
        y = F.avg_pool3d(y, 2)
    (y * du).sum().backward()
    # forward statistics as cwdm_gn_finalize produces them
    xg = x.view(B, G, -1).double()
    mean = xg.mean(-1)
    rstd = 1.0 / torch.sqrt(xg.var(-1, unbiased=False) + 1e-5)
    mr = torch.stack([mean, rstd], -1).float().contiguous()
    cpg = C // G
    sc = gamma[None] * rstd.float().repeat_interleave(cpg, 1)
    sh = beta[None] - mean.float().repeat_interleave(cpg, 1) * sc
    ss = torch.stack([sc, sh], -1).contiguous()
    xd = _nd(x).to(DEV, tdt)
    x0 = xd[..., :c0].contiguous()
    x1 = xd[..., c0:].contiguous() if c1 else None
    dud = _nd(du).to(DEV, tdt)
    base0 = (0.01 * torch.randn(B, *grid, c0, generator=g)).to(tdt)
    dx0 = base0.to(DEV).clone()             # acc0 = 1
    dx1 = torch.empty(B, *grid, c1, device=DEV, dtype=tdt) if c1 else None   # acc1 = 0
    dgam = torch.empty(C, device=DEV)
    dbet = torch.empty(C, device=DEV)
    L = lib()
    nws = L.cwdm_gn_silu_bwd_workspace_bytes(C, B, *grid)
    ws = torch.empty(nws, dtype=torch.uint8, device=DEV)
    ssd, mrd, gd = ss.to(DEV), mr.to(DEV), gamma.to(DEV)
    check(L.cwdm_gn_silu_bwd(x0.data_ptr(), c0, x1.data_ptr() if c1 else None, c1, dud.data_ptr(), mode,
                             ssd.data_ptr(), mrd.data_ptr(), gd.data_ptr(), G, B, *grid, dtype,
                             dx0.data_ptr(), 1, dx1.data_ptr() if c1 else None, 0, dgam.data_ptr(), dbet.data_ptr(),
                             ws.data_ptr(), nws, None))
    got = dx0.float().cpu() - base0.float()
    if c1:
        got = torch.cat([got, dx1.float().cpu()], -1)
    tol = 1e-4 if dtype_name == "fp32" else 3e-2
    assert rel_err(_nc(got), xr.grad) < tol
    assert rel_err(dgam, gr.grad) < tol
    assert rel_err(dbet, br.grad) < tol


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_resample_add_and_channel_sum(mode):
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    L = lib()
    g = torch.Generator().manual_seed(10)
    B, C, grid = 2, 16, (4, 6, 8)
    sgrid = {0: grid, 1: tuple(2 * s for s in grid), 2: tuple(s // 2 for s in grid)}[mode]
    src = torch.randn(B, C, *sgrid, generator=g)
    dst0 = torch.randn(B, C, *grid, generator=g)
    xr = torch.zeros(B, C, *grid, requires_grad=True)
    y = {0: xr, 1: F.interpolate(xr, scale_factor=2, mode="nearest") if mode == 1 else None,
         2: F.avg_pool3d(xr, 2) if mode == 2 else None}[mode]
    (y * src).sum().backward()
    d = _nd(dst0).to(DEV)
    s = _nd(src).to(DEV)
    check(L.cwdm_resample_add(d.data_ptr(), s.data_ptr(), C, B, *grid, mode, 1, _lib.CWDM_F32, None))
    assert rel_err(_nc(d.cpu()) - dst0, xr.grad) < 1e-6
    V = s[0, ..., 0].numel()
    ref_bc = src.sum(dim=(2, 3, 4))[:, :12]
    # the workspace is required (no atomic fallback)
    out_bc = torch.zeros(B, 24, device=DEV)
    out_c = torch.zeros(C, device=DEV)
    rc = L.cwdm_channel_sum(s.data_ptr(), _lib.CWDM_F32, B, V, 12, C, out_bc.data_ptr(), 24, out_c.data_ptr(),
                            None, None, 0, None)
    assert rc == _lib.E_WORKSPACE
    runs = []
    for _ in range(2):
        ws = torch.empty(L.cwdm_channel_sum_workspace_bytes(B, V, 12), dtype=torch.uint8, device=DEV)
        out_bc = torch.zeros(B, 24, device=DEV)
        out_c = torch.zeros(C, device=DEV)
        check(L.cwdm_channel_sum(s.data_ptr(), _lib.CWDM_F32, B, V, 12, C, out_bc.data_ptr(), 24, out_c.data_ptr(),
                                 None, ws.data_ptr(), ws.numel(), None))
        assert rel_err(out_bc[:, :12], ref_bc) < 1e-5
        assert rel_err(out_c[:12], ref_bc.sum(0)) < 1e-5
        runs.append((out_bc.clone(), out_c.clone()))
    # the per-workgroup sums finish in a fixed order: bitwise repeatable
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


def test_adamw_matches_torch():
    from cwdm_hip._lib import check, lib
    g = torch.Generator().manual_seed(11)
    n = 10007
    p0 = torch.randn(n, generator=g)
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pr], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, foreach=False)
    p = p0.to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g)
        pr.grad = grad.clone()
        opt.step()
        gd = grad.to(DEV)
        check(lib().cwdm_adamw(p.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8,
                               0.01, step, None))
    assert rel_err(p, pr.detach()) < 1e-6
    st = opt.state[pr]
    assert rel_err(m, st["exp_avg"]) < 1e-6
    assert rel_err(v, st["exp_avg_sq"]) < 1e-6


def test_adamw_maxabs_matches_separate_reductions():
    """cwdm_adamw_maxabs: the same update bit for bit as cwdm_adamw, plus max |p| before
    the update and max |g| exactly (the reference's norm/param_max, norm/grad_max,
    train_util.py:370-375); a NaN gradient propagates to the max."""
    from cwdm_hip._lib import check, lib
    g = torch.Generator().manual_seed(12)
    n = 300007
    p0 = torch.randn(n, generator=g).to(DEV) * 3
    gd = torch.randn(n, generator=g).to(DEV)
    outs = []
    for fused in (False, True):
        p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        mx = torch.full((2,), -1.0, device=DEV)
        if fused:
            check(lib().cwdm_adamw_maxabs(p.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9,
                                          0.999, 1e-8, 0.01, 1, mx.data_ptr(), None))
            assert float(mx[0]) == float(p0.abs().max()) and float(mx[1]) == float(gd.abs().max())
        else:
            check(lib().cwdm_adamw(p.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999,
                                   1e-8, 0.01, 1, None))
        outs.append((p, m, v))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    gd[n // 2] = float("nan")
    p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    mx = torch.zeros(2, device=DEV)
    check(lib().cwdm_adamw_maxabs(p.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999,
                                  1e-8, 0.01, 1, mx.data_ptr(), None))
    assert torch.isnan(mx[1]) and float(mx[0]) == float(p0.abs().max())


# --------------------------------------------------------------------------- whole U-Net backward
def _product_model(cfg, groups, params, dtype):
    from guided_diffusion.unet import UNetModel
    m = UNetModel(image_size=32, in_channels=cfg["in_channels"], model_channels=cfg["model_channels"],
                  out_channels=cfg["out_channels"], num_res_blocks=cfg["num_res_blocks"], attention_resolutions=(),
                  channel_mult=cfg["channel_mult"], dims=3, resblock_updown=True, bottleneck_attention=False,
                  resample_2d=False, num_groups=groups, compute_dtype=dtype)
    m.load_state_dict(params)
    return m.to(DEV)


def _unet_grads(cfg, G, P, x, t, R, dtype, keep=True):
    model = _product_model(cfg, G, P, dtype)
    model.keep_activations = keep
    out = model(x.to(DEV), t.to(DEV))
    (out * R.to(DEV)).sum().backward()
    return out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in model.named_parameters()}, model


def _oracle_grads(cfg, G, P, x, t, R):
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    out = ou.unet_forward(Pr, x, t, num_groups=G, **cfg)
    (out * R).sum().backward()
    return out.detach(), {k: v.grad for k, v in Pr.items()}


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-3), ("bf16", 8e-2), ("fp16", 1.5e-2)])
def test_unet_backward_vs_oracle_autograd(dtype, tol):
    cfg, G = cases.C1_CFG, cases.C1_GROUPS
    P = ou.random_params(seed=21, **cfg)
    g = torch.Generator().manual_seed(22)
    x = torch.randn(2, 32, 16, 16, 16, generator=g)
    t = torch.tensor([5, 700])
    R = torch.randn(2, 8, 16, 16, 16, generator=g)
    out, grads, model = _unet_grads(cfg, G, P, x, t, R, dtype)
    ref_out, ref = _oracle_grads(cfg, G, P, x, t, R)
    assert rel_err(out, ref_out) < tol
    assert set(grads) == set(ref)
    worst = {}
    for k in ref:
        a, b = grads[k].double(), ref[k].double()
        worst[k] = float((a - b).norm() / b.norm().clamp_min(1e-30))
    bad = {k: v for k, v in worst.items() if v > tol}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:8]
    # the flat gradient the native backward wrote is what the optimizer sees
    flat = model.flat_grad()
    assert flat.numel() == sum(p.numel() for p in model.parameters())


def test_unet_backward_segments_and_hook():
    """Segment-wise backward with a per-segment hook (DDP bucket seam) gives the
    same gradients and covers the flat buffer exactly once."""
    cfg, G = cases.C1_CFG, cases.C1_GROUPS
    P = ou.random_params(seed=23, **cfg)
    g = torch.Generator().manual_seed(24)
    x = torch.randn(1, 32, 16, 16, 16, generator=g)
    t = torch.tensor([42])
    R = torch.randn(1, 8, 16, 16, 16, generator=g)
    _, g_all, _ = _unet_grads(cfg, G, P, x, t, R, "fp32")
    model = _product_model(cfg, G, P, "fp32")
    seen = []

    def hook(seg, flat, off, n):
        if seg is not None:
            seen.append((seg, off, n))
    model._grad_hook = hook
    out = model(x.to(DEV), t.to(DEV))
    (out * R.to(DEV)).sum().backward()
    n = sum(p.numel() for p in model.parameters())
    assert sum(s[2] for s in seen) == n
    assert [s[0] for s in seen] == list(range(model.plan.num_segments))
    for name, p in model.named_parameters():
        assert rel_err(p.grad, g_all[name]) < 1e-5, name


def test_autograd_grad_returns_gradients():
    """torch.autograd.grad over the native backward returns the gradients and
    leaves .grad alone (direct .grad hand-over is TrainLoop / FlatAdamW's)."""
    cfg, G = cases.C1_CFG, cases.C1_GROUPS
    P = ou.random_params(seed=25, **cfg)
    g = torch.Generator().manual_seed(26)
    x = torch.randn(1, 32, 16, 16, 16, generator=g)
    t = torch.tensor([17])
    R = torch.randn(1, 8, 16, 16, 16, generator=g)
    _, g_all, _ = _unet_grads(cfg, G, P, x, t, R, "fp32")
    model = _product_model(cfg, G, P, "fp32")
    names, params = zip(*model.named_parameters())
    out = model(x.to(DEV), t.to(DEV))
    grads = torch.autograd.grad((out * R.to(DEV)).sum(), params)
    assert all(p.grad is None for p in params)
    for n, gr in zip(names, grads):
        assert gr is not None and rel_err(gr, g_all[n]) < 1e-5, n


def test_train_switch_dtype_then_train_again():
    """Packed buffers are per dtype: bf16 training, then fp32 training on the
    same model re-packs into buffers of the fp32 size (no out-of-bounds pack)."""
    from cwdm_hip.optim import FlatAdamW
    cfg, G = cases.C1_CFG, cases.C1_GROUPS
    P = ou.random_params(seed=27, **cfg)
    g = torch.Generator().manual_seed(28)
    x = torch.randn(1, 32, 16, 16, 16, generator=g).to(DEV)
    t = torch.tensor([9]).to(DEV)
    R = torch.randn(1, 8, 16, 16, 16, generator=g).to(DEV)
    model = _product_model(cfg, G, P, "bf16")
    opt = FlatAdamW(model, lr=1e-4, weight_decay=0.0)
    for dt in ("bf16", "fp32"):
        model.set_compute_dtype(dt)
        opt.zero_grad()
        (model(x, t) * R).sum().backward()
        opt.step()
        assert model._packed.numel() >= model.plan.packed_bytes
        assert model._packed_bwd.numel() >= model.plan.packed_bwd_bytes
    # the fp32 gradients after the switch match a fresh fp32 model at the same weights
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    opt.zero_grad()
    (model(x, t) * R).sum().backward()
    _, ref, _ = _unet_grads(cfg, G, sd, x.cpu(), t.cpu(), R.cpu(), "fp32")
    for n, p in model.named_parameters():
        assert rel_err(p.grad, ref[n]) < 1e-5, n


def _c1_model_and_diffusion(P, dtype="fp32"):
    from guided_diffusion import script_util
    args = script_util.run_sh_model_args(num_channels=32, channel_mult="1,2", num_res_blocks=1, num_groups=8)
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: args[k] for k in keys})
    model.set_compute_dtype(dtype)
    model.load_state_dict(P)
    return model.to(DEV), diffusion


def test_training_step_vs_oracle():
    """training_losses -> loss.backward() -> FlatAdamW.step() (TrainLoop.forward_backward
    + run_step) against the oracle's loss/autograd and torch.optim.AdamW."""
    from cwdm_hip.optim import FlatAdamW
    from oracle import diffusion as od
    vols = {k: v.to(DEV) for k, v in cases.data.brats_batch(32, seed=4, batch=2).items()}
    P = ou.random_params(seed=31, **cases.C1_CFG)
    model, diffusion = _c1_model_and_diffusion(P)
    t = torch.tensor([5, 700], device=DEV)
    noise = torch.randn(2, 1, 32, 32, 32, device=DEV)
    terms, out, _ = diffusion.training_losses(model, vols, t, mode="i2i", contr="t2w", noise=noise)
    loss = terms["mse_wav"].mean()
    loss.backward()
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"))
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}

    def om(x, tt, **kw):
        return ou.unet_forward(Pr, x, tt, num_groups=8, **cases.C1_CFG)
    rterms, rout, _ = od.training_losses(tab, om, {k: v.cpu() for k, v in vols.items()}, t.cpu(), noise.cpu(),
                                         contr="t2w")
    rloss = rterms["mse_wav"].mean()
    rloss.backward()
    assert abs(float(loss) - float(rloss)) / float(rloss) < 1e-4
    for n, p in model.named_parameters():
        err = float((p.grad.double().cpu() - Pr[n].grad.double()).norm() / Pr[n].grad.double().norm().clamp_min(1e-30))
        assert err < 1e-3, (n, err)
    # optimizer: one fused launch == torch.optim.AdamW on the same gradients
    p0 = model.flat_params.detach().clone()
    g = model.flat_grad().detach().clone()
    opt = FlatAdamW(model, lr=1e-3, weight_decay=0.01)
    opt.step()
    ref = p0.cpu().clone().requires_grad_(True)
    topt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=0.01, foreach=False)
    ref.grad = g.cpu()
    topt.step()
    assert rel_err(model.flat_params, ref.detach()) < 1e-6
    # the packed kernel weights follow the update: the stepped model equals a
    # fresh model loaded with the updated parameters, forward and gradient
    xq = torch.randn(1, 32, 16, 16, 16, device=DEV)
    tq = torch.tensor([3], device=DEV)
    Pn = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
    fresh, _ = _c1_model_and_diffusion(Pn)
    with torch.no_grad():
        o2, o2_ref = model(xq, tq), fresh(xq, tq)
    assert rel_err(o2, o2_ref) < 1e-6
    assert rel_err(o2.cpu(), ou.unet_forward(Pn, xq.cpu(), tq.cpu(), num_groups=8, **cases.C1_CFG)) < 1e-3
    # a second training step's gradient is taken at the updated weights
    opt.zero_grad()
    terms2, _, _ = diffusion.training_losses(model, vols, t, mode="i2i", contr="t2w", noise=noise)
    terms2["mse_wav"].mean().backward()
    Pr2 = {k: v.clone().requires_grad_(True) for k, v in Pn.items()}

    def om2(x, tt, **kw):
        return ou.unet_forward(Pr2, x, tt, num_groups=8, **cases.C1_CFG)
    r2, _, _ = od.training_losses(tab, om2, {k: v.cpu() for k, v in vols.items()}, t.cpu(), noise.cpu(),
                                  contr="t2w")
    r2["mse_wav"].mean().backward()
    for n, p in model.named_parameters():
        err = float((p.grad.double().cpu() - Pr2[n].grad.double()).norm() /
                    Pr2[n].grad.double().norm().clamp_min(1e-30))
        assert err < 1e-3, ("step 2", n, err)


def test_trainloop_runs_and_learns(tmp_path, monkeypatch):
    from guided_diffusion import dist_util, train_util
    monkeypatch.setenv("CWDM_LOGDIR", str(tmp_path))
    dist_util.setup_dist()
    P = ou.random_params(seed=41, **cases.C1_CFG)
    model, diffusion = _c1_model_and_diffusion(P)
    batch = cases.data.brats_batch(32, seed=5, batch=1)
    data = [batch] * 2
    loop = train_util.TrainLoop(model=model, diffusion=diffusion, data=data, batch_size=1, in_channels=32,
                                image_size=64, microbatch=-1, lr=1e-4, ema_rate="0.9999", log_interval=1,
                                contr="t1n", save_interval=100, resume_checkpoint="", resume_step=0,
                                lr_anneal_steps=4, mode="i2i", diffusion_steps=1000)
    p0 = model.flat_params.detach().clone()
    loop.run_loop()
    assert loop.step == 4
    assert not torch.equal(p0, model.flat_params)
    assert torch.isfinite(model.flat_params).all()
    assert float(loop.last_info["norm/grad_max"]) > 0
    # the fused norms (cwdm_adamw_maxabs) == the reference's reductions over the same buffers
    pb = model.flat_params.detach().clone()
    loop.run_step({k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in batch.items()}, {}, info={})
    assert float(loop.last_info["norm/param_max"]) == float(pb.abs().max())
    assert float(loop.last_info["norm/grad_max"]) == float(model.flat_grad().abs().max())
    assert os.path.exists(os.path.join(tmp_path, "checkpoints", "brats_t1n_BEST_direct_1000.pt"))
    sd = torch.load(os.path.join(tmp_path, "checkpoints", "brats_t1n_BEST_direct_1000.pt"), weights_only=True)
    assert set(sd) == set(P)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def test_trainloop_fp16_device_scaled_step_matches_gradscaler_step(tmp_path, monkeypatch):
    """fp16 TrainLoop (dynamic loss scaling): the sync-free step (FlatAdamW skips
    on GradScaler's device found_inf, the step count on the device) against
    GradScaler.step (found_inf read back, optimizer.step skipped on the host):
    the same parameters and moments after a normal step and two overflowing ones
    (scale forced to 2^60: both skip, the scale halves each time), and the same
    saved step count."""
    import numpy as np
    from guided_diffusion import dist_util, train_util
    monkeypatch.setenv("CWDM_LOGDIR", str(tmp_path))
    dist_util.setup_dist()
    P = ou.random_params(seed=43, **cases.C1_CFG)
    batch = cases.data.brats_batch(32, seed=6, batch=1)
    bdev = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in batch.items()}
    res = {}
    for dev_step in (False, True):
        model, diffusion = _c1_model_and_diffusion(P, dtype="fp16")
        loop = train_util.TrainLoop(model=model, diffusion=diffusion, data=[batch], batch_size=1, in_channels=32,
                                    image_size=64, microbatch=-1, lr=1e-4, ema_rate="0.9999", log_interval=100,
                                    contr="t1n", save_interval=100, resume_checkpoint="", resume_step=0,
                                    lr_anneal_steps=0, mode="i2i", diffusion_steps=1000)
        assert loop.grad_scaler.is_enabled()
        loop.device_scaled_step = dev_step
        torch.manual_seed(0)
        np.random.seed(0)
        p_after = []
        for i in range(3):
            if i == 1:
                loop.grad_scaler.update(2.0 ** 60)
            loop.run_step(bdev, {}, info={})
            p_after.append(model.flat_params.detach().clone())
        torch.cuda.synchronize()
        step = float(next(iter(loop.opt.state_dict()["state"].values()))["step"])
        res[dev_step] = (p_after, loop.opt._m.clone(), loop.opt._v.clone(), step, float(loop.grad_scaler.get_scale()))
    (pa, ma, va, sa, ka), (pb, mb, vb, sb, kb) = res[False], res[True]
    assert sa == sb == 1.0, (sa, sb)
    assert ka == kb == 2.0 ** 58, (ka, kb)
    assert torch.equal(pa[1], pa[0]) and torch.equal(pb[1], pb[0]) and torch.equal(pb[2], pb[0])
    for x, y in ((pa[2], pb[2]), (ma, mb), (va, vb)):
        assert float((x - y).abs().max()) <= 1e-6 * float(x.abs().max().clamp_min(1e-30)), float((x - y).abs().max())
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


# --------------------------------------------------------------------------- production-size backward (config 3)
PROD_CFG = dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4))
PROD_GRID = (32, 32, 64)   # W % 32 == 0 at R0 and R1: the DMA-staged kernel runs forward and dgrad


def _prod_case(seed=51):
    P = ou.random_params(seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(1, 32, *PROD_GRID, generator=g)
    t = torch.tensor([500])
    R = torch.randn(1, 8, *PROD_GRID, generator=g)
    return P, x, t, R


_PROD_REF = {}


def _prod_oracle(seed=51):
    if seed not in _PROD_REF:
        P, x, t, R = _prod_case(seed)
        _PROD_REF[seed] = _oracle_grads(PROD_CFG, 32, P, x, t, R)
    return _PROD_REF[seed]


@pytest.mark.parametrize("path", [2, 0])
def test_production_unet_backward_vs_oracle_autograd(path):
    """The run.sh U-Net (81.5 M parameters) backward at a grid where the
    DMA-staged conv kernel runs the forward and the dgrad convs (path 2 forces
    it wherever the shape allows; path 0 is the production auto policy), fp32:
    every parameter gradient within 1e-3 rel-L2 of the oracle's autograd."""
    from cwdm_hip._lib import lib
    P, x, t, R = _prod_case()
    prev = lib().cwdm_conv3d_set_path(path)
    try:
        out, grads, _ = _unet_grads(PROD_CFG, 32, P, x, t, R, "fp32")
    finally:
        lib().cwdm_conv3d_set_path(prev)
    ref_out, ref = _prod_oracle()
    assert rel_err(out, ref_out) < 1e-3
    assert set(grads) == set(ref) and len(ref) == len(P)
    worst = {k: float((grads[k].double() - ref[k].double()).norm() / ref[k].double().norm().clamp_min(1e-30))
             for k in ref}
    bad = {k: v for k, v in worst.items() if v > 1e-3}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:8]
    print("max grad rel-L2", max(worst.values()))


@pytest.mark.parametrize("dtype,tol_out,tol_grad", [("bf16", 5e-2, 8e-2), ("fp16", 1e-2, 1.5e-2)])
def test_production_unet_backward_half_close_to_fp32(dtype, tol_out, tol_grad):
    """The 16-bit training paths (bf16: the config-3 benchmark dtype; fp16:
    config 5's) on the same case: every gradient within tol_grad rel-L2 of the
    fp32 oracle (16-bit activations and weights, fp32 accumulation; bf16
    measured worst 4.7e-2, GroupNorm affine grads of the 16^3/8^3 levels)."""
    from cwdm_hip._lib import lib
    P, x, t, R = _prod_case()
    prev = lib().cwdm_conv3d_set_path(2)
    try:
        out, grads, _ = _unet_grads(PROD_CFG, 32, P, x, t, R, dtype)
    finally:
        lib().cwdm_conv3d_set_path(prev)
    ref_out, ref = _prod_oracle()
    worst = {k: float((grads[k].double() - ref[k].double()).norm() / ref[k].double().norm().clamp_min(1e-30))
             for k in ref}
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:5]
    print(dtype, "out rel", rel_err(out, ref_out), "worst grads", top)
    assert rel_err(out, ref_out) < tol_out
    assert top[0][1] < tol_grad, top


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_production_unet_backward_kept_activations(dtype):
    """The training workspace (cwdm_unet_train_workspace_bytes): the forward
    keeps every DMA-staged conv's activated input and their weight gradients
    stage it by LDS-DMA (wgrad u_cm) instead of recomputing GroupNorm+SiLU --
    the same products up to the recompute's 16-bit rounding and the atomics'
    order: every gradient within 5e-3 rel-L2 of the recompute path, and the
    output bit-identical (the forward only writes the pre-pass elsewhere)."""
    from cwdm_hip._lib import lib
    P, x, t, R = _prod_case()
    prev = lib().cwdm_conv3d_set_path(2)
    try:
        out_k, g_k, m = _unet_grads(PROD_CFG, 32, P, x, t, R, dtype, keep=True)
        B, _, D, H, W = x.shape
        assert m.plan.train_workspace_bytes(B, D, H, W) > m.plan.workspace_bytes(B, D, H, W)
        out_r, g_r, _ = _unet_grads(PROD_CFG, 32, P, x, t, R, dtype, keep=False)
    finally:
        lib().cwdm_conv3d_set_path(prev)
    assert torch.equal(out_k, out_r)
    worst = {k: float((g_k[k].double() - g_r[k].double()).norm() / g_r[k].double().norm().clamp_min(1e-30))
             for k in g_r}
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:5]
    print(dtype, "kept vs recompute worst", top)
    assert top[0][1] < 5e-3, top


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_production_unet_backward_skip_dgrad_row_major_epilogue_bitwise(dtype):
    """The fused 1x1 skip dgrad + GroupNorm-backward apply (pw_kernel) with the
    row-major LDS epilogue (default) against the swapped-lane epilogue it
    replaced: the same products summed in the same order, so every gradient is
    bitwise equal -- and the row-major instance did run."""
    from cwdm_hip._lib import lib
    L = lib()
    P, x, t, R = _prod_case()
    prev, prevlt = L.cwdm_conv3d_set_path(0), L.cwdm_debug_pw_lt(1)
    try:
        n0 = L.cwdm_debug_pw_lt(-1)
        out_a, g_a, _ = _unet_grads(PROD_CFG, 32, P, x, t, R, dtype)
        n1 = L.cwdm_debug_pw_lt(-1)
        L.cwdm_debug_pw_lt(0)
        out_b, g_b, _ = _unet_grads(PROD_CFG, 32, P, x, t, R, dtype)
        assert L.cwdm_debug_pw_lt(-1) == n1
    finally:
        L.cwdm_conv3d_set_path(prev)
        L.cwdm_debug_pw_lt(prevlt)
    assert n1 > n0, "the row-major skip dgrad did not run"
    assert torch.equal(out_a, out_b)
    bad = [k for k in g_b if not torch.equal(g_a[k], g_b[k])]
    assert not bad, bad[:8]


def test_flat_adamw_state_dict_per_parameter_steps():
    """FlatAdamW keeps one step tensor for all parameters (one host fill per step);
    its state_dict hands out a separate step tensor per parameter, as
    torch.optim.AdamW keeps them, and a reload restores the step count."""
    from cwdm_hip.optim import FlatAdamW
    P, x, t, R = _prod_case()
    model = _product_model(PROD_CFG, 32, P, "bf16")
    opt = FlatAdamW(model, lr=1e-3, weight_decay=0.01, direct_grads=True)
    for _ in range(2):
        opt.zero_grad()
        out = model(x.to(DEV), t.to(DEV))
        (out * R.to(DEV)).sum().backward()
        opt.step()
    sd = opt.state_dict()
    steps = [v["step"] for v in sd["state"].values()]
    assert len(steps) == len(list(model.parameters()))
    assert len({id(s) for s in steps}) == len(steps)
    assert all(float(s) == 2.0 for s in steps)
    opt2 = FlatAdamW(model, lr=1e-3, weight_decay=0.01)
    opt2.load_state_dict(sd)
    assert opt2._step == 2 and torch.equal(opt2._m, opt._m) and torch.equal(opt2._v, opt._v)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
def test_production_training_two_steps_bitwise_reproducible(dtype):
    """Determinism of the training step: two runs of two steps each (forward with
    kept activations, backward, fused AdamW) from the same weights and inputs give
    bitwise-identical gradients and parameters.  Every reduction of the backward
    -- weight-gradient tiles (per-range slabs + a fixed-order pass), bias /
    emb-projection channel sums, GroupNorm statistics -- is summed in a fixed
    order, none by fp32 atomics."""
    from cwdm_hip._lib import lib
    from cwdm_hip.optim import FlatAdamW
    P, x, t, R = _prod_case()
    g = torch.Generator().manual_seed(77)
    x2 = torch.randn(x.shape, generator=g)
    prev = lib().cwdm_conv3d_set_path(0)

    def run():
        model = _product_model(PROD_CFG, 32, P, dtype)
        model.keep_activations = True
        opt = FlatAdamW(model, lr=1e-3, weight_decay=0.01, direct_grads=True)
        grads = []
        for xi in (x, x2):
            opt.zero_grad()
            out = model(xi.to(DEV), t.to(DEV))
            (out * R.to(DEV)).sum().backward()
            grads.append(model.flat_grad().detach().clone())
            opt.step()
        torch.cuda.synchronize()
        return grads, model.flat_params.detach().clone()

    try:
        g_a, p_a = run()
        g_b, p_b = run()
    finally:
        lib().cwdm_conv3d_set_path(prev)
    for i in range(2):
        assert torch.isfinite(g_a[i]).all()
        assert torch.equal(g_a[i], g_b[i]), ("step", i, float((g_a[i] - g_b[i]).abs().max()))
    assert not torch.equal(g_a[0], g_a[1])
    assert torch.equal(p_a, p_b)


@pytest.mark.parametrize("k", [0, 1], ids=["tiny", "runsh"])
def test_unet_resblock_updown_false_backward_vs_oracle_autograd(k):
    """Backward of the stride-2 Downsample conv (expanded-weight wgrad folded
    back onto the 27 taps, dgrad + depth-to-space) and of the Upsample conv
    (wgrad on the nearest-x2 input, dgrad + the nearest adjoint), whole U-Net,
    fp32: every gradient within 1e-3 rel-L2 of the oracle's autograd."""
    from guided_diffusion.unet import UNetModel
    cfgs = [(dict(in_channels=32, model_channels=32, out_channels=8, num_res_blocks=1, channel_mult=(1, 2)), 8,
             (16, 16, 16)),
            (dict(in_channels=32, model_channels=64, out_channels=8, num_res_blocks=2, channel_mult=(1, 2, 2, 4, 4)),
             32, (16, 32, 32))]
    cfg, G, grid = cfgs[k]
    P = ou.random_params(seed=27, resblock_updown=False, **cfg)
    m = UNetModel(image_size=2 * grid[0], in_channels=cfg["in_channels"], model_channels=cfg["model_channels"],
                  out_channels=cfg["out_channels"], num_res_blocks=cfg["num_res_blocks"], attention_resolutions=(),
                  channel_mult=cfg["channel_mult"], dims=3, resblock_updown=False, bottleneck_attention=False,
                  resample_2d=False, num_groups=G, compute_dtype="fp32")
    m.load_state_dict(P)
    m.to(DEV)
    g = torch.Generator().manual_seed(28)
    x = torch.randn(2, 32, *grid, generator=g)
    t = torch.tensor([9, 444])
    R = torch.randn(2, 8, *grid, generator=g)
    out = m(x.to(DEV), t.to(DEV))
    (out * R.to(DEV)).sum().backward()
    Pr = {kk: v.clone().requires_grad_(True) for kk, v in P.items()}
    ref = ou.unet_forward(Pr, x, t, num_groups=G, resblock_updown=False, **cfg)
    (ref * R).sum().backward()
    assert rel_err(out.detach(), ref.detach()) < 1e-3
    worst = {n: float((p.grad.double().cpu() - Pr[n].grad.double()).norm() / Pr[n].grad.double().norm().clamp_min(1e-30))
             for n, p in m.named_parameters()}
    bad = {n: v for n, v in worst.items() if v > 1e-3}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:8]
    assert any(".op." in n for n in worst) and any(".conv." in n for n in worst)
