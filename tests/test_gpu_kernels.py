"""Kernel-level parity on the GPU (libcwdm through the C ABI) against the
oracle / plain PyTorch-CPU fp32 references of the same op."""
import ctypes
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import haar

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dtn():
    from cwdm_hip import _lib
    return {"fp32": (_lib.CWDM_F32, torch.float32), "bf16": (_lib.CWDM_BF16, torch.bfloat16),
            "fp16": (_lib.CWDM_F16, torch.float16)}


class _LazyDTN(dict):
    def __missing__(self, k):
        self.update(_dtn())
        return dict.__getitem__(self, k)


_DTN = _LazyDTN()   # dtype name -> (CWDM_*, torch dtype)


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


# --------------------------------------------------------------------------- wavelets
@pytest.mark.parametrize("shape", [(1, 1, 2, 2, 2), (2, 3, 8, 12, 10), (1, 1, 64, 64, 64), (2, 1, 18, 6, 4)])
def test_dwt_idwt_bitexact_vs_oracle(shape):
    from cwdm_hip import ops
    g = torch.Generator().manual_seed(0)
    x = torch.rand(shape, generator=g)
    bands = ops.dwt3d(x.to(DEV)).cpu()
    ref = haar.dwt3d(x)
    for k in range(8):
        assert torch.equal(bands[k], ref[k]), k
    B, C, D, H, W = shape
    v = (D // 2) * (H // 2) * (W // 2)
    rec = ops.idwt3d(bands.to(DEV).contiguous(), (B * C * v, C * v, v, 1), B, C, D // 2, H // 2, W // 2).cpu()
    assert torch.equal(rec, haar.idwt3d(*ref))
    assert (rec - x).abs().max() < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_idwt_from_separate_planes_bitexact(dtype):
    """IDWT_3D's eight arguments go to the kernel as eight pointers (no stack
    copy): bit-exact vs the oracle on the same (dtype-rounded) bands."""
    from cwdm_hip import ops
    g = torch.Generator().manual_seed(4)
    bands = [torch.randn(2, 3, 4, 6, 5, generator=g).to(dtype) for _ in range(8)]
    got = ops.idwt3d_planes([b.to(DEV) for b in bands]).cpu()
    assert torch.equal(got, haar.idwt3d(*[b.float() for b in bands]))


@pytest.mark.parametrize("shape", [(1, 1, 8, 8, 8), (2, 1, 16, 12, 20)])
def test_prepare_batch_bitexact_vs_oracle(shape):
    """cwdm_prepare_batch (training_losses front end, gaussian_diffusion.py:1131-1149):
    the 32-channel model input and the x0 target equal the oracle's DWTs and
    q_sample bit for bit."""
    from cwdm_hip import ops
    from oracle import diffusion as od
    from guided_diffusion import script_util
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i")
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"))
    g = torch.Generator().manual_seed(6)
    vols = [torch.rand(shape, generator=g) for _ in range(4)]
    eps = torch.randn(shape, generator=g)
    t = torch.tensor([0, 999][:shape[0]]) if shape[0] <= 2 else torch.randint(0, 1000, (shape[0],))
    x_in, x0 = ops.prepare_batch(*[v.to(DEV) for v in vols], eps.to(DEV), d.q_coef_table(DEV), t.to(DEV), 1000)
    rx0 = haar.dwt_cat(vols[0])
    cond = torch.cat([haar.dwt_cat(v) for v in vols[1:]], 1)
    reps = torch.cat(list(haar.dwt3d(eps)), 1)
    rxt = od.q_sample(tab, rx0, t, reps)
    assert torch.equal(x0.cpu(), rx0)
    assert torch.equal(x_in[:, 8:].cpu(), cond)
    assert torch.equal(x_in[:, :8].cpu(), rxt)


def test_dwt_module_api_and_autograd():
    from DWT_IDWT.DWT_IDWT_layer import DWT_3D, IDWT_3D
    x = torch.rand(2, 1, 8, 8, 8, device=DEV, requires_grad=True)
    bands = DWT_3D("haar")(x)
    assert len(bands) == 8 and bands[0].shape == (2, 1, 4, 4, 4)
    y = [torch.randn_like(b) for b in bands]
    loss = sum((b * yy).sum() for b, yy in zip(bands, y))
    loss.backward()
    adj = IDWT_3D("haar")(*y)           # adjoint == inverse for Haar
    assert torch.allclose(x.grad, adj, atol=1e-5)
    ref = haar.dwt3d_matrix(x.detach().cpu())
    for b, r in zip(bands, ref):
        assert torch.allclose(b.detach().cpu(), r, atol=1e-6)


def test_dwt_bf16_and_strided_output_into_channel_slice():
    from cwdm_hip import ops
    x = torch.rand(2, 1, 16, 16, 16)
    V = 8 ** 3
    buf = torch.zeros(2, 32, 8, 8, 8, device=DEV)
    ops.dwt3d(x.to(DEV), lll_div3=True, out=buf[:, 8:], out_strides=(V, 32 * V, 0, 1))
    ref = haar.dwt_cat(x)
    assert torch.equal(buf[:, 8:16].cpu(), ref)
    assert torch.count_nonzero(buf[:, :8]) == 0 and torch.count_nonzero(buf[:, 16:]) == 0
    out = torch.empty(8, 2, 1, 8, 8, 8, device=DEV, dtype=torch.bfloat16)
    ops.dwt3d(x.to(DEV), out=out, out_strides=(2 * V, V, V, 1))
    refb = torch.stack(haar.dwt3d(x), 0).to(torch.bfloat16)
    assert torch.equal(out.cpu(), refb)
    outh = torch.empty(8, 2, 1, 8, 8, 8, device=DEV, dtype=torch.float16)
    ops.dwt3d(x.to(DEV), out=outh, out_strides=(2 * V, V, V, 1))
    assert torch.equal(outh.cpu(), torch.stack(haar.dwt3d(x), 0).to(torch.float16))


# --------------------------------------------------------------------------- sampler
@pytest.mark.parametrize("clip", [True, False])
@pytest.mark.parametrize("mean_type", [0, 1])
def test_sampler_step_vs_oracle(clip, mean_type):
    from oracle import diffusion as od
    from guided_diffusion import script_util
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=(mean_type == 0), mode="i2i")
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"))
    g = torch.Generator().manual_seed(1)
    B, n = 3, 6
    mo = torch.randn(B, 8, n, n, n, generator=g) * 0.5
    x = torch.randn(B, 8, n, n, n, generator=g)
    noise = torch.randn(B, 8, n, n, n, generator=g)
    t = torch.tensor([0, 17, 999])
    sample, pred = d._epilogue(mo.to(DEV), x.to(DEV), t.to(DEV), clip, None, noise.to(DEV))
    if mean_type == 0:
        x0 = mo
    else:
        x0 = od.extract(tab.sqrt_recip_alphas_cumprod, t, x.shape) * x - \
            od.extract(tab.sqrt_recipm1_alphas_cumprod, t, x.shape) * mo
    pref = od.process_xstart(x0) if clip else x0
    mean = od.extract(tab.posterior_mean_coef1, t, x.shape) * pref + od.extract(tab.posterior_mean_coef2, t, x.shape) * x
    mask = (t != 0).float().view(-1, 1, 1, 1, 1)
    sref = mean + mask * torch.exp(0.5 * od.extract(tab.fixed_large_log_variance, t, x.shape)) * noise
    assert rel_err(pred, pref) < 1e-6
    assert rel_err(sample, sref) < 1e-6
    assert torch.equal(sample[0].cpu(), mean[0]) or rel_err(sample[0], mean[0]) < 1e-6  # t = 0: no noise


@pytest.mark.parametrize("eta", [0.0, 0.5])
def test_ddim_step_vs_oracle(eta):
    """The DDIM update of the fused kernel (update=1) vs oracle.ddim_sample on
    respaced ddim10 tables, model output injected: bit-level agreement."""
    from oracle import diffusion as od
    from guided_diffusion import script_util
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                              timestep_respacing="ddim10")
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), use_timesteps=od.space_timesteps(1000, "ddim10"))
    g = torch.Generator().manual_seed(3)
    B, n = 3, 6
    mo = torch.randn(B, 8, n, n, n, generator=g) * 0.5 + 0.2
    x = torch.randn(B, 8, n, n, n, generator=g)
    cond = torch.zeros(B, 24, n, n, n)
    t = torch.tensor([0, 4, 9])
    sample, pred = d._epilogue(mo.to(DEV), x.to(DEV), t.to(DEV), True, None, None, update=1, eta=eta)
    ref = od.ddim_sample(tab, lambda xc, tt: mo, x, t, cond, clip_denoised=True, eta=eta)
    assert rel_err(pred, ref["pred_xstart"]) < 1e-6
    assert rel_err(sample, ref["sample"]) < 1e-6
    assert torch.equal(sample[0].cpu(), pred[0].cpu())   # t = 0: acp_prev = 1, the sample is x0


# --------------------------------------------------------------------------- conv3d
def _conv_call(dtype, out_grid, a0, a1, amode, gn, w, bias, bvec_bstride=0, b0=None, b1=None, wb=None, res=None,
               rmode=-1, out_f32=False, stats=True, split=True, wsplit=False):
    """Run cwdm_conv3d_forward on NDHWC tensors; returns (out, stats)."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    B, D, H, W = out_grid
    cout = w.shape[0]
    tdt = {_lib.CWDM_F32: torch.float32, _lib.CWDM_BF16: torch.bfloat16, _lib.CWDM_F16: torch.float16}[dtype]
    L = lib()

    def pack(wt, k):
        nbytes = L.cwdm_conv3d_packed_bytes(cout, wt.shape[1], k, dtype)
        assert nbytes > 0
        buf = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
        check(L.cwdm_conv3d_pack(ctypes.c_void_p(wt.data_ptr()), cout, wt.shape[1], k, dtype,
                                 ctypes.c_void_p(buf.data_ptr()), None))
        return buf

    pa = pack(w.to(DEV).contiguous(), 3)
    pb = pack(wb.to(DEV).contiguous(), 1) if wb is not None else None
    out = torch.empty(B, D, H, W, cout, device=DEV, dtype=torch.float32 if out_f32 else tdt)
    parts = L.cwdm_conv3d_parts(dtype, D, H, W, cout)
    st = torch.zeros(B, parts, cout, 2, device=DEV) if stats else None
    d = _lib.ConvDesc()
    d.dtype, d.B, d.D, d.H, d.W, d.cout = dtype, B, D, H, W, cout
    d.a0, d.a_c0 = a0.data_ptr(), a0.shape[-1]
    d.a1, d.a_c1 = (a1.data_ptr(), a1.shape[-1]) if a1 is not None else (None, 0)
    d.a_mode = amode
    d.a_gn = gn.data_ptr() if gn is not None else None
    d.a_w = pa.data_ptr()
    if wb is not None:
        d.b0, d.b_c0 = b0.data_ptr(), b0.shape[-1]
        d.b1, d.b_c1 = (b1.data_ptr(), b1.shape[-1]) if b1 is not None else (None, 0)
        d.b_w = pb.data_ptr()
    d.bias, d.bias_bstride = bias.data_ptr(), bvec_bstride
    d.res, d.res_mode = (res.data_ptr() if res is not None else None), rmode
    d.out, d.out_dtype = out.data_ptr(), (_lib.CWDM_F32 if out_f32 else dtype)
    d.stats = st.data_ptr() if st is not None else None
    psplit = None
    if wsplit:   # the accurate fast mode's split-bf16 weights (fp32 convs)
        psplit = torch.empty(L.cwdm_conv3d_packed_split_bytes(cout, w.shape[1]), dtype=torch.uint8, device=DEV)
        check(L.cwdm_conv3d_pack_split(ctypes.c_void_p(w.to(DEV).contiguous().data_ptr()), cout, w.shape[1],
                                       ctypes.c_void_p(psplit.data_ptr()), None))
        d.a_w_split = psplit.data_ptr()
    nws = L.cwdm_conv3d_workspace_bytes(ctypes.byref(d))
    ws = None
    if nws > 0 and split:
        ws = torch.empty(nws, dtype=torch.uint8, device=DEV)
        d.workspace, d.ws_bytes = ws.data_ptr(), nws
    check(L.cwdm_conv3d_forward(ctypes.byref(d), None))
    torch.cuda.synchronize()
    return out, st


def _nd(x):  # NCDHW -> NDHWC
    return x.permute(0, 2, 3, 4, 1).contiguous()


def _nc(x):
    return x.permute(0, 4, 1, 2, 3).contiguous()


CASES = [
    # name, B, grid(out), c0, c1, cout, amode, gn, skip1x1, rmode
    ("plain", 1, (8, 16, 32), 32, 0, 64, 0, False, False, -1),
    ("gn_concat_skip", 2, (8, 8, 16), 32, 16, 64, 0, True, True, -1),
    ("down_pool_res", 1, (4, 8, 16), 64, 0, 64, 2, True, False, 2),
    ("up_res", 1, (8, 16, 32), 32, 0, 32, 1, True, False, 1),
    ("same_res", 1, (6, 10, 12), 64, 0, 64, 0, True, False, 0),
    ("cout8", 2, (8, 8, 8), 64, 0, 8, 0, True, False, -1),
    ("small_grid", 1, (4, 4, 4), 128, 128, 128, 0, True, True, -1),
]


@pytest.mark.parametrize("split", [True, False], ids=["splitk", "nosplit"])
@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv3d_fused_vs_torch(case, dtype_name, split):
    _run_conv_case(case, dtype_name, split)


def _random_conv_cases(n, seed):
    """Seeded shapes drawn inside the ABI's limits (channels multiples of 16; even grids for resampling):
    odd extents, partial bricks and partial x tiles, every input/residual mode, GN, concat, 1x1 skip."""
    import random
    r = random.Random(seed)
    out = []
    for i in range(n):
        amode = r.choice([0, 0, 1, 2])
        rmode = r.choice([-1, 0, 1, 2])
        even = amode == 1 or rmode == 1
        ext = [r.randint(1, 10) * (2 if even else 1) for _ in range(2)] + [r.choice([r.randint(2, 24), r.randint(32, 72)])]
        if even:
            ext[2] += ext[2] % 2
        cout = r.choice([8, 16, 24, 32, 64, 96, 128, 192])
        if r.random() < 0.4:  # shapes the DMA kernel takes (W >= 32, D, H % 4 == 0, cout % 64 == 0)
            ext[0], ext[1], ext[2] = 4 * r.randint(1, 3), 4 * r.randint(1, 3), 2 * r.randint(16, 36)
            cout = r.choice([64, 128, 192])
        c0 = 16 * r.randint(1, 6)
        c1 = r.choice([0, 0, 16, 32])
        out.append((f"rand{i}", r.randint(1, 2), tuple(ext), c0, c1, cout, amode, r.random() < 0.7,
                    amode == 0 and r.random() < 0.4, rmode))   # the 1x1 skip reads the output grid
    return out


RANDOM_CASES = _random_conv_cases(24, 20261016)


@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", RANDOM_CASES, ids=[c[0] for c in RANDOM_CASES])
def test_conv3d_random_shapes_vs_torch(case, dtype_name):
    _run_conv_case(case, dtype_name, True)


def _run_conv_case(case, dtype_name, split):
    from cwdm_hip import _lib
    name, B, grid, c0, c1, cout, amode, use_gn, skip, rmode = case
    dtype, tdt = _DTN[dtype_name]
    g = torch.Generator().manual_seed(7)
    D, H, W = grid
    sD, sH, sW = {0: (D, H, W), 1: (D // 2, H // 2, W // 2), 2: (2 * D, 2 * H, 2 * W)}[amode]
    cin = c0 + c1
    a0 = torch.randn(B, c0, sD, sH, sW, generator=g)
    a1 = torch.randn(B, c1, sD, sH, sW, generator=g) if c1 else None
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
    bias = torch.randn(cout, generator=g) * 0.1
    x = torch.cat([a0, a1], 1) if c1 else a0
    # quantise inputs to the compute dtype so both sides see the same operands
    x = x.to(tdt).float()
    a0q, a1q = x[:, :c0], (x[:, c0:] if c1 else None)
    wq = w.to(tdt).float()
    gn = None
    if use_gn:
        scale = 1 + 0.2 * torch.randn(B, cin, generator=g)
        shift = 0.2 * torch.randn(B, cin, generator=g)
        gn = torch.stack([scale, shift], -1).contiguous()
        h = F.silu(x * scale[:, :, None, None, None] + shift[:, :, None, None, None])
    else:
        h = x
    if amode == 2:
        h = F.avg_pool3d(h, 2)
    elif amode == 1:
        h = F.interpolate(h, scale_factor=2, mode="nearest")
    if dtype_name != "fp32":
        h = h.to(tdt).float()   # the kernel stages the transformed halo in bf16 / fp16
    ref = F.conv3d(h, wq, bias, padding=1)
    wb = b0 = b1 = None
    if skip:
        wb = torch.randn(cout, cin, 1, 1, 1, generator=g) / math.sqrt(cin)
        ref = ref + F.conv3d(x, wb.to(tdt).float())
        b0, b1 = a0q, a1q
    res = None
    if rmode >= 0:
        rsh = {0: (D, H, W), 1: (D // 2, H // 2, W // 2), 2: (2 * D, 2 * H, 2 * W)}[rmode]
        res = torch.randn(B, cout, *rsh, generator=g).to(tdt).float()
        rr = {0: res, 1: F.interpolate(res, scale_factor=2, mode="nearest"), 2: F.avg_pool3d(res, 2)}[rmode]
        ref = ref + rr
    out, st = _conv_call(
        dtype, (B, D, H, W), _nd(a0q).to(DEV, tdt), _nd(a1q).to(DEV, tdt) if c1 else None, amode,
        gn.to(DEV) if gn is not None else None, wq.to(DEV), bias.to(DEV),
        b0=_nd(b0).to(DEV, tdt) if skip else None, b1=_nd(b1).to(DEV, tdt) if (skip and c1) else None,
        wb=wb.to(tdt).float().to(DEV) if skip else None, res=_nd(res).to(DEV, tdt) if res is not None else None,
        rmode=rmode, out_f32=(cout == 8), split=split)
    got = _nc(out.float().cpu())
    tol = {"fp32": 2e-5, "bf16": 2e-2, "fp16": 3e-3}[dtype_name]   # output rounding: 2^-8 / 2^-11
    assert rel_err(got, ref) < tol, name
    # per-channel statistics of the stored (pre-rounding) output
    s = st.sum(1).cpu()
    ref_sum = ref.sum(dim=(2, 3, 4))
    assert torch.allclose(s[..., 0], ref_sum, rtol=1e-3, atol=1e-2 * ref.abs().max().item() * 8)


V4_CASES = [
    # name, B, grid(out), c0, c1, cout, amode, gn, skip1x1, rmode  (W >= 32, H, D % 4 == 0, cout % 64 == 0)
    ("v4_plain", 1, (8, 8, 64), 32, 0, 64, 0, False, False, -1),
    ("v4_gn_concat_skip_res", 2, (4, 8, 32), 32, 16, 64, 0, True, True, 0),
    ("v4_up_res", 1, (8, 4, 64), 32, 0, 128, 1, True, False, 1),
    ("v4_concat_nogn", 1, (4, 12, 32), 16, 32, 128, 0, False, False, 0),
    # K-split work items (fewer tiles than CU slots): partial slices + finish pass
    ("v4_ksplit_gn_skip", 1, (8, 4, 32), 96, 32, 128, 0, True, True, 0),
    ("v4_ksplit_up", 2, (8, 8, 32), 64, 0, 64, 1, True, False, 1),
    # W not a multiple of 32: the last x tile is partial (masked stores / statistics)
    ("v4_partial_x_gn_res", 1, (4, 8, 56), 64, 0, 64, 0, True, False, 0),
    ("v4_partial_x_ksplit_up", 1, (8, 4, 40), 64, 0, 64, 1, True, False, 1),
    ("v4_partial_x_concat_skip", 2, (4, 4, 48), 32, 16, 64, 0, True, True, -1),
    # 24 <= W < 32 (r03): one partial x tile (config 5's 28^3 level, 32-channel tiles)
    ("v4_w28_config5_res", 1, (28, 28, 28), 128, 0, 128, 0, True, False, 0),
    ("v4_w24_concat_skip", 1, (8, 8, 24), 64, 64, 64, 0, True, True, -1),
    ("v4_w26_up_res", 2, (8, 8, 26), 64, 0, 64, 1, True, False, 1),
]


@pytest.mark.parametrize("path", [3, 2], ids=["v4", "v5"])
@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", V4_CASES, ids=[c[0] for c in V4_CASES])
def test_conv3d_dma_kernel_vs_torch(case, dtype_name, path):
    """The DMA-staged wide-grid kernels, forced on small shapes, against
    F.conv3d: path 3 = conv3d_v4.hpp (GroupNorm pre-pass, K split), path 2 =
    the warp-specialised conv3d_v5.hip for 16-bit shapes it takes (GroupNorm +
    SiLU in LDS, helper-wave epilogue; fp32 stays on v4)."""
    from cwdm_hip._lib import lib
    L = lib()
    prev = L.cwdm_conv3d_set_path(path)
    try:  # with a workspace: the GroupNorm pre-pass, the 1x1 skip and the K-split partials live there
        test_conv3d_fused_vs_torch(case, dtype_name, True)
    finally:
        L.cwdm_conv3d_set_path(prev)


V5_CASES = [
    # name, B, grid(out), c0, c1, cout, amode, gn, skip1x1, rmode  -- shapes with enough tiles for
    # several per workgroup under a capped grid: the three-buffer halo rotation, the staged tile
    # hand-off and the two-part drain across tiles of 2..12 chunks
    ("v5_gn_res_2chunk", 2, (8, 8, 64), 32, 0, 64, 0, True, False, 0),
    ("v5_gn_concat_c128", 1, (8, 12, 64), 64, 32, 128, 0, True, False, -1),
    ("v5_up_res_up", 1, (8, 8, 64), 64, 0, 64, 1, True, False, 1),
    ("v5_partial_x_res", 2, (4, 8, 56), 48, 16, 64, 0, True, False, 0),
    ("v5_nogn_c192", 1, (4, 8, 96), 32, 32, 192, 0, False, False, -1),
    ("v5_skip_c12", 1, (4, 4, 64), 128, 64, 64, 0, True, True, -1),
    ("v5_w24_up_nogn", 2, (4, 8, 24), 32, 0, 64, 1, False, False, 1),
]


@pytest.mark.parametrize("cap", [1, 5, 0])
@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("case", V5_CASES, ids=[c[0] for c in V5_CASES])
def test_conv3d_v5_kernel_vs_torch(case, dtype_name, cap):
    """conv3d_v5.hip against F.conv3d with the persistent grid capped at 1 / 5
    workgroups (every workgroup streams many tiles back to back) or uncapped."""
    from cwdm_hip._lib import lib
    L = lib()
    prev, prevg = L.cwdm_conv3d_set_path(2), L.cwdm_debug_v5_grid(cap)
    try:
        _run_conv_case(case, dtype_name, True)
    finally:
        L.cwdm_conv3d_set_path(prev)
        L.cwdm_debug_v5_grid(prevg)


SPLIT_CASES = [
    # name, B, grid(out), c0, c1, cout, amode, gn, skip1x1, rmode (fp32, cout % 64 == 0, W >= 24)
    ("x_gn_res", 2, (8, 8, 64), 32, 0, 64, 0, True, False, 0),
    ("x_gn_concat_c128", 1, (8, 12, 64), 64, 32, 128, 0, True, False, -1),
    ("x_up_gnpre_res_up", 1, (8, 8, 64), 64, 0, 64, 1, True, False, 1),
    ("x_partial_x_nogn", 2, (4, 8, 56), 48, 16, 64, 0, False, False, 0),
    ("x_skip", 1, (4, 4, 64), 128, 64, 64, 0, True, True, -1),
    ("x_w24_up_nogn", 2, (4, 8, 24), 32, 0, 64, 1, False, False, 1),
    # a residual AND a 1x1 skip: the split path refuses it (the skip pre-pass would
    # take the residual slot); the exact-fp32 kernels add both
    ("x_skip_res", 1, (4, 4, 64), 64, 0, 64, 0, True, True, 0),
]


@pytest.mark.parametrize("cap", [3, 0])
@pytest.mark.parametrize("case", SPLIT_CASES, ids=[c[0] for c in SPLIT_CASES])
def test_conv3d_split_bf16_accurate_mode_vs_torch(case, cap):
    """The accurate fast mode (conv3d_v5s_kernel): fp32 in / out, MFMAs on bf16
    hi/lo splits of both operands (hi.hi + lo.hi + hi.lo: 3 passes per 16 channels) -- within 2e-5
    of fp32 F.conv3d on the UNquantised fp32 operands (bf16 is ~1e-2)."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import lib
    L = lib()
    name, B, grid, c0, c1, cout, amode, use_gn, skip, rmode = case
    g = torch.Generator().manual_seed(17)
    D, H, W = grid
    sD, sH, sW = (D // 2, H // 2, W // 2) if amode == 1 else (D, H, W)
    cin = c0 + c1
    x = torch.randn(B, cin, sD, sH, sW, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
    bias = torch.randn(cout, generator=g) * 0.1
    gn = None
    h = x
    if use_gn:
        scale = 1 + 0.2 * torch.randn(B, cin, generator=g)
        shift = 0.2 * torch.randn(B, cin, generator=g)
        gn = torch.stack([scale, shift], -1).contiguous()
        h = F.silu(x * scale[:, :, None, None, None] + shift[:, :, None, None, None])
    if amode == 1:
        h = F.interpolate(h, scale_factor=2, mode="nearest")
    ref = F.conv3d(h.double(), w.double(), bias.double(), padding=1)
    wb = None
    if skip:
        wb = torch.randn(cout, cin, 1, 1, 1, generator=g) / math.sqrt(cin)
        ref = ref + F.conv3d(x.double(), wb.double())
    res = None
    if rmode >= 0:
        res = torch.randn(B, cout, *((D, H, W) if rmode == 0 else (D // 2, H // 2, W // 2)), generator=g)
        ref = ref + (res if rmode == 0 else F.interpolate(res, scale_factor=2, mode="nearest")).double()
    prev, prevg = L.cwdm_conv3d_set_path(0), L.cwdm_debug_v5_grid(cap)
    try:
        out, st = _conv_call(_lib.CWDM_F32, (B, D, H, W), _nd(x[:, :c0]).to(DEV), _nd(x[:, c0:]).to(DEV) if c1 else None,
                             amode, gn.to(DEV) if gn is not None else None, w.to(DEV), bias.to(DEV),
                             b0=_nd(x[:, :c0]).to(DEV) if skip else None,
                             b1=_nd(x[:, c0:]).to(DEV) if (skip and c1) else None,
                             wb=wb.to(DEV) if skip else None, res=_nd(res).to(DEV) if res is not None else None,
                             rmode=rmode, wsplit=True)
    finally:
        L.cwdm_conv3d_set_path(prev)
        L.cwdm_debug_v5_grid(prevg)
    got = _nc(out.cpu()).double()
    assert rel_err(got, ref) < 2e-5, name
    s = st.sum(1).cpu().double()
    assert torch.allclose(s[..., 0], ref.sum(dim=(2, 3, 4)), rtol=1e-4, atol=1e-5 * ref.abs().max().item() * D * H * W)


V5_EXACT_CASES = [
    # >= 256 tiles of 64 channels: v4 runs them without K split or 32-channel tiles
    ("v5x_gn_concat", 1, (16, 32, 128), 64, 32, 128, 0, True, False, -1),
    ("v5x_up_gn", 1, (16, 32, 128), 64, 0, 128, 1, True, False, -1),
    ("v5x_nogn_partial_x", 2, (16, 16, 120), 32, 0, 64, 0, False, False, -1),
]


@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("case", V5_EXACT_CASES, ids=lambda c: c[0])
def test_conv3d_v5_bitexact_vs_v4(case, dtype_name):
    """Without a residual the warp-specialised conv (GroupNorm+SiLU in LDS) stores
    exactly what v4 stores after the cwdm_gn_apply pre-pass: same transform, same
    MFMA order per accumulator, one rounding."""
    from cwdm_hip._lib import lib
    L = lib()
    name, B, grid, c0, c1, cout, amode, use_gn, skip, rmode = case
    dtype, tdt = _DTN[dtype_name]
    g = torch.Generator().manual_seed(9)
    D, H, W = grid
    sD, sH, sW = (D // 2, H // 2, W // 2) if amode == 1 else (D, H, W)
    a0 = torch.randn(B, sD, sH, sW, c0, generator=g).to(DEV, tdt)
    a1 = torch.randn(B, sD, sH, sW, c1, generator=g).to(DEV, tdt) if c1 else None
    w = (torch.randn(cout, c0 + c1, 3, 3, 3, generator=g) / math.sqrt(27 * (c0 + c1))).to(DEV)
    bias = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    gn = None
    if use_gn:
        gn = torch.stack([1 + 0.2 * torch.randn(B, c0 + c1, generator=g), 0.2 * torch.randn(B, c0 + c1, generator=g)],
                         -1).contiguous().to(DEV)
    outs = {}
    for path in (3, 2):
        prev, prevg = L.cwdm_conv3d_set_path(path), L.cwdm_debug_v5_grid(7)
        try:
            outs[path] = _conv_call(dtype, (B, D, H, W), a0, a1, amode, gn, w, bias)
        finally:
            L.cwdm_conv3d_set_path(prev)
            L.cwdm_debug_v5_grid(prevg)
    (o4, s4), (o5, s5) = outs[3], outs[2]
    assert torch.equal(o4.view(torch.int16), o5.view(torch.int16)), name
    # v4 sums the unrounded fp32 outputs, v5 the stored 16-bit ones (the tensor
    # the next GroupNorm normalises): sums agree to the storage rounding
    assert rel_err(s5.cpu(), s4.cpu()) < {"bf16": 2e-3, "fp16": 3e-4}[dtype_name], name


AA_CASES = [
    # name, grid (D, H, W), c0, c1, cout, rmode, grid cap -- batch 1, GroupNorm'd input.  Capped grids
    # whose sweep iterations cover whole z-rows of tiles: several ranges past the lead (2 for >= 8
    # chunks, else 3), each transformed by every workgroup and waited on through its counter
    ("aa_64_res_8wg", (32, 16, 64), 64, 0, 64, 0, 8),
    ("aa_concat_c128_16wg", (32, 16, 64), 64, 64, 128, -1, 16),
    ("aa_partial_x_res_8wg", (24, 16, 56), 64, 0, 64, 0, 8),
    ("aa_c192_cout64_4wg", (16, 8, 64), 128, 64, 64, -1, 4),
    # uncapped: one iteration past the prologue's ranges (or none)
    ("aa_concat_uncapped", (32, 32, 128), 64, 32, 128, -1, 0),
]


@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("case", AA_CASES, ids=lambda c: c[0])
def test_conv3d_v5_apply_ahead_bitexact_vs_prepass(case, dtype_name):
    """Apply-ahead (the warp-specialised conv writes the SiLU(GroupNorm) copy of
    its input itself, range by range ahead of its tile sweep, synchronised by
    per-range counters across workgroups) stores exactly what the cwdm_gn_apply
    pre-pass + the same conv store, statistics included; run twice (the last
    workgroup out re-zeroes the counters for the next launch)."""
    from cwdm_hip._lib import lib
    L = lib()
    name, grid, c0, c1, cout, rmode, cap = case
    dtype, tdt = _DTN[dtype_name]
    g = torch.Generator().manual_seed(23)
    D, H, W = grid
    cin = c0 + c1
    a0 = torch.randn(1, D, H, W, c0, generator=g).to(DEV, tdt)
    a1 = torch.randn(1, D, H, W, c1, generator=g).to(DEV, tdt) if c1 else None
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)).to(DEV)
    bias = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    gn = torch.stack([1 + 0.2 * torch.randn(1, cin, generator=g), 0.2 * torch.randn(1, cin, generator=g)],
                     -1).contiguous().to(DEV)
    res = torch.randn(1, D, H, W, cout, generator=g).to(DEV, tdt) if rmode >= 0 else None
    outs = {}
    n0 = L.cwdm_debug_v5_aa(-1)
    for aa in (0, 1, 1):
        prev, prevg, preva = L.cwdm_conv3d_set_path(2), L.cwdm_debug_v5_grid(cap), L.cwdm_debug_v5_aa(2 * aa)
        try:
            outs.setdefault(aa, []).append(_conv_call(dtype, (1, D, H, W), a0, a1, 0, gn, w, bias, res=res, rmode=rmode))
        finally:
            L.cwdm_conv3d_set_path(prev)
            L.cwdm_debug_v5_grid(prevg)
            L.cwdm_debug_v5_aa(preva)
    assert L.cwdm_debug_v5_aa(-1) - n0 == 2, f"{name}: the apply-ahead path did not run"
    (o0, s0), = outs[0]
    for o1, s1 in outs[1]:
        assert torch.equal(o0.view(torch.int16), o1.view(torch.int16)), name
        assert torch.equal(s0, s1), name


def test_conv3d_v5_apply_ahead_timeout_reported():
    """A counter wait of the apply-ahead sweep that runs out (forced here: every
    wait needs one arrival more than the grid has, 256 sleep rounds) is reported
    through the device error word (cwdm_device_status), not swallowed; the next
    normal launch is clean and equals the pre-pass conv again.  A debug grid cap
    above the CU count is clamped to what can be resident at once (the waits span
    the whole grid)."""
    from cwdm_hip._lib import check, lib
    L = lib()
    name, (D, H, W), c0, c1, cout, rmode, cap = AA_CASES[0]
    dtype, tdt = _DTN["bf16"]
    g = torch.Generator().manual_seed(29)
    a0 = torch.randn(1, D, H, W, c0, generator=g).to(DEV, tdt)
    w = (torch.randn(cout, c0, 3, 3, 3, generator=g) / math.sqrt(27 * c0)).to(DEV)
    bias = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    gn = torch.stack([1 + 0.2 * torch.randn(1, c0, generator=g), 0.2 * torch.randn(1, c0, generator=g)],
                     -1).contiguous().to(DEV)
    res = torch.randn(1, D, H, W, cout, generator=g).to(DEV, tdt)
    assert L.cwdm_device_status(1) >= 0
    assert L.cwdm_device_status(0) == 0

    def run(aa, capn):
        prev, prevg, preva = L.cwdm_conv3d_set_path(2), L.cwdm_debug_v5_grid(capn), L.cwdm_debug_v5_aa(2 * aa)
        try:
            return _conv_call(dtype, (1, D, H, W), a0, None, 0, gn, w, bias, res=res, rmode=rmode)
        finally:
            L.cwdm_conv3d_set_path(prev)
            L.cwdm_debug_v5_grid(prevg)
            L.cwdm_debug_v5_aa(preva)

    ref = run(0, cap)
    n0 = L.cwdm_debug_v5_aa(-1)
    check(L.cwdm_debug_v5_aa_timeout(1, 256))
    try:
        run(1, cap)
    finally:
        check(L.cwdm_debug_v5_aa_timeout(0, 0))
    assert L.cwdm_debug_v5_aa(-1) - n0 == 1
    st = L.cwdm_device_status(1)
    assert st & 1, f"forced apply-ahead timeout not reported (status {st})"
    assert L.cwdm_device_status(0) == 0
    # clean again, bit-identical to the pre-pass conv
    o, s = run(1, cap)
    assert L.cwdm_device_status(0) == 0
    assert torch.equal(o.view(torch.int16), ref[0].view(torch.int16))
    assert torch.equal(s, ref[1])
    # 512 tiles with the debug cap far above the CU count: the grid is clamped to what is resident
    # (unclamped, 512 workgroups would wait on each other with only one per CU resident)
    name, (D, H, W), c0, c1, cout, rmode, _ = AA_CASES[4]
    a0 = torch.randn(1, D, H, W, c0, generator=g).to(DEV, tdt)
    a1 = torch.randn(1, D, H, W, c1, generator=g).to(DEV, tdt)
    w = (torch.randn(cout, c0 + c1, 3, 3, 3, generator=g) / math.sqrt(27 * (c0 + c1))).to(DEV)
    bias = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    gn = torch.stack([1 + 0.2 * torch.randn(1, c0 + c1, generator=g), 0.2 * torch.randn(1, c0 + c1, generator=g)],
                     -1).contiguous().to(DEV)
    outs = []
    for aa, capn in ((0, 0), (1, 1 << 20)):
        prev, prevg, preva = L.cwdm_conv3d_set_path(2), L.cwdm_debug_v5_grid(capn), L.cwdm_debug_v5_aa(2 * aa)
        try:
            outs.append(_conv_call(dtype, (1, D, H, W), a0, a1, 0, gn, w, bias))
        finally:
            L.cwdm_conv3d_set_path(prev)
            L.cwdm_debug_v5_grid(prevg)
            L.cwdm_debug_v5_aa(preva)
    assert L.cwdm_device_status(0) == 0
    assert torch.equal(outs[0][0].view(torch.int16), outs[1][0].view(torch.int16))
    assert torch.equal(outs[0][1], outs[1][1])


SG_CASES = [
    # name, B, grid(out), c0, c1, cout, amode, gn, skip1x1, rmode  (16-bit; W < 32, cout % 64 == 0,
    # 32-channel K chunks: the small-grid kernel, conv3d_sg.hip, incl. its 1x1 skip mode and K split)
    ("sg16_gn_res", 1, (16, 16, 16), 64, 0, 64, 0, True, False, 0),
    ("sg16_concat_skip", 2, (4, 8, 16), 48, 16, 128, 0, True, True, -1),
    ("sg16_up_res", 1, (8, 4, 16), 32, 0, 64, 1, True, False, 1),
    ("sg8_gn_concat_res", 1, (8, 8, 8), 96, 32, 64, 0, True, False, 0),
    ("sg8_up_nogn", 2, (4, 8, 8), 32, 0, 128, 1, False, False, -1),
    ("sg8_production", 1, (8, 8, 8), 256, 256, 256, 0, True, True, -1),
    ("sg16_production_skip", 1, (16, 16, 16), 256, 256, 256, 0, True, True, -1),
    # partial bricks (r03: config 5's 28^3 / 14^3 levels and any W < 32): the last brick of
    # an axis computes zero-padded voxels and drops them (stores, residual, statistics)
    ("sg28_config5_res", 1, (28, 28, 28), 128, 0, 128, 0, True, False, 0),
    ("sg14_config5_concat_skip", 1, (14, 14, 14), 128, 128, 128, 0, True, True, -1),
    ("sg20_up_res", 1, (12, 20, 20), 64, 0, 64, 1, True, False, 1),
    ("sg12_concat_nogn", 2, (6, 10, 12), 32, 32, 64, 0, False, False, -1),
    ("sg_odd_gn_res", 1, (5, 7, 9), 32, 0, 64, 0, True, False, 0),
    ("sg14_ksplit_skip", 1, (7, 7, 14), 256, 0, 256, 0, True, True, -1),
    ("sg14_ksplit_res", 1, (7, 7, 14), 256, 0, 256, 0, True, False, 0),
    # a 1x1 skip AND a residual: not a U-Net shape; the DMA / small-grid path
    # refuses it (the skip is its residual slot) and the brick kernels run it
    ("sg_skip_plus_res_legacy", 1, (4, 8, 12), 64, 0, 64, 0, True, True, 0),
]


@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("case", SG_CASES, ids=[c[0] for c in SG_CASES])
def test_conv3d_small_grid_kernel_vs_torch(case, dtype_name):
    """The small-grid kernel (16^3 / 8^3 levels: one statistics brick x 16 output
    channels per workgroup, whole K, 16x16x32 MFMA) against F.conv3d, with the
    per-brick GroupNorm partials."""
    _run_conv_case(case, dtype_name, True)


HEAD_CASES = [((4, 4, 32), 1, 64), ((8, 8, 64), 2, 64), ((4, 8, 32), 1, 32),
              # second head: W % 16 only, partial z segments, several columns per workgroup
              ((12, 8, 48), 1, 64), ((100, 32, 64), 1, 64), ((8, 128, 128), 2, 64)]


@pytest.mark.parametrize("gen", [-1, 0, 3], ids=["head1", "head2", "head2_grid3"])
@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("grid,B,cin", HEAD_CASES)
def test_output_head_kernel_vs_torch(grid, B, cin, dtype_name, gen):
    """The narrow-output head kernels (conv3d_head.hip: GN+SiLU fused, 16x16x32
    MFMA, 8 of 16 output lanes real; the second one a z-rolling ring of halo
    planes filled by helper waves): bf16 / fp16 operands, fp32 output, vs
    F.conv3d; the two heads agree to fp32 rounding where both run."""
    from cwdm_hip._lib import lib
    if gen == -1 and grid[2] % 32:
        pytest.skip("the first head needs W % 32")
    if gen == 3 and (cin != 64 or grid[0] * grid[1] * grid[2] > 300000):
        pytest.skip("grid cap: the second head's larger cases")
    dtype, tdt = _DTN[dtype_name]
    g = torch.Generator().manual_seed(11)
    D, H, W = grid
    cout = 8
    x = torch.randn(B, cin, D, H, W, generator=g).to(tdt).float()
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)).to(tdt).float()
    bias = torch.randn(cout, generator=g) * 0.1
    scale = 1 + 0.2 * torch.randn(B, cin, generator=g)
    shift = 0.2 * torch.randn(B, cin, generator=g)
    gn = torch.stack([scale, shift], -1).contiguous()
    h = F.silu(x * scale[:, :, None, None, None] + shift[:, :, None, None, None]).to(tdt).float()
    ref = F.conv3d(h, w, bias, padding=1)
    prev = lib().cwdm_debug_head2(gen)
    try:
        out, _ = _conv_call(dtype, (B, D, H, W), _nd(x).to(DEV, tdt), None, 0, gn.to(DEV),
                            w.to(DEV), bias.to(DEV), out_f32=True, stats=False)
        if gen != -1 and grid[2] % 32 == 0:
            lib().cwdm_debug_head2(-1)
            out1, _ = _conv_call(dtype, (B, D, H, W), _nd(x).to(DEV, tdt), None, 0, gn.to(DEV),
                                 w.to(DEV), bias.to(DEV), out_f32=True, stats=False)
            # the same products; the second head adds the two 32-channel halves' sums at the end
            assert rel_err(out, out1) < 1e-5
    finally:
        lib().cwdm_debug_head2(prev)
    assert rel_err(_nc(out.float().cpu()), ref) < (1e-2 if dtype_name == "bf16" else 1e-3)


def test_gn_apply_matches_torch():
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    g = torch.Generator().manual_seed(3)
    B, V, c0, c1 = 2, 300, 24, 16
    x0 = torch.randn(B, V, c0, generator=g)
    x1 = torch.randn(B, V, c1, generator=g)
    sc = 1 + 0.3 * torch.randn(B, c0 + c1, generator=g)
    sh = 0.3 * torch.randn(B, c0 + c1, generator=g)
    gn = torch.stack([sc, sh], -1).contiguous()
    ref = F.silu(torch.cat([x0, x1], -1) * sc[:, None] + sh[:, None])
    out = torch.empty(B, V, c0 + c1, device=DEV)
    x0d, x1d, gnd = x0.to(DEV), x1.to(DEV), gn.to(DEV)
    check(lib().cwdm_gn_apply(x0d.data_ptr(), c0, x1d.data_ptr(), c1, gnd.data_ptr(), B, V, _lib.CWDM_F32,
                              out.data_ptr(), None))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-5


# (parts of source 0, parts of source 1, B, C0, C1, grid): 4 to 4096 part rows, the two sources'
# part counts different as for a decoder concat
@pytest.mark.parametrize("p0,p1,B,C0,C1,n", [(4, 4, 2, 64, 32, 8), (1024, 512, 2, 64, 128, 16),
                                             (4096, 4096, 1, 192, 0, 16), (2048, 1024, 1, 128, 64, 16),
                                             (4096, 4096, 1, 64, 0, 16), (512, 4096, 1, 384, 128, 16),
                                             (2048, 2048, 4, 128, 0, 16)])
def test_gn_finalize_matches_group_norm(p0, p1, B, C0, C1, n):
    """cwdm_gn_finalize vs F.group_norm, three calls on fresh data (no state carried
    between calls) and a repeat on the same data that must be bit-identical (fixed
    reduction order), up to the 128^3 levels' 4096 part rows and concat sources with
    different part counts."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    G = 32
    D = H = W = n
    prev = None
    for rep in range(3):
        g = torch.Generator().manual_seed(3 + rep)
        x = torch.randn(B, C0 + C1, D, H, W, generator=g) * (2 + rep) + 0.5 - rep
        # fake per-tile partials: the voxels split into p0 (source 0) / p1 (source 1) parts
        def parts_of(xs, P):
            xv = xs.reshape(B, xs.shape[1], P, -1)
            return torch.stack([xv.sum(-1), (xv ** 2).sum(-1)], -1).permute(0, 2, 1, 3).contiguous()  # B, P, C, 2
        s0 = parts_of(x[:, :C0], p0).to(DEV)
        s1 = parts_of(x[:, C0:], p1).to(DEV) if C1 else None
        gamma = (1 + 0.1 * torch.randn(C0 + C1, generator=g)).to(DEV)
        beta = (0.1 * torch.randn(C0 + C1, generator=g)).to(DEV)
        outs = []
        for _ in range(2):
            out = torch.empty(B, C0 + C1, 2, device=DEV)
            mr = torch.empty(B, G, 2, device=DEV)
            check(lib().cwdm_gn_finalize(ctypes.c_void_p(s0.data_ptr()), p0, C0,
                                         ctypes.c_void_p(s1.data_ptr()) if C1 else None, p1, C1,
                                         ctypes.c_void_p(gamma.data_ptr()), ctypes.c_void_p(beta.data_ptr()), G, B,
                                         D * H * W, 1e-5, ctypes.c_void_p(out.data_ptr()),
                                         ctypes.c_void_p(mr.data_ptr()), None))
            outs.append((out.cpu(), mr.cpu()))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        o, mr = outs[0]
        if prev is not None:
            assert not torch.equal(o, prev)
        prev = o
        y = x * o[..., 0][:, :, None, None, None] + o[..., 1][:, :, None, None, None]
        ref = F.group_norm(x, G, gamma.cpu(), beta.cpu(), eps=1e-5)
        assert rel_err(y, ref) < 1e-5
        xg = x.double().view(B, G, -1)
        assert torch.allclose(mr[..., 0].double(), xg.mean(-1), rtol=1e-5, atol=1e-6)
        assert torch.allclose(mr[..., 1].double(), 1 / torch.sqrt(xg.var(-1, unbiased=False) + 1e-5), rtol=1e-5)


@pytest.mark.parametrize("dtype_name", ["bf16", "fp16"])
@pytest.mark.parametrize("concat", [False, True], ids=["single", "concat"])
@pytest.mark.parametrize("cpg", [1, 2, 4, 8, 16])
def test_gn_fin_apply_matches_finalize_plus_apply(cpg, concat, dtype_name):
    """The fused finalize + pre-pass of the small levels (gn_fin_apply_kernel,
    GnFinFuse) == cwdm_gn_finalize + cwdm_gn_apply: the (scale, shift) and
    (mean, rstd) it writes for the backward within 1e-6, and its chunk-major
    activated output within one 16-bit ulp of the unfused pair's."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    dt, tdt = _DTN[dtype_name]
    g = torch.Generator().manual_seed(40 + cpg)
    B, C, parts, V = 2, 64, 8, 512
    c0, c1 = (32, 32) if concat else (64, 0)
    G = C // cpg
    x = (torch.randn(B, V, C, generator=g) * 1.5 + 0.3).to(tdt).float()
    xv = x.view(B, parts, V // parts, C)
    st = torch.stack([xv.sum(2), (xv ** 2).sum(2)], -1).contiguous()     # [B][P][C][2]
    s0, s1 = st[:, :, :c0].contiguous().to(DEV), st[:, :, c0:].contiguous().to(DEV)
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    x0 = x[..., :c0].contiguous().to(DEV, tdt)
    x1 = x[..., c0:].contiguous().to(DEV, tdt) if c1 else None
    L = lib()
    ss_a, mr_a = torch.empty(B, C, 2, device=DEV), torch.empty(B, G, 2, device=DEV)
    act_a = torch.empty(B, V, C, device=DEV, dtype=tdt)
    check(L.cwdm_gn_finalize(s0.data_ptr(), parts, c0, s1.data_ptr() if c1 else None, parts, c1, gamma.data_ptr(),
                             beta.data_ptr(), G, B, V, 1e-5, ss_a.data_ptr(), mr_a.data_ptr(), None))
    check(L.cwdm_gn_apply(x0.data_ptr(), c0, x1.data_ptr() if c1 else None, c1, ss_a.data_ptr(), B, V, dt,
                          act_a.data_ptr(), None))
    ss_b, mr_b = torch.empty_like(ss_a), torch.empty_like(mr_a)
    act_b = torch.empty(B, C // 16, V, 16, device=DEV, dtype=tdt)
    check(L.cwdm_debug_gn_fin_apply(s0.data_ptr(), parts, c0, s1.data_ptr() if c1 else None, parts, c1,
                                    gamma.data_ptr(), beta.data_ptr(), G, B, V, 1e-5, x0.data_ptr(),
                                    x1.data_ptr() if c1 else None, dt, ss_b.data_ptr(), mr_b.data_ptr(),
                                    act_b.data_ptr(), None))
    torch.cuda.synchronize()
    assert rel_err(ss_b, ss_a) < 1e-6
    assert rel_err(mr_b, mr_a) < 1e-6
    a = act_a.float().view(B, V, C // 16, 16).permute(0, 2, 1, 3).cpu()
    b = act_b.float().cpu()
    ulp = {"bf16": 2.0 ** -7, "fp16": 2.0 ** -10}[dtype_name]
    assert torch.all((a - b).abs() <= ulp * a.abs() + 1e-6), float((a - b).abs().max())


def test_copy3_layouts():
    from cwdm_hip import ops
    x = torch.randn(2, 24, 5, 6, 7, device=DEV)
    V = 5 * 6 * 7
    buf = torch.zeros(2, 5, 6, 7, 32, device=DEV, dtype=torch.bfloat16)
    ops.copy3(x, (24 * V, V, 1), buf[..., 8:], (V * 32, 1, 32), 2, 24, V)
    assert torch.equal(buf[..., 8:].float().cpu(), x.permute(0, 2, 3, 4, 1).to(torch.bfloat16).float().cpu())
    back = torch.empty(2, 24, 5, 6, 7, device=DEV)
    ops.copy3(buf[..., 8:], (V * 32, 1, 32), back, (24 * V, V, 1), 2, 24, V)
    assert torch.equal(back.cpu(), x.to(torch.bfloat16).float().cpu())


@pytest.mark.parametrize("dtype_name", ["fp32", "bf16", "fp16"])
def test_gn_silu_pool(dtype_name):
    from cwdm_hip import _lib
    from cwdm_hip._lib import check, lib
    dt, tdt = _DTN[dtype_name]
    g = torch.Generator().manual_seed(9)
    B, C, d = 2, 64, 4
    x = torch.randn(B, C, 2 * d, 2 * d, 2 * d, generator=g).to(tdt).float()
    scale = 1 + 0.2 * torch.randn(B, C, generator=g)
    shift = 0.2 * torch.randn(B, C, generator=g)
    gn = torch.stack([scale, shift], -1).contiguous().to(DEV)
    xd = _nd(x).to(DEV, tdt)
    oh = torch.empty(B, d, d, d, C, device=DEV, dtype=tdt)
    ox = torch.empty_like(oh)
    check(lib().cwdm_gn_silu_pool(ctypes.c_void_p(xd.data_ptr()), C, ctypes.c_void_p(gn.data_ptr()), B, d, d, d, dt,
                                  ctypes.c_void_p(oh.data_ptr()), ctypes.c_void_p(ox.data_ptr()), None))
    h = F.avg_pool3d(F.silu(x * scale[:, :, None, None, None] + shift[:, :, None, None, None]), 2)
    tol = {"fp32": 1e-5, "bf16": 1e-2, "fp16": 2e-3}[dtype_name]
    assert rel_err(_nc(oh.float().cpu()), h) < tol
    assert rel_err(_nc(ox.float().cpu()), F.avg_pool3d(x, 2)) < tol


FATS_SHIFT = [-1.2, 0.4, 0.5, 0.9, 0.3, 0.8, 1.0, 1.6]


@pytest.mark.parametrize("update,eta", [(0, 0.0), (1, 0.0), (1, 0.4)], ids=["ddpm", "ddim", "ddim_eta"])
def test_fats_per_band_sampler_step_vs_oracle(update, eta):
    """FATS: the fused step reads one coefficient row per subband (per_band):
    vs the oracle's p_sample / ddim_sample on per-band tables."""
    from oracle import diffusion as od
    from guided_diffusion import script_util
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                              timestep_respacing="ddim10", band_log_snr_shift=FATS_SHIFT)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), use_timesteps=od.space_timesteps(1000, "ddim10"),
                    band_shift=FATS_SHIFT)
    g = torch.Generator().manual_seed(9)
    B, n = 3, 6
    mo = torch.randn(B, 8, n, n, n, generator=g) * 0.5 + 0.2
    x = torch.randn(B, 8, n, n, n, generator=g)
    noise = torch.randn(B, 8, n, n, n, generator=g)
    cond = torch.zeros(B, 24, n, n, n)
    t = torch.tensor([0, 4, 9])
    sample, pred = d._epilogue(mo.to(DEV), x.to(DEV), t.to(DEV), True, None,
                               None if update else noise.to(DEV), update=update, eta=eta)
    if update:
        ref = od.ddim_sample(tab, lambda xc, tt: mo, x, t, cond, clip_denoised=True, eta=eta)
    else:
        ref = od.p_sample(tab, lambda xc, tt: mo, x, t, cond, noise)
    assert rel_err(pred, ref["pred_xstart"]) < 1e-6
    assert rel_err(sample, ref["sample"]) < 1e-6


def test_fats_per_band_prepare_batch_bitexact():
    from cwdm_hip import ops
    from oracle import diffusion as od
    from guided_diffusion import script_util
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                              band_log_snr_shift=FATS_SHIFT)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), band_shift=FATS_SHIFT)
    g = torch.Generator().manual_seed(10)
    shape = (2, 1, 8, 12, 10)
    vols = [torch.rand(shape, generator=g) for _ in range(4)]
    eps = torch.randn(shape, generator=g)
    t = torch.tensor([3, 871])
    x_in, x0 = ops.prepare_batch(*[v.to(DEV) for v in vols], eps.to(DEV), d.q_coef_table(DEV), t.to(DEV), 1000,
                                 per_band=True)
    rx0 = haar.dwt_cat(vols[0])
    reps = torch.cat(list(haar.dwt3d(eps)), 1)
    assert torch.equal(x0.cpu(), rx0)
    assert torch.equal(x_in[:, :8].cpu(), od.q_sample(tab, rx0, t, reps))


# --------------------------------------------------------------------------- channels-last Haar (WavUNetModel)
def _haar_nd(src, C, d, h, w, inverse=0, high_in=None, lll=1.0, high=1.0, all8=0, want_high=False, bias=None,
             stats=False):
    """cwdm_haar_nd through the C ABI; src/high_in channels-last device tensors."""
    from cwdm_hip import _lib
    from cwdm_hip._lib import check
    from cwdm_hip.ops import _stream
    L = _lib.lib()
    B = src.shape[0]
    dt = {torch.bfloat16: _lib.CWDM_BF16, torch.float16: _lib.CWDM_F16}.get(src.dtype, _lib.CWDM_F32)
    shape = (B, 2 * d, 2 * h, 2 * w, C) if inverse else ((B, d, h, w, 8, C) if all8 else (B, d, h, w, C))
    out = torch.empty(shape, dtype=src.dtype, device=DEV)
    ho = torch.empty((B, d, h, w, 7, C), dtype=src.dtype, device=DEV) if want_high else None
    parts = int(L.cwdm_haar_nd_parts(d, h, w))
    st = torch.empty((B, parts, C, 2), dtype=torch.float32, device=DEV) if stats else None
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    desc = _lib.HaarNdDesc(dtype=dt, B=B, d=d, h=h, w=w, C=C, inverse=inverse, src=ptr(src), high_in=ptr(high_in),
                           lll_scale=lll, high_scale=high, out=ptr(out), all8=all8, high_out=ptr(ho),
                           bias=ptr(bias), bias_bstride=C, stats=ptr(st))
    check(L.cwdm_haar_nd(ctypes.byref(desc), _stream()), "haar_nd")
    torch.cuda.synchronize()
    return out, ho, st


def _same(a, b, what=""):
    a, b = a.cpu(), b.cpu()
    if not torch.equal(a, b):
        d = (a.double() - b.double()).abs()
        raise AssertionError(f"{what}: not bit-exact, max |diff| {float(d.max()):.3e} at {int(d.argmax())}")


def _cl(x):  # NCDHW -> NDHWC
    return x.permute(0, 2, 3, 4, 1).contiguous()


@pytest.mark.parametrize("C", [32, 96])
@pytest.mark.parametrize("grid", [(3, 5, 4), (8, 8, 6)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_haar_nd_analysis_vs_oracle(C, grid, dtype):
    """Downsample(use_freq) of a ResBlock (wunet.py:120-128, :239-252): LLL x 1/3
    + emb bias and the 7 high bands, bit-exact vs the oracle DWT on the same
    (dtype-rounded) input; the GroupNorm statistics of the output vs float64."""
    d, h, w = grid
    g = torch.Generator().manual_seed(31)
    x = torch.randn(2, C, 2 * d, 2 * h, 2 * w, generator=g).to(dtype)
    bias = torch.randn(2, C, generator=g)
    third = torch.tensor(1.0 / 3.0, dtype=torch.float32)
    out, ho, st = _haar_nd(_cl(x).to(DEV), C, d, h, w, lll=float(third), want_high=True, bias=bias.to(DEV),
                           stats=True)
    bands = haar.dwt3d(x.float())
    ref = (bands[0] * third + bias[:, :, None, None, None]).to(dtype)
    _same(out, _cl(ref), "LLL")
    for k in range(7):
        _same(ho[:, :, :, :, k], _cl(bands[k + 1].to(dtype)), f"band {k + 1}")
    r64 = (bands[0] * third + bias[:, :, None, None, None]).double()
    s = st.double().sum(1).cpu()
    assert torch.allclose(s[..., 0], r64.sum((2, 3, 4)), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[..., 1], (r64 * r64).sum((2, 3, 4)), rtol=1e-5, atol=1e-4)


def test_haar_nd_all_bands_pyramid_vs_oracle():
    """WaveletDownsample input (wunet.py:141-144): cat(8 bands) / 3, band-major
    channels, bit-exact vs the oracle."""
    g = torch.Generator().manual_seed(32)
    x = torch.randn(1, 32, 8, 12, 6, generator=g)
    third = torch.tensor(1.0 / 3.0, dtype=torch.float32)
    out, _, _ = _haar_nd(_cl(x).to(DEV), 32, 4, 6, 3, lll=float(third), high=float(third), all8=1)
    ref = torch.cat([b * third for b in haar.dwt3d(x)], dim=1)
    _same(out.reshape(1, 4, 6, 3, 256), _cl(ref), "all bands")


@pytest.mark.parametrize("C", [64, 40])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_haar_nd_synthesis_vs_oracle(C, dtype):
    """Upsample(use_freq) of a ResBlock (wunet.py:62-80, :236-252): IDWT(3 h,
    skip bands) + emb bias, bit-exact vs the oracle IDWT; statistics vs float64."""
    d, h, w = 4, 3, 5
    g = torch.Generator().manual_seed(33)
    low = torch.randn(2, C, d, h, w, generator=g).to(dtype)
    highs = [torch.randn(2, C, d, h, w, generator=g).to(dtype) for _ in range(7)]
    bias = torch.randn(2, C, generator=g)
    hi = torch.stack([_cl(b) for b in highs], dim=4).contiguous()
    out, _, st = _haar_nd(_cl(low).to(DEV), C, d, h, w, inverse=1, high_in=hi.to(DEV), lll=3.0, bias=bias.to(DEV),
                          stats=True)
    rf = haar.idwt3d(low.float() * 3.0, *[b.float() for b in highs]) + bias[:, :, None, None, None]
    _same(out, _cl(rf.to(dtype)), "synthesis")
    s = st.double().sum(1).cpu()
    r64 = rf.double()
    assert torch.allclose(s[..., 0], r64.sum((2, 3, 4)), rtol=1e-5, atol=1e-4)
    assert torch.allclose(s[..., 1], (r64 * r64).sum((2, 3, 4)), rtol=1e-5, atol=1e-4)
