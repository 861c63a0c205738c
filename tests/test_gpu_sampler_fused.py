"""The sampling step fused into the U-Net's output head
(cwdm_unet_forward_step) and the in-kernel Philox noise.

* the fused step (head conv + process_xstart + posterior mean / DDIM + noise,
  x_{t-1}, pred_xstart and the mirror into the next input, all from the conv's
  accumulators) is bit-identical to cwdm_unet_forward + cwdm_sampler_step on
  the same inputs, for every branch the sampler has (START_X / EPSILON, clip,
  ancestral / DDIM, shared / per-band schedules, tensor / Philox noise);
* the Philox noise both sampler kernels draw equals oracle/philox.py (whose
  block function is pinned by Random123's known-answer vectors) to float
  rounding of the transcendental functions;
* the graph-captured loop with fused steps and Philox noise is bit-identical to
  the eager loop.
"""
import numpy as np
import pytest
import torch

from oracle import cases, philox, unet as ou

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(dtype, steps=50, respacing=""):
    from guided_diffusion import script_util
    args = script_util.run_sh_model_args(num_channels=32, channel_mult="1,2", num_res_blocks=1, num_groups=8,
                                         diffusion_steps=steps, sample_schedule="direct",
                                         timestep_respacing=respacing)
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: args[k] for k in keys}, compute_dtype=dtype)
    model.load_state_dict(ou.random_params(seed=1, **cases.C1_CFG))
    return model.to(DEV), diffusion


def _coef(T, per_band, g):
    shape = (T, 8, 8) if per_band else (T, 8)
    c = 0.2 + torch.rand(shape, generator=g)     # positive, away from 0 (coef[4] divides in DDIM)
    return c.reshape(T, -1).contiguous().to(DEV)


CASES = [
    # (mean_type, clip, update, per_band, noise)
    (0, True, 0, False, "philox"),
    (0, True, 0, False, "tensor"),
    (1, True, 0, True, "philox"),
    (0, False, 0, False, "philox"),
    (0, True, 1, False, None),
    (1, False, 1, True, None),
]


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("case", CASES)
def test_fused_step_bit_identical_to_unfused(dtype, case):
    from cwdm_hip import ops
    mean_type, clip, update, per_band, noise_kind = case
    model, _ = _model(dtype)
    B, d, h, w = 2, 32, 32, 32
    V, C, cin = d * h * w, 8, model.in_channels
    g = torch.Generator().manual_seed(31)
    T = 50
    coef = _coef(T, per_band, g)
    t = torch.tensor([T - 1, 3], device=DEV)
    t_model = t.float()
    x_t = torch.randn(B, C, d, h, w, generator=g).to(DEV)
    xin = torch.randn(B, d, h, w, cin, generator=g).to(DEV).to(model.plan.torch_dtype)
    noise = torch.randn(B, C, d, h, w, generator=g).to(DEV) if noise_kind == "tensor" else None
    seed = 0x1234_5678_9ABC if noise_kind == "philox" else None
    s = ops.ncdhw_strides(x_t)

    def run(fused_path):
        xi = xin.clone()
        out_nd = torch.full((B, d, h, w, C), float("nan"), device=DEV)
        dst = torch.empty_like(x_t)
        pred = torch.empty_like(x_t)
        kw = dict(clip_denoised=clip, pred_xstart=pred, px_s=s, mirror=xi, mr_s=(V * cin, 1, cin),
                  mean_type=mean_type, update=update, per_band=per_band, levels=1, noise_seed=seed)
        nz_s = s if noise is not None else (0, 0, 0)
        if fused_path:
            a = ops.sampler_args(out_nd, (V * C, 1, C), x_t, s, dst, s, noise, nz_s, coef, t, T, B, d, h, w, **kw)
            assert model.forward_step_ndhwc(xi, t_model, a)
            assert torch.isnan(out_nd).all()          # the fp32 model output never left the head
        else:
            model.forward_ndhwc(xi, t_model, out_nd)
            ops.sampler_step(out_nd, (V * C, 1, C), x_t, s, dst, s, noise, nz_s, coef, t, T, B, d, h, w, **kw)
        torch.cuda.synchronize()
        return dst, pred, xi

    fused, ref = run(True), run(False)
    for a, b, name in zip(fused, ref, ("x_prev", "pred_xstart", "mirror/input")):
        assert torch.equal(a, b), name
    assert torch.isfinite(fused[0]).all()


def test_forward_step_falls_back_when_not_eligible():
    """fp32 plans and grids the head kernel does not tile (W % 32) run the
    forward and cwdm_sampler_step back to back -- same results, fused False."""
    from cwdm_hip import ops
    for dtype, grid in (("fp32", (32, 32, 32)), ("bf16", (16, 16, 16))):
        model, diffusion = _model(dtype)
        B, (d, h, w) = 1, grid
        V, C, cin = d * h * w, 8, model.in_channels
        g = torch.Generator().manual_seed(2)
        coef = diffusion.coef_table(DEV)
        t = torch.tensor([7], device=DEV)
        x_t = torch.randn(B, C, d, h, w, generator=g).to(DEV)
        xin = torch.randn(B, d, h, w, cin, generator=g).to(DEV).to(model.plan.torch_dtype)
        s = ops.ncdhw_strides(x_t)
        outs = []
        for fused_path in (True, False):
            xi, out_nd, dst = xin.clone(), torch.empty(B, d, h, w, C, device=DEV), torch.empty_like(x_t)
            kw = dict(mirror=xi, mr_s=(V * cin, 1, cin), noise_seed=99)
            if fused_path:
                a = ops.sampler_args(out_nd, (V * C, 1, C), x_t, s, dst, s, None, (0, 0, 0), coef, t,
                                     diffusion.num_timesteps, B, d, h, w, **kw)
                assert not model.forward_step_ndhwc(xi, t.float(), a)
            else:
                model.forward_ndhwc(xi, t.float(), out_nd)
                ops.sampler_step(out_nd, (V * C, 1, C), x_t, s, dst, s, None, (0, 0, 0), coef, t,
                                 diffusion.num_timesteps, B, d, h, w, **kw)
            outs.append((dst, xi))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("levels", [1, 2])
def test_philox_noise_matches_oracle(levels):
    """A coefficient row (0, 0, 1) makes x_{t-1} = the noise itself: both
    sampler kernels' Philox draws vs oracle.philox (5e-5 abs: hardware
    v_log / v_sqrt / v_sin / v_cos accuracy at |z| < 5.8), and t = 0 draws none."""
    from cwdm_hip import ops
    B, d, h, w = 2, 8, 12, 16
    C = 8 if levels == 1 else 64
    T = 6
    coef = torch.zeros(T, 8)
    coef[:, 2] = 1.0
    coef = coef.to(DEV)
    seed = (0xDEADBEEF << 20) | 77
    t = torch.tensor([5, 2], device=DEV)
    zeros = torch.zeros(B, C, d, h, w, device=DEV)
    dst = torch.full_like(zeros, float("nan"))
    s = ops.ncdhw_strides(zeros)
    ops.sampler_step(zeros, s, zeros, s, dst, s, None, (0, 0, 0), coef, t, T, B, d, h, w, clip_denoised=False,
                     levels=levels, noise_seed=seed)
    want = torch.from_numpy(philox.noise_ncdhw(seed, [5, 2], B, C, d, h, w))
    got = dst.cpu()
    assert float((got - want).abs().max()) < 5e-5
    assert abs(float(got.mean())) < 0.05 and abs(float(got.std()) - 1.0) < 0.05
    t0 = torch.tensor([0, 0], device=DEV)
    ops.sampler_step(zeros, s, zeros, s, dst, s, None, (0, 0, 0), coef, t0, T, B, d, h, w, clip_denoised=False,
                     levels=levels, noise_seed=seed)
    assert torch.equal(dst, zeros)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_fused_graph_loop_equals_eager_and_is_seeded(dtype):
    """32^3 subband grid (the head kernel's tiling): every step fused, Philox
    noise.  Graph replay == eager bit for bit with the same torch seed; another
    seed gives another trajectory; a noise_fn (tensor noise) with the oracle's
    Philox draws reproduces the fused loop's first step."""
    model, diffusion = _model(dtype, steps=1000, respacing="12")
    g = torch.Generator().manual_seed(5)
    cond = torch.rand(1, 24, 32, 32, 32, generator=g).to(DEV)
    x_T = torch.randn(1, 8, 32, 32, 32, generator=g).to(DEV)

    def run(graph, seed=11, noise_fn=None):
        diffusion.use_hip_graph = graph
        torch.manual_seed(seed)
        return [o["sample"] for o in diffusion.p_sample_loop_progressive(model, x_T.shape, noise=x_T, cond=cond,
                                                                        progress=False, noise_fn=noise_fn)]

    eager, graph = run(False), run(True)
    other = run(True, seed=12)
    diffusion.use_hip_graph = True
    assert len(eager) == len(graph) == diffusion.num_timesteps
    for a, b in zip(eager, graph):
        assert torch.equal(a, b)
    assert not torch.equal(other[-1], graph[-1])
    # the loop's seed is the first draw of torch's CPU generator after manual_seed
    torch.manual_seed(11)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    ts = iter(range(diffusion.num_timesteps - 1, -1, -1))

    def oracle_noise(x):
        tt = next(ts)
        return torch.from_numpy(philox.noise_ncdhw(seed, [tt], 1, 8, 32, 32, 32)).to(DEV)

    tensor_path = run(False, noise_fn=oracle_noise)
    # the first step: the same model output, the same noise up to the hardware
    # transcendentals' ulps (x sigma_t < 1); later steps feed 16-bit inputs, where
    # one flipped rounding grows through the U-Net (bf16: 0.15 after 12 steps)
    err = float((tensor_path[0] - eager[0]).abs().max())
    assert err < 1e-4, err


@pytest.mark.parametrize("mirror", [None, "bf16", "fp16"])
@pytest.mark.parametrize("clip,mean_type,per_band,update", [(True, 0, True, 0), (False, 1, False, 0),
                                                           (True, 0, False, 1)])
def test_sampler2_staged_kernel_equals_strided(clip, mean_type, per_band, update, mirror):
    """Levels 2 with channels-last model_out / x_t / x_prev and Philox noise runs
    the LDS-staged kernel (sampler2_lds_kernel: whole 256-byte rows per 16-lane
    group); NCDHW strides run the per-voxel kernel.  Same expressions in the same
    order: bit-identical outputs, a partial last workgroup, two batch entries
    (t = 0 draws no noise), and the 16-bit mirror equal to x_prev rounded."""
    from cwdm_hip import ops
    from guided_diffusion import script_util
    shift = [-1.0 + 0.15 * k for k in range(15)] if per_band else None
    diff = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=(mean_type == 0), mode="i2i",
                                                 wavelet_levels=2, band_log_snr_shift=shift)
    g = torch.Generator().manual_seed(21)
    B, C, d, h, w = 2, 64, 5, 6, 7          # 210 voxels per entry: one partial workgroup of 256
    mo = (torch.rand(B, C, d, h, w, generator=g) * 0.4).to(DEV)
    x = torch.randn(B, C, d, h, w, generator=g).to(DEV)
    t = torch.tensor([0, 417], device=DEV)
    coef = diff.coef_table(DEV, 0.3 if update else 0.0)
    seed = 0x5151_2A2A_77
    kw = dict(clip_denoised=clip, mean_type=mean_type, update=update, per_band=diff.per_band, levels=2,
              noise_seed=seed)
    s = ops.ncdhw_strides(x)
    ref = torch.full_like(x, float("nan"))
    ops.sampler_step(mo, s, x, s, ref, s, None, (0, 0, 0), coef, t, diff.num_timesteps, B, d, h, w, **kw)
    cl = lambda z: z.permute(0, 2, 3, 4, 1).contiguous()
    V = d * h * w
    cs = (V * C, 1, C)
    out = torch.full((B, d, h, w, C), float("nan"), device=DEV)
    mir, ms = None, (0, 0, 0)
    if mirror:
        tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[mirror]
        mir = torch.zeros(B, d, h, w, 96, device=DEV, dtype=tdt)   # the U-Net input: channels 0..63 of 96
        ms = (V * 96, 1, 96)
    ops.sampler_step(cl(mo), cs, cl(x), cs, out, cs, None, (0, 0, 0), coef, t, diff.num_timesteps, B, d, h, w,
                     mirror=mir, mr_s=ms, **kw)
    assert torch.equal(out, cl(ref))
    if mirror:
        assert torch.equal(mir[..., :64], out.to(mir.dtype))
        assert mir[..., 64:].abs().max() == 0
    # the native loop's layout: channels-last model_out, channel-planar (NCDHW)
    # x_t / x_prev -> the staged kernel's planar variant; also in place
    for inplace in (False, True):
        xs = x.clone()
        outp = xs if inplace else torch.full_like(x, float("nan"))
        if mirror:
            mir.zero_()
        ops.sampler_step(cl(mo), cs, xs, s, outp, s, None, (0, 0, 0), coef, t, diff.num_timesteps, B, d, h, w,
                         mirror=mir, mr_s=ms, **kw)
        assert torch.equal(outp, ref), inplace
        if mirror:
            assert torch.equal(mir[..., :64], cl(ref).to(mir.dtype))
            assert mir[..., 64:].abs().max() == 0
