"""Config 5 (BASELINE.json: 2-level DWT + FATS per-band schedule; spec-only,
SURVEY.md §8(d) C5) on the GPU: the 64-channel two-level block
representation (csrc/wavelet2.hip) bit-exact against its oracle
(oracle/wavelet2.py, pinned to PyWavelets wavedecn in
tests/test_wavelet2_cpu.py), the 2-level fused sampler step, and the whole
native HIP-graph loop with FATS per-subband schedules vs the oracle loop."""
import pytest
import torch

from oracle import cases, diffusion as od, unet as ou, wavelet2 as w2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _same(a, b, what=""):
    a, b = a.cpu(), b.cpu()
    if not torch.equal(a, b):
        d = (a.double() - b.double()).abs()
        raise AssertionError(f"{what}: not bit-exact, max |diff| {float(d.max()):.3e}")


def _cl(x):
    return x.permute(0, 2, 3, 4, 1).contiguous()


@pytest.mark.parametrize("shape", [(1, 1, 4, 4, 4), (2, 1, 8, 12, 16), (1, 1, 32, 16, 24)])
def test_wavelet2_analysis_synthesis_bitexact(shape):
    from cwdm_hip import ops
    x = torch.rand(shape, generator=torch.Generator().manual_seed(3))
    ref = w2.analysis2(x)
    got = ops.wavelet2_analysis(x.to(DEV))
    _same(got, _cl(ref), "analysis")
    _same(ops.wavelet2_synthesis(got), w2.synthesis2(ref), "synthesis")
    assert (ops.wavelet2_synthesis(got).cpu() - x).abs().max() < 1e-5


def test_wavelet2_analysis_into_channel_slice_bf16():
    """Straight into channels [64, 128) of a bf16 channels-last U-Net input."""
    from cwdm_hip import ops
    x = torch.rand(2, 1, 8, 8, 12, generator=torch.Generator().manual_seed(4))
    buf = torch.zeros(2, 2, 2, 3, 256, dtype=torch.bfloat16, device=DEV)
    ops.wavelet2_analysis(x.to(DEV), out=buf, c0=64)
    _same(buf[..., 64:128], _cl(w2.analysis2(x)).to(torch.bfloat16), "bf16 slice")
    assert buf[..., :64].abs().max() == 0 and buf[..., 128:].abs().max() == 0


@pytest.mark.parametrize("clip,mean_type,per_band", [(True, 0, False), (True, 1, True), (False, 0, True)])
def test_sampler2_step_vs_oracle(clip, mean_type, per_band):
    """cwdm_sampler_step(levels=2): 2-level process_xstart + posterior + noise
    (per-channel FATS rows when per_band) vs the oracle, NCDHW strides."""
    from guided_diffusion import script_util
    shift = [-1.0 + 0.15 * k for k in range(15)] if per_band else None
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=(mean_type == 0), mode="i2i",
                                              wavelet_levels=2, band_log_snr_shift=shift)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"),
                    band_shift=w2.channel_shift(shift) if per_band else None)
    g = torch.Generator().manual_seed(5)
    B, n = 3, 3
    mo = torch.rand(B, 64, n, n, n, generator=g) * 0.4
    x = torch.randn(B, 64, n, n, n, generator=g)
    noise = torch.randn(B, 64, n, n, n, generator=g)
    t = torch.tensor([0, 17, 999])
    sample, pred = d._epilogue(mo.to(DEV), x.to(DEV), t.to(DEV), clip, None, noise.to(DEV))
    if mean_type == 0:
        x0 = mo
    else:
        x0 = od.extract(tab.sqrt_recip_alphas_cumprod, t, x.shape) * x - \
            od.extract(tab.sqrt_recipm1_alphas_cumprod, t, x.shape) * mo
    pref = w2.process_xstart2(x0) if clip else x0
    mean = od.extract(tab.posterior_mean_coef1, t, x.shape) * pref + od.extract(tab.posterior_mean_coef2, t, x.shape) * x
    mask = (t != 0).float().view(-1, 1, 1, 1, 1)
    sref = mean + mask * torch.exp(0.5 * od.extract(tab.fixed_large_log_variance, t, x.shape)) * noise
    assert rel_err(pred, pref) < 1e-6
    assert rel_err(sample, sref) < 1e-6


C5_CFG = dict(in_channels=256, model_channels=32, out_channels=64, num_res_blocks=1, channel_mult=(1, 2, 2))


def _c5_model(dtype="fp32"):
    from guided_diffusion import script_util
    return script_util.create_model(image_size=32, num_channels=32, num_res_blocks=1, channel_mult="1,2,2",
                                    attention_resolutions="", dims=3, num_groups=8, in_channels=256,
                                    out_channels=64, bottleneck_attention=False, resample_2d=False,
                                    resblock_updown=True, compute_dtype=dtype)


@pytest.mark.parametrize("sampler", ["ddpm", "ddim"])
def test_config5_fats_loop_vs_oracle(sampler):
    """The config-5 pipeline at a reduced size: 32^3 images -> 2-level
    analysis (cond straight into the channels-last model input) -> 3-level
    U-Net on the 8^3 level-2 grid (256 -> 64 channels) -> 2-level fused
    sampler step with FATS per-subband schedules, HIP-graph loop over ddim10
    tables; vs the oracle loop (process_xstart2, per-channel tables), fp32 1e-3."""
    from cwdm_hip import ops
    from guided_diffusion import script_util
    shift = [-1.5, 0.2, 0.3, 0.5, 0.2, 0.4, 0.6, 1.0] + [0.8, 1.0, 1.2, 1.0, 1.2, 1.4, 1.8]
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      timestep_respacing="ddim10", band_log_snr_shift=shift,
                                                      wavelet_levels=2)
    P = ou.random_params(seed=2, **C5_CFG)
    model = _c5_model()
    model.load_state_dict(P)
    model.to(DEV)
    vols = cases.data.brats_batch(32, seed=9, batch=1)
    cond = torch.cat([w2.analysis2(vols[k]) for k in ("t1c", "t2w", "t2f")], dim=1)
    cond_dev = torch.cat([ops.wavelet2_analysis(vols[k].to(DEV)).permute(0, 4, 1, 2, 3) for k in ("t1c", "t2w", "t2f")],
                         dim=1)
    _same(cond_dev, cond, "cond analysis")
    g = torch.Generator().manual_seed(12)
    x_T = torch.randn(1, 64, 8, 8, 8, generator=g)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), use_timesteps=od.space_timesteps(1000, "ddim10"),
                    band_shift=w2.channel_shift(shift))
    om = ou.OracleUNet(P, num_groups=8, **C5_CFG)
    if sampler == "ddim":
        out = diffusion.ddim_sample_loop(model, x_T.shape, noise=x_T.to(DEV), cond=cond_dev.contiguous())
        ref = od.ddim_sample_loop(tab, om, x_T, cond, process=w2.process_xstart2)
    else:
        noises = [torch.randn(x_T.shape, generator=g) for _ in range(10)]
        it = iter([z.to(DEV) for z in noises])
        out = diffusion.p_sample_loop(model, x_T.shape, noise=x_T.to(DEV), cond=cond_dev.contiguous(), progress=False,
                                      noise_fn=lambda x: next(it))
        ref = od.p_sample_loop(tab, om, x_T, cond, noises, process=w2.process_xstart2)
    assert rel_err(out, ref) < 1e-3
    img = ops.wavelet2_synthesis(_cl(out).contiguous())
    assert img.shape == (1, 1, 32, 32, 32)
    assert torch.allclose(img.cpu(), w2.synthesis2(ref), atol=1e-3 * float(ref.abs().max()) * 8)


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
def test_config5_graph_loop_runs_at_224(dtype):
    """The config-5 sizes themselves: 224^3 -> 56^3 x 64 channels, fp16 (the
    config's dtype) and bf16 graph loops, 3 steps; finite, and the eager loop
    agrees with the graph replay."""
    from guided_diffusion import script_util
    model = script_util.create_model(image_size=224, num_channels=64, num_res_blocks=2, channel_mult="1,2,2",
                                     attention_resolutions="", dims=3, num_groups=32, in_channels=256,
                                     out_channels=64, bottleneck_attention=False, resample_2d=False,
                                     resblock_updown=True, compute_dtype=dtype)
    # seeded non-degenerate weights: the reference initialisation zeroes out_layers.3
    # and out.2, which would make the U-Net output exactly 0
    model.load_state_dict(ou.random_params(seed=5, **C5_FULL_CFG))
    model.to(DEV)
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      timestep_respacing="3", wavelet_levels=2)
    g = torch.Generator(device=DEV).manual_seed(1)
    cond = torch.rand(1, 192, 56, 56, 56, device=DEV, generator=g)
    x_T = torch.randn(1, 64, 56, 56, 56, device=DEV, generator=g)
    outs = []
    for graph in (True, False):
        diffusion.use_hip_graph = graph
        torch.manual_seed(0)
        outs.append(diffusion.p_sample_loop(model, x_T.shape, noise=x_T, cond=cond, progress=False))
    assert torch.isfinite(outs[0]).all()
    assert float(outs[0].abs().max()) > 0
    assert torch.equal(outs[0], outs[1])


C5_FULL_CFG = dict(in_channels=256, model_channels=64, out_channels=64, num_res_blocks=2, channel_mult=(1, 2, 2))
C5_SHIFT = [-1.5, 0.2, 0.3, 0.5, 0.2, 0.4, 0.6, 1.0] + [0.8, 1.0, 1.2, 1.0, 1.2, 1.4, 1.8]
_C5_REF = {}


def _c5_full_case():
    """224^3 phantoms -> 2-level analysis (cond: 3 x 64 channels on the 56^3 grid),
    x_t and the step noise, seeded; the oracle step (cached: four dtypes use it)."""
    if not _C5_REF:
        from oracle import data
        g = torch.Generator().manual_seed(31)
        cond = torch.cat([w2.analysis2(data.phantom(224, seed=60 + k)) for k in range(3)], dim=1)
        x_t = torch.randn(1, 64, 56, 56, 56, generator=g)
        noise = torch.randn(1, 64, 56, 56, 56, generator=g)
        P = ou.random_params(seed=5, **C5_FULL_CFG)
        tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), band_shift=w2.channel_shift(C5_SHIFT))
        torch.set_num_threads(16)
        with torch.no_grad():
            ref = od.p_sample(tab, ou.OracleUNet(P, num_groups=32, **C5_FULL_CFG), x_t, torch.tensor([_C5_T]), cond,
                              noise, process=w2.process_xstart2)
        _C5_REF.update(P=P, cond=cond, x_t=x_t, noise=noise, ref=ref)
    return _C5_REF


_C5_T = 480


@pytest.mark.parametrize("dtype", ["fp32", "fp32x", "fp16", "bf16"])
def test_config5_step_at_224_vs_oracle(dtype):
    """Config 5 at its own size with non-degenerate weights: one denoising step
    of the native loop (3-level U-Net 256 -> 64 channels, mc 64, mult 1,2,2,
    2 res blocks, on the 56^3 level-2 grid of 224^3 images; the 2-level fused
    sampler with FATS per-subband rows) against the CPU oracle's p_sample with
    process_xstart2.  fp32 and the accurate fast mode fp32x within 1e-3 (fp32x
    runs the split-bf16 warp-specialised conv at 56^3); fp16 (the config's dtype)
    and bf16 run the 16-bit 56^3 v5 / 28^3 v4 / 14^3 small-grid convs, bounded
    at their measured rounding error."""
    from guided_diffusion import script_util
    c = _c5_full_case()
    model = script_util.create_model(image_size=224, num_channels=64, num_res_blocks=2, channel_mult="1,2,2",
                                     attention_resolutions="", dims=3, num_groups=32, in_channels=256,
                                     out_channels=64, bottleneck_attention=False, resample_2d=False,
                                     resblock_updown=True, compute_dtype=dtype)
    model.load_state_dict(c["P"])
    model.to(DEV)
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      band_log_snr_shift=C5_SHIFT, wavelet_levels=2)
    it = iter([c["noise"].to(DEV)])
    loop = diffusion._native_loop(model, c["x_t"].to(DEV), [_C5_T], c["cond"].to(DEV).contiguous(), True,
                                  noise_fn=lambda x: next(it), graph=False)
    out = next(loop)
    sample, pred = out["sample"].cpu(), out["pred_xstart"].cpu()
    ref = c["ref"]
    l2 = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())  # noqa: E731
    e = {"pred_max": rel_err(pred, ref["pred_xstart"]), "sample_max": rel_err(sample, ref["sample"]),
         "pred_l2": l2(pred, ref["pred_xstart"]), "sample_l2": l2(sample, ref["sample"])}
    print(f"config 5 at 224^3, {dtype} step vs oracle:", {k: f"{v:.3e}" for k, v in e.items()})
    assert torch.isfinite(sample).all() and float(ref["pred_xstart"].abs().max()) > 0
    if dtype in ("fp32", "fp32x"):
        assert e["pred_max"] < 1e-3 and e["sample_max"] < 1e-3, e
    else:
        # 16-bit activations: bounded like the config-2 full-size half step
        # (test_gpu_fullsize.test_fullsize_half_step_close_to_fp32)
        bound = {"fp16": 1e-2, "bf16": 6e-2}[dtype]
        assert e["pred_l2"] < bound and e["sample_l2"] < bound, e


@pytest.mark.parametrize("per_band", [False, True])
def test_prepare_batch2_bitexact_vs_oracle(per_band):
    """cwdm_prepare_batch2 (config-5 training front end): x0 = analysis2(target),
    the three conditions' analyses and q_sample with the noise image's unscaled
    2-level transform (per-channel FATS rows when per_band), bit for bit."""
    from cwdm_hip import ops
    from guided_diffusion import script_util
    shift = [-1.0 + 0.15 * k for k in range(15)] if per_band else None
    d = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i", wavelet_levels=2,
                                              band_log_snr_shift=shift)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"),
                    band_shift=w2.channel_shift(shift) if per_band else None)
    g = torch.Generator().manual_seed(14)
    shape = (2, 1, 8, 12, 16)
    vols = [torch.rand(shape, generator=g) for _ in range(4)]
    eps = torch.randn(shape, generator=g)
    t = torch.tensor([0, 613])
    x_in, x0 = ops.prepare_batch2(*[v.to(DEV) for v in vols], eps.to(DEV), d.q_coef_table(DEV), t.to(DEV), 1000,
                                  per_band=per_band)
    rx0 = w2.analysis2(vols[0])
    _same(x0, rx0, "x0")
    _same(x_in[:, 64:], torch.cat([w2.analysis2(v) for v in vols[1:]], 1), "cond")
    _same(x_in[:, :64], od.q_sample(tab, rx0, t, w2.analysis2(eps, scale=False)), "x_t")


def test_config5_training_step_vs_oracle():
    """Config-5 training (levels = 2): training_losses -> loss.backward() on the
    native U-Net (256 -> 64 channels, 3 levels, 8^3 level-2 grid from 32^3
    volumes, FATS per-channel rows) vs the oracle's loss and autograd, fp32."""
    from guided_diffusion import script_util
    shift = [-1.5, 0.2, 0.3, 0.5, 0.2, 0.4, 0.6, 1.0] + [0.8, 1.0, 1.2, 1.0, 1.2, 1.4, 1.8]
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      band_log_snr_shift=shift, wavelet_levels=2)
    P = ou.random_params(seed=21, **C5_CFG)
    model = _c5_model()
    model.load_state_dict(P)
    model.to(DEV)
    vols = {k: v.to(DEV) for k, v in cases.data.brats_batch(32, seed=5, batch=2).items()}
    t = torch.tensor([11, 802], device=DEV)
    noise = torch.randn(2, 1, 32, 32, 32, generator=torch.Generator().manual_seed(8)).to(DEV)
    terms, out, out_img = diffusion.training_losses(model, vols, t, mode="i2i", contr="t1n", noise=noise)
    assert terms["mse_wav"].shape == (64,)
    terms["mse_wav"].mean().backward()
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), band_shift=w2.channel_shift(shift))
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}

    def om(x, tt, **kw):
        return ou.unet_forward(Pr, x, tt, num_groups=8, **C5_CFG)
    rterms, rout, rimg = od.training_losses(tab, om, {k: v.cpu() for k, v in vols.items()}, t.cpu(), noise.cpu(),
                                            contr="t1n", levels=2)
    rloss = rterms["mse_wav"].mean()
    rloss.backward()
    assert rel_err(out.detach(), rout.detach()) < 1e-3
    assert rel_err(out_img, rimg.detach()) < 1e-3
    assert abs(float(terms["mse_wav"].mean()) - float(rloss)) / float(rloss) < 1e-4
    for n, p in model.named_parameters():
        err = float((p.grad.double().cpu() - Pr[n].grad.double()).norm() / Pr[n].grad.double().norm().clamp_min(1e-30))
        assert err < 1e-3, (n, err)


def test_config5_fp16_loop_close_to_oracle():
    """Config 5 as specified, fp16 (BASELINE.json config 5): the reduced-size
    FATS pipeline of test_config5_fats_loop_vs_oracle (32^3 images, 2-level
    analysis, 3-level U-Net, 10 ddim10 DDPM steps) with the U-Net in fp16
    against the fp32 oracle loop.  Measured bound."""
    from cwdm_hip import ops
    from guided_diffusion import script_util
    shift = [-1.5, 0.2, 0.3, 0.5, 0.2, 0.4, 0.6, 1.0] + [0.8, 1.0, 1.2, 1.0, 1.2, 1.4, 1.8]
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      timestep_respacing="ddim10", band_log_snr_shift=shift,
                                                      wavelet_levels=2)
    P = ou.random_params(seed=2, **C5_CFG)
    outs = {}
    vols = cases.data.brats_batch(32, seed=9, batch=1)
    cond = torch.cat([w2.analysis2(vols[k]) for k in ("t1c", "t2w", "t2f")], dim=1)
    g = torch.Generator().manual_seed(12)
    x_T = torch.randn(1, 64, 8, 8, 8, generator=g)
    noises = [torch.randn(x_T.shape, generator=g) for _ in range(10)]
    for dt in ("fp16", "bf16"):
        model = _c5_model(dt)
        model.load_state_dict(P)
        model.to(DEV)
        it = iter([z.to(DEV) for z in noises])
        outs[dt] = diffusion.p_sample_loop(model, x_T.shape, noise=x_T.to(DEV), cond=cond.to(DEV).contiguous(),
                                           progress=False, noise_fn=lambda x: next(it)).cpu()
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), use_timesteps=od.space_timesteps(1000, "ddim10"),
                    band_shift=w2.channel_shift(shift))
    ref = od.p_sample_loop(tab, ou.OracleUNet(P, num_groups=8, **C5_CFG), x_T, cond, noises,
                           process=w2.process_xstart2)
    errs = {dt: float((o.double() - ref.double()).norm() / ref.double().norm()) for dt, o in outs.items()}
    print("config-5 10-step loop vs fp32 oracle, rel L2:", errs)
    # measured (r03): fp16 1.76e-2, bf16 1.19e-1 -- the fp16 loop is ~7x closer to fp32
    assert errs["fp16"] < 3e-2, errs
    assert errs["fp16"] < 0.5 * errs["bf16"], errs


def test_config5_fp16_training_gradients_with_loss_scaling():
    """Config-5 training in fp16: the MSE gradient of the 64-channel output is
    far below fp16's normal range, so training scales the loss (amp.GradScaler,
    the reference's use_fp16 path, train_util.py:84-87, :457-458) and unscales
    the flat gradient before AdamW.  Scaled fp16 gradients vs the fp32 oracle's
    autograd."""
    from cwdm_hip.optim import FlatAdamW
    from guided_diffusion import script_util
    shift = [-1.5, 0.2, 0.3, 0.5, 0.2, 0.4, 0.6, 1.0] + [0.8, 1.0, 1.2, 1.0, 1.2, 1.4, 1.8]
    diffusion = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                      band_log_snr_shift=shift, wavelet_levels=2)
    P = ou.random_params(seed=21, **C5_CFG)
    model = _c5_model("fp16")
    model.load_state_dict(P)
    model.to(DEV)
    vols = {k: v.to(DEV) for k, v in cases.data.brats_batch(32, seed=5, batch=2).items()}
    t = torch.tensor([11, 802], device=DEV)
    noise = torch.randn(2, 1, 32, 32, 32, generator=torch.Generator().manual_seed(8)).to(DEV)
    terms, out, _ = diffusion.training_losses(model, vols, t, mode="i2i", contr="t1n", noise=noise)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 16)
    scaler.scale(terms["mse_wav"].mean()).backward()
    opt = FlatAdamW(model, lr=1e-5, weight_decay=0.0)
    scaler.unscale_(opt)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), band_shift=w2.channel_shift(shift))
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}

    def om(x, tt, **kw):
        return ou.unet_forward(Pr, x, tt, num_groups=8, **C5_CFG)
    rterms, rout, _ = od.training_losses(tab, om, {k: v.cpu() for k, v in vols.items()}, t.cpu(), noise.cpu(),
                                         contr="t1n", levels=2)
    rterms["mse_wav"].mean().backward()
    assert rel_err(out.detach(), rout.detach()) < 1e-2
    worst = {n: float((p.grad.double().cpu() - Pr[n].grad.double()).norm() / Pr[n].grad.double().norm().clamp_min(1e-30))
             for n, p in model.named_parameters()}
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:5]
    print("fp16 + loss scaling, worst gradients vs fp32 oracle:", top)
    assert top[0][1] < 3e-2, top
    before = model.flat_params.clone()
    scaler.step(opt)
    scaler.update()
    assert not torch.equal(before, model.flat_params)    # finite gradients: the step was taken
