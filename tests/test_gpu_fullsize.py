"""Parity at BASELINE.json's full size (config 2: 256^3 images, 128^3
subbands, the 81.5 M-parameter production U-Net): the wavelets bit-exact,
one whole denoising step (native channels-last loop: U-Net + fused epilogue)
against the CPU oracle within 1e-3 (fp32), and the bf16 throughput mode
against fp32 at the same size."""
import pytest
import torch

from oracle import data, diffusion as od, haar, unet as ou

pytestmark = pytest.mark.gpu
DEV = "cuda"
N = 128


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_fullsize_haar_bitexact_and_roundtrip():
    from cwdm_hip import ops
    x = data.phantom(2 * N, seed=3)                      # (1, 1, 256, 256, 256)
    bands = ops.dwt3d(x.to(DEV)).cpu()
    ref = haar.dwt3d(x)
    for k in range(8):
        assert torch.equal(bands[k], ref[k]), k
    v = N ** 3
    rec = ops.idwt3d(bands.to(DEV).contiguous(), (v, v, v, 1), 1, 1, N, N, N).cpu()
    assert torch.equal(rec, haar.idwt3d(*ref))
    assert float((rec - x).abs().max()) < 1e-5
    # Parseval (orthonormal Haar): energy is preserved
    e_img, e_b = float((x.double() ** 2).sum()), float((bands.double() ** 2).sum())
    assert abs(e_img - e_b) / e_img < 1e-6


def _production(dtype, P):
    from guided_diffusion import script_util
    args = script_util.run_sh_model_args(diffusion_steps=1000, sample_schedule="direct")
    keys = script_util.model_and_diffusion_defaults().keys()
    model, diffusion = script_util.create_model_and_diffusion(**{k: args[k] for k in keys}, compute_dtype=dtype)
    diffusion.mode = "i2i"
    model.load_state_dict(P)
    return model.to(DEV), diffusion


def _step_inputs():
    g = torch.Generator().manual_seed(21)
    cond = torch.cat([haar.dwt_cat(data.phantom(2 * N, seed=30 + k)) for k in range(3)], dim=1)  # (1, 24, N^3)
    x_t = torch.randn(1, 8, N, N, N, generator=g)
    noise = torch.randn(1, 8, N, N, N, generator=g)
    return cond, x_t, noise


def _native_step(model, diffusion, cond, x_t, noise, t):
    it = iter([noise.to(DEV)])
    loop = diffusion._native_loop(model, x_t.to(DEV), [t], cond.to(DEV), True, noise_fn=lambda x: next(it),
                                  graph=False)
    out = next(loop)
    return out["sample"].cpu(), out["pred_xstart"].cpu()


def test_fullsize_denoising_step_fp32_vs_oracle():
    P = ou.random_params(seed=5)
    model, diffusion = _production("fp32", P)
    cond, x_t, noise = _step_inputs()
    t = 640
    sample, pred = _native_step(model, diffusion, cond, x_t, noise, t)
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"))
    torch.set_num_threads(16)
    with torch.no_grad():
        ref = od.p_sample(tab, ou.OracleUNet(P), x_t, torch.tensor([t]), cond, noise)
    assert rel_err(pred, ref["pred_xstart"]) < 1e-3
    assert rel_err(sample, ref["sample"]) < 1e-3


def test_fullsize_bf16_step_close_to_fp32():
    P = ou.random_params(seed=5)
    cond, x_t, noise = _step_inputs()
    outs = {}
    for dt in ("fp32", "bf16"):
        model, diffusion = _production(dt, P)
        outs[dt] = _native_step(model, diffusion, cond, x_t, noise, 640)
        del model
        torch.cuda.empty_cache()
    # bf16 is the throughput mode (SURVEY.md §7 iii: judged on a looser,
    # documented bound): relative L2 over the 16.8 M outputs, and the max-norm
    # (a few outliers among 16.8 M values after 81 M bf16 parameters)
    for k in (0, 1):
        a, b = outs["bf16"][k].double(), outs["fp32"][k].double()
        l2 = float((a - b).norm() / b.norm())
        print(f"bf16 vs fp32 full size, output {k}: rel L2 {l2:.3e}, rel max {rel_err(a, b):.3e}")
        assert l2 < 4e-2, l2
        assert rel_err(a, b) < 0.25
