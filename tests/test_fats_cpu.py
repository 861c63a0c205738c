"""FATS (frequency-adaptive per-subband schedules; by specification, see
guided_diffusion/fats.py) on CPU: the product's float64 tables equal the
oracle's restatement, respacing keeps them consistent, zero shifts reproduce
the shared schedule, and the shifts equalise the effective SNR."""
import numpy as np
import torch

from oracle import diffusion as od

SHIFT = np.array([-1.2, 0.4, 0.5, 0.9, 0.3, 0.8, 1.0, 1.6])


def _product(respacing=""):
    from guided_diffusion import script_util
    return script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                                 timestep_respacing=respacing, band_log_snr_shift=SHIFT)


def test_per_band_tables_equal_oracle():
    d = _product()
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), band_shift=SHIFT)
    assert d.alphas_cumprod.shape == (1000, 8)
    for name in ("alphas_cumprod", "alphas_cumprod_prev", "posterior_mean_coef1", "posterior_mean_coef2",
                 "sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod", "posterior_variance"):
        assert np.array_equal(getattr(d, name), getattr(tab, name)), name
    v, _ = d._fixed_variance()
    assert np.array_equal(v, tab.fixed_large_variance)
    # each band is a valid monotone schedule with the requested log-SNR offset
    lam = np.log(d.base_alphas_cumprod / (1 - d.base_alphas_cumprod))
    lam_k = np.log(d.alphas_cumprod / (1 - d.alphas_cumprod))
    assert np.allclose(lam_k - lam[:, None], SHIFT[None, :], atol=1e-6)
    assert (np.diff(d.alphas_cumprod, axis=0) < 0).all()


def test_respaced_per_band_tables_equal_oracle():
    d = _product("ddim10")
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"), use_timesteps=od.space_timesteps(1000, "ddim10"),
                    band_shift=SHIFT)
    assert d.num_timesteps == 10 and d.alphas_cumprod.shape == (10, 8)
    assert np.allclose(d.alphas_cumprod, tab.alphas_cumprod, rtol=1e-12, atol=0)
    assert np.allclose(d.posterior_mean_coef1, tab.posterior_mean_coef1, rtol=1e-10, atol=1e-15)
    # a kept step keeps its per-band acp: respacing commutes with the band offsets
    full = _product()
    assert np.allclose(d.alphas_cumprod, full.alphas_cumprod[d.timestep_map], rtol=1e-12)


def test_zero_shift_is_the_shared_schedule():
    from guided_diffusion import script_util
    base = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i")
    z = script_util.create_gaussian_diffusion(steps=1000, predict_xstart=True, mode="i2i",
                                              band_log_snr_shift=np.zeros(8))
    assert np.allclose(z.alphas_cumprod, base.alphas_cumprod[:, None], rtol=1e-12)
    assert np.allclose(z.posterior_mean_coef2, base.posterior_mean_coef2[:, None], rtol=1e-9)


def test_shifts_equalise_effective_snr():
    from guided_diffusion import fats
    g = torch.Generator().manual_seed(0)
    scale = torch.tensor([1.0, 0.2, 0.2, 0.05, 0.2, 0.05, 0.05, 0.01])
    x0 = torch.randn(2, 8, 6, 6, 6, generator=g) * scale.view(1, 8, 1, 1, 1)
    e = fats.band_energy(x0)
    sh = fats.band_log_snr_shifts(e, max_shift=10.0)
    assert abs(sh.sum()) < 1e-9 and sh[0] < 0 and sh[7] > 0
    d = fats.create_fats_diffusion(energy=e, max_shift=10.0, steps=1000, predict_xstart=True, mode="i2i")
    snr = d.alphas_cumprod / (1 - d.alphas_cumprod) * e[None, :]
    spread = np.log(snr).max(axis=1) - np.log(snr).min(axis=1)
    assert spread.max() < 1e-6          # equal effective SNR in every band at every t
