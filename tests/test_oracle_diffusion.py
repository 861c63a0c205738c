"""Pin the oracle's schedules / tables by closed-form float64 recomputation."""
import numpy as np
import pytest

from oracle import diffusion as od


@pytest.mark.parametrize("T", [20, 50, 100, 1000])
def test_direct_schedule(T):
    b = od.beta_schedule("linear", T, "direct")
    s = 1000.0 / T
    assert b.dtype == np.float64 and len(b) == T
    assert b[0] == pytest.approx(1e-4 * s, rel=1e-12)
    assert b[-1] == pytest.approx(0.02 * s, rel=1e-12)
    assert np.allclose(np.diff(b), (0.02 * s - 1e-4 * s) / (T - 1))


@pytest.mark.parametrize("T", [2, 10, 50, 1000])
def test_sampled_schedule(T):
    b = od.beta_schedule("linear", T, "sampled")
    full = np.cumprod(1 - np.linspace(1e-4, 0.02, 1000))
    idx = np.linspace(0, 999, T).astype(int)
    acp = np.cumprod(1 - b)
    # clipping only binds at the ends; away from the clip the product matches the 1000-step curve
    unclipped = (b > 1e-4) & (b < 0.999)
    assert np.allclose(acp[unclipped.cumprod().astype(bool)], full[idx][unclipped.cumprod().astype(bool)])
    assert b.min() >= 1e-4 and b.max() <= 0.999


def test_sampled_T2_is_the_C1_schedule():
    b = od.beta_schedule("linear", 2, "sampled")
    assert b[0] == pytest.approx(1e-4) and b[1] == pytest.approx(0.999)


def test_direct_below_20_fails_beta_assert():
    with pytest.raises(AssertionError):
        od.Tables(od.beta_schedule("linear", 10, "direct"))


def test_tables_closed_form():
    tab = od.Tables(od.beta_schedule("linear", 1000, "direct"))
    acp = np.cumprod(1 - tab.betas)
    prev = np.append(1.0, acp[:-1])
    assert np.allclose(tab.posterior_mean_coef1, tab.betas * np.sqrt(prev) / (1 - acp))
    assert np.allclose(tab.posterior_mean_coef2, (1 - prev) * np.sqrt(1 - tab.betas) / (1 - acp))
    pv = tab.betas * (1 - prev) / (1 - acp)
    assert np.allclose(tab.fixed_large_variance, np.append(pv[1], tab.betas[1:]))
    assert tab.posterior_mean_coef1[0] == pytest.approx(1.0)  # x0 is returned exactly at t=0


def test_space_timesteps():
    assert od.space_timesteps(1000, "ddim50") == set(range(0, 1000, 20))
    assert od.space_timesteps(300, [10, 15, 20]) == od.space_timesteps(300, "10,15,20")
    assert len(od.space_timesteps(300, [10, 15, 20])) == 45
    with pytest.raises(ValueError):
        od.space_timesteps(10, [20])


def test_respaced_betas_preserve_alphas_cumprod():
    base = od.Tables(od.beta_schedule("linear", 1000, "direct"))
    use = sorted(od.space_timesteps(1000, "ddim50"))
    sp = od.Tables(od.beta_schedule("linear", 1000, "direct"), use)
    assert sp.num_timesteps == 50 and sp.timestep_map == use
    assert np.allclose(sp.alphas_cumprod, base.alphas_cumprod[use])
