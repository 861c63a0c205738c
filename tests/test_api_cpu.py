"""Host-side API mirror: factories, state_dict contract, diffusion tables and
error conventions (no GPU needed; no kernel launched)."""
import numpy as np
import pytest
import torch

from oracle import diffusion as od
from oracle import unet as ou


def _model_and_diffusion(**kw):
    from guided_diffusion import script_util
    args = script_util.run_sh_model_args(**kw)
    keys = script_util.model_and_diffusion_defaults().keys()
    return script_util.create_model_and_diffusion(**{k: args[k] for k in keys})


def test_run_sh_factory_state_dict_matches_reference_contract():
    model, diffusion = _model_and_diffusion()
    sd = model.state_dict()
    want = ou.param_shapes()
    assert list(sd.keys()) == [n for n, _ in want]
    assert all(tuple(sd[n].shape) == tuple(s) for n, s in want)
    # zero_module on out_layers.3 and out.2 (unet.py:259-261, :724)
    assert torch.count_nonzero(sd["out.2.weight"]) == 0
    assert torch.count_nonzero(sd["input_blocks.1.0.out_layers.3.weight"]) == 0
    assert torch.all(sd["input_blocks.1.0.in_layers.0.weight"] == 1)
    assert diffusion.num_timesteps == 1000


def test_state_dict_roundtrip_with_oracle_params():
    model, _ = _model_and_diffusion(num_channels=32, channel_mult="1,2", num_res_blocks=1, num_groups=8)
    P = ou.random_params(seed=3, model_channels=32, channel_mult=(1, 2), num_res_blocks=1)
    model.load_state_dict(P)
    for k, v in model.state_dict().items():
        assert torch.equal(v, P[k])


@pytest.mark.parametrize("T,sched,resp", [(1000, "direct", ""), (10, "sampled", ""), (1000, "direct", "ddim50"),
                                          (100, "direct", "10,20")])
def test_spaced_tables_match_oracle(T, sched, resp):
    from guided_diffusion import script_util
    d = script_util.create_gaussian_diffusion(steps=T, predict_xstart=True, sample_schedule=sched,
                                              timestep_respacing=resp, mode="i2i")
    use = od.space_timesteps(T, resp) if resp else range(T)
    tab = od.Tables(od.beta_schedule("linear", T, sched), sorted(use))
    assert d.timestep_map == tab.timestep_map
    for name in ("betas", "alphas_cumprod", "posterior_mean_coef1", "posterior_mean_coef2", "posterior_variance",
                 "posterior_log_variance_clipped", "sqrt_recip_alphas_cumprod"):
        np.testing.assert_array_equal(getattr(d, name), getattr(tab, name))
    coef = d.coef_table("cpu")
    assert coef.shape == (d.num_timesteps, 8)
    np.testing.assert_allclose(coef[:, 2].numpy(),
                               torch.exp(0.5 * torch.from_numpy(tab.fixed_large_log_variance).float()).numpy(),
                               rtol=0, atol=0)
    for i in (0, d.num_timesteps - 1):
        assert d._model_timestep(i) == float(tab.timestep_map[i])


def test_direct_below_20_asserts_like_reference():
    from guided_diffusion import script_util
    with pytest.raises(AssertionError):
        script_util.create_gaussian_diffusion(steps=10, sample_schedule="direct")


def test_unsupported_configs_raise():
    from guided_diffusion.unet import UNetModel
    with pytest.raises(NotImplementedError):
        UNetModel(64, 32, 64, 8, 2, (4,), dims=3, resblock_updown=True, bottleneck_attention=False,
                  resample_2d=False)
    with pytest.raises(NotImplementedError):
        UNetModel(64, 32, 64, 8, 2, (), dims=2, resblock_updown=True, bottleneck_attention=False)


def test_cpu_tensors_fail_loudly():
    model, diffusion = _model_and_diffusion(num_channels=32, channel_mult="1,2", num_res_blocks=1, num_groups=8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        model(torch.zeros(1, 32, 16, 16, 16), torch.zeros(1, dtype=torch.long))
    from DWT_IDWT.DWT_IDWT_layer import DWT_3D
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        DWT_3D("haar")(torch.zeros(1, 1, 4, 4, 4))
    with pytest.raises(NotImplementedError):
        DWT_3D("db2")


def test_extract_into_tensor_index_error():
    from guided_diffusion.gaussian_diffusion import _extract_into_tensor
    with pytest.raises(IndexError):
        _extract_into_tensor(np.ones(10), torch.tensor([10]), (1, 1))
