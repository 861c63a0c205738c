"""Shared parity cases (TEST INFRASTRUCTURE ONLY): the BASELINE.json config 1
plumbing case and a few seeded inputs used by tests/ and the golden fixtures."""
import torch

from . import data, diffusion, haar, unet

C1_CFG = dict(in_channels=32, model_channels=32, out_channels=8, num_res_blocks=1, channel_mult=(1, 2))
C1_GROUPS = 8


def c1_inputs(size=64):
    """Config 1: one 64^3 synthetic volume set, tiny UNet with seeded non-zero
    weights (seed 1), 2-step 'sampled' schedule, noise from seed 2."""
    vols = data.brats_batch(size, seed=0, batch=1)
    cond = torch.cat([haar.dwt_cat(vols[k]) for k in ("t1c", "t2w", "t2f")], dim=1)  # contr = t1n
    n = size // 2
    g = torch.Generator().manual_seed(2)
    x_T = torch.randn(1, 8, n, n, n, generator=g)
    step_noises = [torch.randn(1, 8, n, n, n, generator=g) for _ in range(2)]
    params = unet.random_params(seed=1, **C1_CFG)
    return vols, cond, x_T, step_noises, params


def c1_run(size=64):
    vols, cond, x_T, step_noises, params = c1_inputs(size)
    tab = diffusion.Tables(diffusion.beta_schedule("linear", 2, "sampled"))
    model = unet.OracleUNet(params, num_groups=C1_GROUPS, **C1_CFG)
    sample = diffusion.p_sample_loop(tab, model, x_T, cond, step_noises)
    img = haar.idwt_split(sample).clamp(0, 1)
    img[vols["t1c"] == 0] = 0
    return sample, img
