"""Volume I/O kernels against numpy / the oracle:
bit-exact (float64 order statistics and normalisation; the sample finish is
the bit-exact IDWT + clamp + mask)."""
import numpy as np
import pytest
import torch

from oracle import haar, volume as ov
from test_volume_cpu import brain_like

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape,seed", [((48, 44, 31), 0), ((17, 9, 5), 1), ((240, 240, 155), 2)])
def test_quantiles_bitexact_vs_numpy(shape, seed):
    from cwdm_hip import ops
    img = brain_like(shape, seed)
    got = ops.quantiles(torch.from_numpy(img).to(DEV), (0.001, 0.999)).cpu().numpy()
    assert got[0] == np.quantile(img, 0.001) and got[1] == np.quantile(img, 0.999)
    got = ops.quantiles(torch.from_numpy(img).to(DEV), (0.5,)).cpu().numpy()
    assert got[0] == np.quantile(img, 0.5)


def test_quantiles_edge_cases():
    from cwdm_hip import ops
    for arr in (np.array([7.0]), np.array([-3.0, 2.0]), np.zeros(1000), np.array([-0.0, 0.0, -1e-300, 1e-300]),
                np.random.default_rng(5).standard_normal(4097)):
        for q in (0.0, 0.001, 0.5, 0.999, 1.0):
            got = ops.quantiles(torch.from_numpy(arr).to(DEV), (q,)).cpu().numpy()[0]
            assert got == np.quantile(arr, q), (arr[:4], q)
    f32 = np.random.default_rng(6).random(5000).astype(np.float32)
    got = ops.quantiles(torch.from_numpy(f32).to(DEV), (0.001, 0.999)).cpu().numpy()
    f64 = f32.astype(np.float64)
    assert got[0] == np.quantile(f64, 0.001) and got[1] == np.quantile(f64, 0.999)
    with pytest.raises(IndexError):
        ops.quantiles(torch.empty(0, dtype=torch.float64, device=DEV), (0.5,))


@pytest.mark.parametrize("shape,pad_z,crop", [((48, 44, 31), 32, 4), ((240, 240, 155), 160, 8)])
def test_prepare_modality_bitexact(shape, pad_z, crop):
    from guided_diffusion import bratsloader
    img = brain_like(shape, 7)
    got = bratsloader.prepare_modality(torch.from_numpy(img).to(DEV), pad_z=pad_z, crop=crop).cpu()
    ref = ov.modality_tensor(img, pad_z=pad_z, crop=crop)
    assert got.shape == ref.shape and torch.equal(got, ref)
    cn = bratsloader.clip_and_normalize(torch.from_numpy(img).to(DEV)).cpu().numpy()
    assert np.array_equal(cn, ov.clip_and_normalize(img))


@pytest.mark.parametrize("keep_z", [155, 160])
def test_sample_finish_bitexact(keep_z):
    from guided_diffusion import bratsloader
    g = torch.Generator().manual_seed(4)
    smp = torch.randn(1, 8, 16, 16, 80, generator=g) * 0.5 + 0.3
    cond_1 = (torch.rand(1, 1, 32, 32, 160, generator=g) > 0.4).float() * torch.rand(1, 1, 32, 32, 160, generator=g)
    got = bratsloader.finish_sample(smp.to(DEV), cond_1.to(DEV), keep_z).cpu()
    ref = ov.sample_finish(smp, cond_1, keep_z)
    assert torch.equal(got, ref)


def test_front_end_to_wavelet_conditioning():
    """prepare_modality -> DWT (LLL/3) equals the oracle chain (the cond tensor of scripts/sample.py:90-97)."""
    from guided_diffusion import bratsloader
    from cwdm_hip import ops
    img = brain_like((48, 48, 30), 9)
    t = bratsloader.prepare_modality(torch.from_numpy(img).to(DEV), pad_z=32, crop=8)
    bands = ops.dwt3d(t.unsqueeze(0), lll_div3=True).cpu()
    ref = haar.dwt3d(ov.modality_tensor(img, pad_z=32, crop=8).unsqueeze(0))
    assert torch.equal(bands[0], ref[0] / 3.0)
    for k in range(1, 8):
        assert torch.equal(bands[k], ref[k])
