"""Volume I/O either side of the path, CPU side: the
oracle restatement against numpy (the reference's own arithmetic for this
step) and the quantile-rank bookkeeping the C ABI is driven with."""
import numpy as np
import pytest
import torch

from oracle import haar, volume as ov


def brain_like(shape, seed):
    """Zero background + a positive ellipsoid of heavy-tailed intensities (the
    shape of a decoded BraTS modality before clip_and_normalize)."""
    rng = np.random.default_rng(seed)
    X, Y, Z = shape
    x, y, z = np.meshgrid(np.linspace(-1, 1, X), np.linspace(-1, 1, Y), np.linspace(-1, 1, Z), indexing="ij")
    mask = (x / 0.8) ** 2 + (y / 0.9) ** 2 + (z / 0.7) ** 2 <= 1
    img = np.where(mask, rng.gamma(2.0, 300.0, size=shape), 0.0)
    img[tuple(rng.integers(0, s, 5) for s in shape)] = 5e4   # a few hot voxels the 0.999 clip removes
    return img


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 8928000, 240 * 240 * 155])
def test_quantile_ranks_match_numpy_linear(n):
    from cwdm_hip import ops
    for q in (0.0, 0.001, 0.25, 0.5, 0.999, 1.0):
        (lo, hi), (g,) = ops.quantile_ranks(n, [q])
        a = np.arange(n, dtype=np.float64) * 3.0 + 1.0   # sorted, distinct: order statistic k = 3 k + 1
        expect = np.quantile(a, q)
        va, vb = a[lo], a[hi]
        d = vb - va
        got = va + d * g if g < 0.5 else vb - d * (1 - g)
        assert got == expect, (n, q, got, expect)


def test_quantile_ranks_reject_bad_q():
    from cwdm_hip import ops
    with pytest.raises(ValueError):
        ops.quantile_ranks(10, [1.5])


def test_oracle_modality_tensor_shape_and_range():
    img = brain_like((40, 36, 31), 0)
    t = ov.modality_tensor(img, pad_z=32, crop=4)
    assert t.shape == (1, 32, 28, 32) and t.dtype == torch.float32
    assert float(t.min()) == 0.0 and float(t.max()) <= 1.0
    assert torch.all(t[..., 31:] == 0)
    ref = torch.tensor(ov.clip_and_normalize(img)).float()[4:-4, 4:-4, :]
    assert torch.equal(t[0, :, :, :31], ref)


def test_oracle_sample_finish_roundtrip():
    g = torch.Generator().manual_seed(3)
    img = torch.rand(2, 1, 8, 6, 10, generator=g)
    bands = haar.dwt3d(img)
    smp = torch.cat([bands[0] / 3.0] + list(bands[1:]), dim=1)
    mask = (torch.rand(2, 1, 8, 6, 10, generator=g) > 0.3).float()
    out = ov.sample_finish(smp, mask, 9)
    assert out.shape == (2, 8, 6, 9)
    ref = (img.clamp(0, 1) * mask).squeeze(1)[..., :9]
    assert (out - ref).abs().max() < 1e-6


def test_worker_host_path_matches_oracle_and_loads_in_workers(tmp_path, monkeypatch):
    """BRATSVolumes inside DataLoader workers (the reference scripts use
    num_workers=12; a forked worker cannot own a HIP context) runs the
    reference's numpy arithmetic and returns CPU tensors equal to the oracle's
    modality tensor.  nibabel is absent here: a stub module decodes .npy files."""
    import sys
    import types
    from guided_diffusion import bratsloader
    img = brain_like((40, 36, 31), 1)
    assert torch.equal(bratsloader._prepare_modality_host(img, pad_z=32, crop=4),
                       ov.modality_tensor(img, pad_z=32, crop=4))
    subj = tmp_path / "BraTS-GLI-00000-000"
    subj.mkdir()
    vols = {}
    for k, key in enumerate(("t1n", "t1c", "t2w", "t2f")):
        v = brain_like((240, 240, 155), 10 + k)
        vols[key] = v
        np.save(subj / f"BraTS-GLI-00000-000-{key}.npy", v)
    stub = types.ModuleType("nibabel")

    class _Img:
        def __init__(self, path):
            self.path = path

        def get_fdata(self):
            return np.load(self.path)
    stub.load = _Img
    monkeypatch.setitem(sys.modules, "nibabel", stub)
    ds = bratsloader.BRATSVolumes(str(tmp_path), mode="train")
    dl = torch.utils.data.DataLoader(ds, batch_size=1, num_workers=2, multiprocessing_context="fork")
    batch = next(iter(dl))
    for key, v in vols.items():
        assert batch[key].shape == (1, 1, 224, 224, 160) and not batch[key].is_cuda
        assert torch.equal(batch[key][0], ov.modality_tensor(v)), key
