"""Seeded synthetic BraTS-like phantoms (TEST INFRASTRUCTURE ONLY).

Mimics the value range of bratsloader.clip_and_normalize output
(guided_diffusion/bratsloader.py:105-109): an ellipsoid "brain" with smooth
Gaussian-blob intensities in [0, 1] and an exactly-zero background
(SURVEY.md §8d).
"""
import torch


def phantom(size, seed, batch=1):
    D = H = W = size
    g = torch.Generator().manual_seed(seed)
    z = torch.linspace(-1, 1, D).view(D, 1, 1)
    y = torch.linspace(-1, 1, H).view(1, H, 1)
    x = torch.linspace(-1, 1, W).view(1, 1, W)
    out = torch.zeros(batch, 1, D, H, W)
    for b in range(batch):
        ax = 0.75 + 0.15 * torch.rand(3, generator=g)
        mask = (z / ax[0]) ** 2 + (y / ax[1]) ** 2 + (x / ax[2]) ** 2 <= 1.0
        img = torch.zeros(D, H, W)
        for _ in range(6):
            c = (torch.rand(3, generator=g) - 0.5) * 1.2
            s = 0.15 + 0.35 * torch.rand(1, generator=g)
            a = 0.3 + 0.7 * torch.rand(1, generator=g)
            img += a * torch.exp(-((z - c[0]) ** 2 + (y - c[1]) ** 2 + (x - c[2]) ** 2) / (2 * s ** 2))
        img = img * mask
        mx = img.max()
        if mx > 0:
            img = img / mx
        out[b, 0] = img.clamp(0, 1)
    return out


def brats_batch(size, seed, batch=1):
    """Four contrasts (t1n, t1c, t2w, t2f) sharing one brain mask."""
    keys = ("t1n", "t1c", "t2w", "t2f")
    base = phantom(size, seed, batch)
    mask = (base > 0).float()
    res = {}
    for k, key in enumerate(keys):
        v = phantom(size, seed * 10 + k + 1, batch)
        res[key] = (0.5 * base + 0.5 * v) * mask
    return res
