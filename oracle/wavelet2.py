"""Oracle: 2-level block wavelet representation for config 5 (TEST INFRASTRUCTURE ONLY).

BASELINE.json config 5 ("2-level DWT (16 subbands) + FATS per-band schedule,
224^3 input") has no reference code (spec-only).  This is
the specification the native path implements, restated with the pinned
single-level Haar of oracle.haar (PyWavelets-pinned):

* level 1: the reference's DWT with LLL / 3 (gaussian_diffusion.py:1139-1140);
* level 2: the same DWT of LLL1 / 3, again LLL / 3;
* the U-Net runs on the level-2 grid (224^3 -> 56^3, a 3-level U-Net since 56
  is not divisible by 16): per modality 64 channels = the 8 level-2 bands
  (LLL2, then the 7 details in band order) followed by the 7 level-1 detail
  bands, each folded 2x2x2 -> 8 channels (space-to-depth, phase
  ph = 4 pz + 2 py + px) -- 15 distinct subbands, i.e. the 16 of a 2-level
  pyramid less the LLL1 that the level-2 bands replace;
* every coarse voxel's 64 channels are exactly the 2-level Haar transform of
  one 4x4x4 image block, so process_xstart (inverse -> clamp(0, 1) ->
  forward) stays voxel-local like the reference's single-level one
  (gaussian_diffusion.py:335-354).
"""
import torch

from . import haar

NBANDS = 15   # LLL2 + 7 level-2 details + 7 level-1 details


def band_of_channel(j):
    """Subband index (0..14) of channel j (0..63) of one modality."""
    return j if j < 8 else 8 + (j - 8) // 8


def _s2d(x):   # (B, C, 2d, 2h, 2w) -> (B, 8C, d, h, w), channel c * 8 + ph
    B, C, D, H, W = x.shape
    y = x.reshape(B, C, D // 2, 2, H // 2, 2, W // 2, 2).permute(0, 1, 3, 5, 7, 2, 4, 6)
    return y.reshape(B, C * 8, D // 2, H // 2, W // 2)


def _d2s(x):   # inverse of _s2d
    B, C8, d, h, w = x.shape
    y = x.reshape(B, C8 // 8, 2, 2, 2, d, h, w).permute(0, 1, 5, 2, 6, 3, 7, 4)
    return y.reshape(B, C8 // 8, 2 * d, 2 * h, 2 * w)


def analysis2(x, scale=True):
    """(B, 1, 4d, 4h, 4w) image -> (B, 64, d, h, w) coefficients.  scale=False:
    no LLL / 3 at either level -- the noise image's transform in
    training_losses (the reference DWTs the noise without the /3,
    gaussian_diffusion.py:1143-1145)."""
    assert x.dim() == 5 and x.shape[1] == 1
    div = 3.0 if scale else 1.0
    b1 = haar.dwt3d(x)
    b2 = haar.dwt3d(b1[0] / div)
    low = [b2[0] / div] + list(b2[1:])
    return torch.cat(low + [_s2d(b) for b in b1[1:]], dim=1)


def synthesis2(c):
    """(B, 64, d, h, w) -> (B, 1, 4d, 4h, 4w) image (inverse of analysis2)."""
    assert c.dim() == 5 and c.shape[1] == 64
    l1 = haar.idwt3d(c[:, 0:1] * 3.0, *[c[:, k:k + 1] for k in range(1, 8)]) * 3.0
    det = [_d2s(c[:, 8 + 8 * k:16 + 8 * k]) for k in range(7)]
    return haar.idwt3d(l1, *det)


def process_xstart2(x):
    """synthesis2 -> clamp(0, 1) -> analysis2 (the 2-level process_xstart)."""
    return analysis2(synthesis2(x).clamp(0.0, 1.0))


def channel_shift(band_shift):
    """15 per-subband log-SNR offsets -> 64 per-channel offsets (FATS)."""
    return [float(band_shift[band_of_channel(j)]) for j in range(64)]
