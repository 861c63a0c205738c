"""CPU restatement of the volume I/O either side of the wavelet path
(TEST INFRASTRUCTURE ONLY: the checker for cwdm_quantiles /
cwdm_volume_prepare / cwdm_sample_finish, never a product path).

* clip_and_normalize: guided_diffusion/bratsloader.py:116-120 (np.quantile
  'linear', np.clip, min-max normalisation, all float64).
* modality tensor: bratsloader.py:44-50 (torch.zeros(1, 240, 240, 160) filled
  in z < 155 with the float64 result cast to fp32, then [:, 8:-8, 8:-8, :]).
* sample finish: scripts/sample.py:113-135 (IDWT of [3 LLL, ...], clamp via
  the two masked assignments, zero outside the t1n brain mask, z[:155]).
numpy is the reference's own dependency for this step, so np.quantile itself is
the pinned arithmetic here.
"""
import numpy as np
import torch

from . import haar


def clip_and_normalize(img):
    img_clipped = np.clip(img, np.quantile(img, 0.001), np.quantile(img, 0.999))
    return (img_clipped - np.min(img_clipped)) / (np.max(img_clipped) - np.min(img_clipped))


def modality_tensor(img_np, pad_z=160, crop=8):
    t = torch.zeros(1, img_np.shape[0], img_np.shape[1], pad_z)
    t[:, :, :, :img_np.shape[2]] = torch.tensor(clip_and_normalize(img_np))
    return t[:, crop:-crop, crop:-crop, :] if crop else t


def sample_finish(sample, cond_1, keep_z):
    B, _, D, H, W = sample.shape
    bands = [sample[:, i].reshape(B, 1, D, H, W) * (3.0 if i == 0 else 1.0) for i in range(8)]
    img = haar.idwt3d(*bands)
    img[img <= 0] = 0
    img[img >= 1] = 1
    if cond_1 is not None:
        img[cond_1 == 0] = 0
    img = img.squeeze(dim=1)
    return img[:, :, :, :keep_z]
