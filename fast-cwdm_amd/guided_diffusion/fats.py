"""FATS -- Frequency-Adaptive Timestep Scheduling, by specification.

The reference has no code for it: README.md:3-9 describes FATS as leveraging
"wavelet energy statistics to learn optimal noise schedules for different
frequency bands".  This module makes that concrete for the i2i wavelet path:

* every Haar subband k diffuses on its own schedule
  acp_k(t) = sigmoid(logit(acp(t)) + shift_k), i.e. a constant log-SNR offset
  of the shared schedule (acp_k stays monotone, acp_k(t) -> acp(t) as shift_k -> 0);
* the offsets come from the subbands' energies E_k = E[x0_k^2] (the wavelet
  energy statistics): shift_k = strength * (mean_j log E_j - log E_k),
  clipped to +-max_shift, which equalises the effective SNR E_k * acp_k /
  (1 - acp_k) across subbands at every t (low-energy high-frequency bands are
  not drowned early, the high-energy LLL band is not left nearly clean late).

GaussianDiffusion(band_log_snr_shift=shifts) then carries [T, 8] tables; the
fused sampler step (cwdm_sampler_step, per_band) and the training front end
(cwdm_prepare_batch, per_band) read one coefficient row per subband, so the
sampling loop, its HIP graph and training run unchanged.  Respacing keeps the
per-band tables consistent (acp_k at a kept step depends only on acp there).
Parity: the oracle restates the same definition (oracle/diffusion.py Tables).
"""
import numpy as np


def band_energy(x0_bands):
    """Mean energy E[x0_k^2] per subband of a (B, 8, d, h, w) wavelet batch
    (LLL already / 3, as training_losses feeds it); float64 numpy [8]."""
    x = x0_bands.detach()
    if x.dim() != 5:
        raise AssertionError("band_energy expects (B, bands, d, h, w)")
    e = (x.double() ** 2).mean(dim=(0, 2, 3, 4))
    return e.cpu().numpy()


def subband_energy(coef, levels=1):
    """band_energy for either representation: (B, 8, ...) single-level bands
    -> [8]; (B, 64, ...) two-level block coefficients (config 5,
    oracle/wavelet2.py) -> [15] (LLL2, 7 level-2 details, 7 level-1 details,
    each level-1 band's 8 folded phases pooled)."""
    e = band_energy(coef)
    if levels == 1:
        return e
    if e.shape[0] != 64:
        raise AssertionError("two-level coefficients have 64 channels")
    return np.concatenate([e[:8], e[8:].reshape(7, 8).mean(axis=1)])


def band_log_snr_shifts(energy, strength=1.0, max_shift=4.0, floor=1e-12):
    """shift_k = strength * (mean_j log E_j - log E_k), clipped to +-max_shift."""
    le = np.log(np.maximum(np.asarray(energy, dtype=np.float64), floor))
    shift = strength * (le.mean() - le)
    return np.clip(shift, -max_shift, max_shift)


def create_fats_diffusion(energy=None, shifts=None, strength=1.0, max_shift=4.0, **diffusion_kwargs):
    """script_util.create_gaussian_diffusion with FATS per-band schedules, from
    band energies (band_energy of training data) or explicit shifts."""
    from .script_util import create_gaussian_diffusion
    if shifts is None:
        if energy is None:
            raise ValueError("FATS needs the subband energies or explicit shifts")
        shifts = band_log_snr_shifts(energy, strength, max_shift)
    return create_gaussian_diffusion(band_log_snr_shift=np.asarray(shifts, dtype=np.float64), **diffusion_kwargs)


__all__ = ["band_energy", "subband_energy", "band_log_snr_shifts", "create_fats_diffusion"]
