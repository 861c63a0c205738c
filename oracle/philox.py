"""Oracle: the sampling loop's in-kernel noise (TEST INFRASTRUCTURE ONLY).

The reference draws each step's noise with ``th.randn_like(x)`` (p_sample,
guided_diffusion/gaussian_diffusion.py:565).  The native loop instead draws it
inside the sampler kernel / fused output head (csrc/sampler.hpp,
cwdm_sampler_args.noise_philox): Philox4x32-10 (Salmon et al., SC'11, as in
Random123 and curand) keyed by a 64-bit seed, counter (voxel lo, voxel hi,
timestep, batch << 8 | channel group), Box-Muller on two 24-bit uniforms.
This module restates that in numpy.  The reference's own stream (torch's
generator) is not reproducible here, so this is parity against our
specification: the block function is pinned by Random123's published
known-answer vectors (tests/test_oracle_philox.py), the Gaussian transform by
moment checks.
"""
import numpy as np

M0, M1 = np.uint32(0xD2511F53), np.uint32(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def _mulhilo(m, x):
    p = x.astype(np.uint64) * np.uint64(m)
    return (p >> np.uint64(32)).astype(np.uint32), (p & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def philox4x32_10(ctr, key):
    """ctr: uint32 array (..., 4); key: uint32 array (..., 2) (broadcast).
    Returns the (..., 4) output block."""
    c = [np.asarray(ctr[..., i], dtype=np.uint32) for i in range(4)]
    k0 = np.asarray(key[..., 0], dtype=np.uint32)
    k1 = np.asarray(key[..., 1], dtype=np.uint32)
    with np.errstate(over="ignore"):
        for _ in range(10):
            hi0, lo0 = _mulhilo(M0, c[0])
            hi1, lo1 = _mulhilo(M1, c[2])
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = (k0 + W0).astype(np.uint32)
            k1 = (k1 + W1).astype(np.uint32)
    return np.stack(np.broadcast_arrays(*c), axis=-1)


def normal4(seed, v, b, t, k):
    """The 4 N(0, 1) values of channels 4k .. 4k+3 at voxel v (int array),
    batch b, timestep t (csrc/sampler.hpp philox_normal4), float32 (..., 4)."""
    v = np.asarray(v, dtype=np.int64)
    ctr = np.stack([(v & 0xFFFFFFFF).astype(np.uint32), (v >> 32).astype(np.uint32),
                    np.full(v.shape, t & 0xFFFFFFFF, np.uint32),
                    np.full(v.shape, ((b << 8) | k) & 0xFFFFFFFF, np.uint32)], axis=-1)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], dtype=np.uint32)
    c = philox4x32_10(ctr, key)
    out = np.empty(v.shape + (4,), np.float32)
    for p in range(2):
        u1 = ((c[..., 2 * p] >> np.uint32(8)).astype(np.float32) + np.float32(1)) * np.float32(1.0 / 16777216.0)
        u2 = (c[..., 2 * p + 1] >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        # the kernel: sqrt(log2(u1) * -2 ln 2), cos / sin of 2 pi u2 (hardware
        # v_log / v_sqrt / v_cos / v_sin: a few ulp from these)
        r = np.sqrt(np.log2(u1) * np.float32(-1.3862943611198906))
        a = np.float64(2 * np.pi) * u2.astype(np.float64)
        out[..., 2 * p] = r * np.cos(a).astype(np.float32)
        out[..., 2 * p + 1] = r * np.sin(a).astype(np.float32)
    return out


def noise_ncdhw(seed, t, B, C, d, h, w):
    """The noise tensor one step draws, (B, C, d, h, w) float32; t: per-batch
    timestep list (already clamped like the kernel)."""
    V = d * h * w
    v = np.arange(V, dtype=np.int64)
    out = np.empty((B, C, V), np.float32)
    for b in range(B):
        for k in range(C // 4):
            out[b, 4 * k:4 * k + 4] = normal4(seed, v, b, int(t[b]), k).T
    return out.reshape(B, C, d, h, w)
