// The per-voxel sampler epilogue (fused a3 + a7 + a9):
// process_xstart (IDWT(3 LLL) -> clamp(0, 1) -> DWT -> LLL / 3,
// guided_diffusion/gaussian_diffusion.py:335-354), q_posterior_mean_variance
// (:244-267) and the noise add of p_sample (:565-573), or the DDIM update of
// ddim_sample (:753-784) -- shared by the standalone sampler kernel
// (wavelet.hip) and the output head that runs it on its own accumulators
// (conv3d_head.hip).  Every product is rounded before the add (mr / ad / sb /
// __fdiv_rn), so both give the same bits.
//
// Noise: a caller's tensor, or (cwdm_sampler_args.philox) drawn here --
// Philox4x32-10 keyed by the loop's 64-bit seed, counter (voxel, batch,
// timestep, draw), Box-Muller on pairs of 24-bit uniforms (u1 in (0, 1]).  The
// counter holds the device timestep t, so a graph-replayed step draws fresh
// noise every replay without any host-side state.
//
// Every add here goes through mr / ad / sb, and the pragmas keep the rest
// uncontracted whatever the including file's -ffp-contract.
#pragma once
#include "common.hpp"
#include "haar8.hpp"

namespace cwdm {

__device__ __forceinline__ void philox4x32_10(unsigned c[4], unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const unsigned hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const unsigned n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// 4 standard normals (channels 4k .. 4k+3) for voxel v of batch b at timestep
// t: counter (v lo, v hi, t, b << 8 | k), key = the seed.
__device__ __forceinline__ void philox_normal4(uint64_t seed, int64_t v, int64_t b, int64_t t, int k, float z[4]) {
#pragma clang fp contract(off)
  unsigned c[4] = {(unsigned)v, (unsigned)((uint64_t)v >> 32), (unsigned)t, ((unsigned)b << 8) | (unsigned)k};
  philox4x32_10(c, (unsigned)seed, (unsigned)(seed >> 32));
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float u1 = ((c[2 * p] >> 8) + 1u) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (c[2 * p + 1] >> 8) * (1.0f / 16777216.0f);      // [0, 1)
    // single hardware instructions (v_log_f32 = log2, v_sqrt_f32, v_sin / v_cos
    // of 2 pi x), not the libm expansions: the same bits in every kernel that
    // includes this, whatever its contraction flags
    const float r = __builtin_amdgcn_sqrtf(__builtin_amdgcn_logf(u1) * -1.3862943611198906f);  // -2 ln 2
    z[2 * p] = r * __builtin_amdgcn_cosf(u2);
    z[2 * p + 1] = r * __builtin_amdgcn_sinf(u2);
  }
}

// the 8-subband step of one voxel: m = the model output's 8 channels (START_X
// x0 or EPSILON eps), xv = x_t; returns x_{t-1} in r and the projected x0 in
// pred.  t is clamped by the caller.  noise8 holds the 8 noise values when
// has_noise (a flag, not a null pointer: the arrays stay in registers).
__device__ __forceinline__ void sampler_voxel8(const cwdm_sampler_args& a, const float* cf, int bs, int64_t t,
                                               float m[8], const float xv[8], bool has_noise, const float noise8[8],
                                               float r[8], float pred[8]) {
#pragma clang fp contract(off)
  if (a.mean_type == 1) {
    // EPSILON: x0 = sqrt(1/acp) * x_t - sqrt(1/acp - 1) * eps (gaussian_diffusion.py:392-397)
#pragma unroll
    for (int q = 0; q < 8; ++q) m[q] = sb(mr(cf[q * bs + 3], xv[q]), mr(cf[q * bs + 4], m[q]));
  }
  if (a.clip_denoised) {
    m[0] = mr(m[0], 3.0f);
    float blk[8];
    haar_inv8(m, blk);
#pragma unroll
    for (int q = 0; q < 8; ++q) blk[q] = fminf(fmaxf(blk[q], 0.0f), 1.0f);
    haar_fwd8(blk, pred);
    pred[0] = __fdiv_rn(pred[0], 3.0f);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) pred[q] = m[q];
  }
  if (a.update == 1) {
    // DDIM (ddim_sample, gaussian_diffusion.py:753-784): eps from x_t and the
    // projected x0 (_predict_eps_from_xstart, :407-415), then
    // x0 * sqrt(acp_prev) + sqrt(1 - acp_prev - sigma^2) * eps, returned
    // without noise like the reference (:784); cf[5], cf[6] hold the two roots
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float* c = cf + q * bs;
      const float eps = __fdiv_rn(sb(mr(c[3], xv[q]), pred[q]), c[4]);
      r[q] = ad(mr(pred[q], c[5]), mr(c[6], eps));
    }
  } else {
    const bool noisy = (t != 0) && has_noise;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float* c = cf + q * bs;
      const float mean = ad(mr(c[0], pred[q]), mr(c[1], xv[q]));
      r[q] = noisy ? ad(mean, mr(c[2], noise8[q])) : mean;
    }
  }
}

}  // namespace cwdm
