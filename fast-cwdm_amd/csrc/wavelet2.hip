// Two-level block wavelet representation (BASELINE config 5: "2-level DWT +
// FATS per-band schedule, 224^3"; no reference code, specification in
// oracle/wavelet2.py).  Level 1 is the reference's Haar DWT with LLL / 3
// (gaussian_diffusion.py:1139-1140), level 2 the same transform of LLL1 / 3;
// the U-Net grid is the level-2 grid and each coarse voxel carries 64
// channels per modality: the 8 level-2 bands, then the 7 level-1 detail bands
// folded 2x2x2 -> 8 channels (phase ph = 4 pz + 2 py + px).  Those 64 values
// are exactly the 2-level transform of one 4x4x4 image block, so analysis,
// synthesis and the sampler's process_xstart are all one-thread-per-block
// register transforms (haar8.hpp, products rounded before adds like the
// single-level kernels: bit-exact against the oracle).
#include "common.hpp"
#include <type_traits>

#include "haar8.hpp"
#include "sampler.hpp"

namespace cwdm {
namespace {

// img: 4x4x4 block [z][y][x] -> c: the 64 coefficients.  SCALE = false: the
// plain orthonormal 2-level transform (no LLL / 3 at either level), the noise
// image's transform in training_losses (the reference DWTs the noise without
// the /3, gaussian_diffusion.py:1143-1145)
template <bool SCALE = true>
__device__ __forceinline__ void wav2_fwd(const float img[64], float c[64]) {
  float l1[8];
#pragma unroll
  for (int ph = 0; ph < 8; ++ph) {
    const int pz = ph >> 2, py = (ph >> 1) & 1, px = ph & 1;
    float v[8], o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = img[(2 * pz + (i >> 2)) * 16 + (2 * py + ((i >> 1) & 1)) * 4 + 2 * px + (i & 1)];
    haar_fwd8(v, o);
    l1[ph] = SCALE ? __fdiv_rn(o[0], 3.0f) : o[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) c[8 + (k - 1) * 8 + ph] = o[k];
  }
  float o2[8];
  haar_fwd8(l1, o2);
  c[0] = SCALE ? __fdiv_rn(o2[0], 3.0f) : o2[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) c[k] = o2[k];
}

__device__ __forceinline__ void wav2_inv(const float c[64], float img[64]) {
  float b2[8], l1[8];
  b2[0] = mr(c[0], 3.0f);
#pragma unroll
  for (int k = 1; k < 8; ++k) b2[k] = c[k];
  haar_inv8(b2, l1);
#pragma unroll
  for (int ph = 0; ph < 8; ++ph) {
    const int pz = ph >> 2, py = (ph >> 1) & 1, px = ph & 1;
    float o[8], v[8];
    o[0] = mr(l1[ph], 3.0f);
#pragma unroll
    for (int k = 1; k < 8; ++k) o[k] = c[8 + (k - 1) * 8 + ph];
    haar_inv8(o, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) img[(2 * pz + (i >> 2)) * 16 + (2 * py + ((i >> 1) & 1)) * 4 + 2 * px + (i & 1)] = v[i];
  }
}

struct S3w { int64_t b, c, v; };

template <typename T>
__device__ __forceinline__ void stw(T* p, int64_t off, float v) { p[off] = Elem<T>::from_f(v); }

__device__ __forceinline__ float4 ld4(const float* base, S3w s, int64_t b, int q, int64_t v, bool vec) {
  const float* p = base + b * s.b + v * s.v;
  if (vec) return *reinterpret_cast<const float4*>(p + q);
  return make_float4(p[q * s.c], p[(q + 1) * s.c], p[(q + 2) * s.c], p[(q + 3) * s.c]);
}
__device__ __forceinline__ void st4(float* base, S3w s, int64_t b, int q, int64_t v, bool vec, float4 u) {
  float* p = base + b * s.b + v * s.v;
  if (vec) {
    *reinterpret_cast<float4*>(p + q) = u;
  } else {
    p[q * s.c] = u.x; p[(q + 1) * s.c] = u.y; p[(q + 2) * s.c] = u.z; p[(q + 3) * s.c] = u.w;
  }
}

// x (B, 1, 4d, 4h, 4w) fp32 contiguous -> out[b * obs + v * ovs + oc0 + j], j < 64
template <typename TO>
__global__ void __launch_bounds__(256) wav2_analysis_kernel(const float* __restrict__ x, int64_t B, int64_t d,
                                                           int64_t h, int64_t w, TO* __restrict__ out, int64_t obs,
                                                           int64_t ovs, int oc0) {
  const int64_t nv = d * h * w;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * nv) return;
  const int64_t b = i / nv, v = i - b * nv;
  const int64_t xx = v % w, yy = (v / w) % h, zz = v / (w * h);
  const int64_t W4 = 4 * w, H4 = 4 * h;
  float img[64], c[64];
#pragma unroll
  for (int r = 0; r < 16; ++r) {   // rows (z, y) of the block: 4 floats each
    const float4 q = *reinterpret_cast<const float4*>(
        x + ((b * 4 * d + 4 * zz + (r >> 2)) * H4 + 4 * yy + (r & 3)) * W4 + 4 * xx);
    img[r * 4 + 0] = q.x; img[r * 4 + 1] = q.y; img[r * 4 + 2] = q.z; img[r * 4 + 3] = q.w;
  }
  wav2_fwd(img, c);
  TO* o = out + b * obs + v * ovs + oc0;
#pragma unroll
  for (int j = 0; j < 64; ++j) stw<TO>(o, j, c[j]);
}

__device__ __forceinline__ void load_block4(const float* __restrict__ x, int64_t b, int64_t d, int64_t h, int64_t w,
                                            int64_t v, float img[64]) {
  const int64_t xx = v % w, yy = (v / w) % h, zz = v / (w * h);
  const int64_t W4 = 4 * w, H4 = 4 * h;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float4 q = *reinterpret_cast<const float4*>(
        x + ((b * 4 * d + 4 * zz + (r >> 2)) * H4 + 4 * yy + (r & 3)) * W4 + 4 * xx);
    img[r * 4 + 0] = q.x; img[r * 4 + 1] = q.y; img[r * 4 + 2] = q.z; img[r * 4 + 3] = q.w;
  }
}

// training_losses front end for the 2-level representation (config 5; the
// levels-1 cwdm_prepare_batch restated, oracle.diffusion.training_losses with
// levels = 2): x0 = analysis2(target), the three conditions' analysis2, the
// noise image's unscaled transform, q_sample with per-channel rows when
// per_band.  One coarse voxel (one 4x4x4 block of each of the 5 volumes) per
// thread; NCDHW fp32 outputs x_in (B, 256, d, h, w), x0 (B, 64, d, h, w).
struct Prep2Args {
  const float* img[5];  // target, c1, c2, c3, eps
  float* x_in; float* x0;
  const float* coef; const int64_t* t; int64_t T;
  int64_t B, d, h, w; int per_band;
};

__global__ void __launch_bounds__(256) prepare_batch2_kernel(Prep2Args a) {
  const int64_t nv = a.d * a.h * a.w;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.B * nv) return;
  const int64_t b = i / nv, v = i - b * nv;
  int64_t t = a.t[b];
  t = t < 0 ? 0 : (t >= a.T ? a.T - 1 : t);
  const float* cq = a.coef + t * (a.per_band ? 128 : 2);
  const int bs = a.per_band ? 2 : 0;
  float img[64], x0[64], c[64];
  load_block4(a.img[0], b, a.d, a.h, a.w, v, img);
  wav2_fwd<true>(img, x0);
  float* o0 = a.x0 + b * 64 * nv + v;
#pragma unroll
  for (int j = 0; j < 64; ++j) o0[j * nv] = x0[j];
  load_block4(a.img[4], b, a.d, a.h, a.w, v, img);
  wav2_fwd<false>(img, c);
  float* xin = a.x_in + b * 256 * nv + v;
#pragma unroll
  for (int j = 0; j < 64; ++j) xin[j * nv] = ad(mr(cq[j * bs], x0[j]), mr(cq[j * bs + 1], c[j]));
  for (int s = 1; s < 4; ++s) {
    load_block4(a.img[s], b, a.d, a.h, a.w, v, img);
    wav2_fwd<true>(img, c);
#pragma unroll
    for (int j = 0; j < 64; ++j) xin[(64 * s + j) * nv] = c[j];
  }
}

// coefficients (fp32, coef[b * cbs + v * cvs + cc0 + j]) -> image (B, 1, 4d, 4h, 4w)
__global__ void __launch_bounds__(256) wav2_synthesis_kernel(const float* __restrict__ coef, int64_t B, int64_t d,
                                                            int64_t h, int64_t w, int64_t cbs, int64_t cvs, int cc0,
                                                            float* __restrict__ out) {
  const int64_t nv = d * h * w;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * nv) return;
  const int64_t b = i / nv, v = i - b * nv;
  const int64_t xx = v % w, yy = (v / w) % h, zz = v / (w * h);
  const int64_t W4 = 4 * w, H4 = 4 * h;
  float c[64], img[64];
  const float* p = coef + b * cbs + v * cvs + cc0;
#pragma unroll
  for (int j = 0; j < 64; ++j) c[j] = p[j];
  wav2_inv(c, img);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    *reinterpret_cast<float4*>(out + ((b * 4 * d + 4 * zz + (r >> 2)) * H4 + 4 * yy + (r & 3)) * W4 + 4 * xx) =
        make_float4(img[r * 4], img[r * 4 + 1], img[r * 4 + 2], img[r * 4 + 3]);
}

// cwdm_sampler_step with levels = 2: 64 channels per coarse voxel; the same
// math as sampler_kernel (wavelet.hip) with the 2-level process_xstart.
// vec bit k: tensor k (model_out, x_t, x_prev, noise, pred, mirror) is
// channel-contiguous and 16-byte aligned -> float4 accesses.
template <typename MirT>
__global__ void __launch_bounds__(256) sampler2_kernel(cwdm_sampler_args a, S3w mo, S3w xt, S3w xp, S3w nz, S3w px,
                                                      S3w mi, int vec) {
  const int64_t nvox = a.d * a.h * a.w;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.B * nvox) return;
  const int64_t b = idx / nvox, v = idx - b * nvox;
  int64_t t = a.t[b];
  t = t < 0 ? 0 : (t >= a.T ? a.T - 1 : t);
  const int bs = a.per_band ? 8 : 0;   // per-channel coefficient rows ([T][64][8]) or one shared row
  const float* cf = a.coef + t * (a.per_band ? 64 * 8 : 8);
  float m[64];
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float4 u = ld4(a.model_out, mo, b, 4 * g, v, vec & 1);
    m[4 * g] = u.x; m[4 * g + 1] = u.y; m[4 * g + 2] = u.z; m[4 * g + 3] = u.w;
  }
  if (a.mean_type == 1) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 u = ld4(a.x_t, xt, b, 4 * g, v, vec & 2);
      const float xq[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = 4 * g + k;
        m[q] = sb(mr(cf[q * bs + 3], xq[k]), mr(cf[q * bs + 4], m[q]));
      }
    }
  }
  float pred[64];
  if (a.clip_denoised) {
    float img[64];
    wav2_inv(m, img);
#pragma unroll
    for (int q = 0; q < 64; ++q) img[q] = fminf(fmaxf(img[q], 0.0f), 1.0f);
    wav2_fwd(img, pred);
  } else {
#pragma unroll
    for (int q = 0; q < 64; ++q) pred[q] = m[q];
  }
  const bool noisy = a.update != 1 && t != 0 && (a.noise || a.noise_philox);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float4 u = ld4(a.x_t, xt, b, 4 * g, v, vec & 2);
    const float xq[4] = {u.x, u.y, u.z, u.w};
    float nq[4] = {0.f, 0.f, 0.f, 0.f};
    if (noisy && a.noise) {
      const float4 n4 = ld4(a.noise, nz, b, 4 * g, v, vec & 8);
      nq[0] = n4.x; nq[1] = n4.y; nq[2] = n4.z; nq[3] = n4.w;
    } else if (noisy) {
      philox_normal4(a.noise_seed, v, b, t, g, nq);
    }
    float r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = 4 * g + k;
      const float* c = cf + q * bs;
      if (a.update == 1) {
        const float eps = __fdiv_rn(sb(mr(c[3], xq[k]), pred[q]), c[4]);
        r[k] = ad(mr(pred[q], c[5]), mr(c[6], eps));
      } else {
        r[k] = ad(mr(c[0], pred[q]), mr(c[1], xq[k]));
        if (noisy) r[k] = ad(r[k], mr(c[2], nq[k]));
      }
    }
    st4(a.x_prev, xp, b, 4 * g, v, vec & 4, make_float4(r[0], r[1], r[2], r[3]));
    if (a.pred_xstart)
      st4(a.pred_xstart, px, b, 4 * g, v, vec & 16, make_float4(pred[4 * g], pred[4 * g + 1], pred[4 * g + 2], pred[4 * g + 3]));
    if (a.mirror) {
      MirT* o = reinterpret_cast<MirT*>(a.mirror) + b * mi.b + v * mi.v;
      if ((vec & 32) && sizeof(MirT) == 2) {
        using M16 = std::conditional_t<sizeof(MirT) == 2, MirT, bf16_t>;
        uint2 q2;
        q2.x = pack2<M16>(r[0], r[1]);
        q2.y = pack2<M16>(r[2], r[3]);
        *reinterpret_cast<uint2*>(o + 4 * g) = q2;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) stw<MirT>(o, (4 * g + k) * mi.c, r[k]);
      }
    }
  }
}

// The same step with every tensor access staged through LDS (the fast path of
// the resident loop: model_out, x_t, x_prev channels-last and 16-byte aligned,
// Philox noise, no pred_xstart).  One thread still owns one coarse voxel's 64
// channels (the 2-level transform mixes all of them), but a thread-per-voxel
// float4 access touches 64 rows of 256 B per wave instruction (1.2 TB/s, 122 us
// per 56^3 step); here each 16-lane group moves one whole 256-byte row.  Rows
// are padded to 272 B so the per-thread row reads are conflict-free.  Bit-
// identical to sampler2_kernel (same expressions in the same order).
// CL = false: x_t and x_prev are channel-planar (voxel stride 1, the native
// loop's NCDHW state): each thread moves its own voxel's 64 channels between
// its row and HBM, one coalesced 256-byte wave access per channel.
constexpr int S2V = 256;               // voxels per workgroup (one per thread)
constexpr int S2P = 68;                // row pitch in floats (272 B)
template <typename MirT, bool CL>
__global__ void __launch_bounds__(256) sampler2_lds_kernel(cwdm_sampler_args a, S3w mo, S3w xt, S3w xp, S3w mi) {
  extern __shared__ __attribute__((aligned(16))) float tile[];   // [S2V][S2P]
  const int64_t nvox = a.d * a.h * a.w, total = a.B * nvox;
  const int64_t i0 = (int64_t)blockIdx.x * S2V;
  const int tid = threadIdx.x;
  // whole rows in / out: pass k moves voxels 16 k + tid / 16, float4 tid % 16
  auto stage_in = [&](const float* base, S3w st) {
#pragma unroll 4
    for (int k = 0; k < S2V / 16; ++k) {
      const int lv = 16 * k + (tid >> 4), g = tid & 15;
      const int64_t idx = i0 + lv;
      float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < total) {
        const int64_t b = idx / nvox, v = idx - b * nvox;
        u = *reinterpret_cast<const float4*>(base + b * st.b + v * st.v + 4 * g);
      }
      *reinterpret_cast<float4*>(tile + lv * S2P + 4 * g) = u;
    }
  };
  const int64_t idx = i0 + tid;
  const bool live = idx < total;
  const int64_t b = live ? idx / nvox : 0, v = live ? idx - b * nvox : 0;
  int64_t t = a.t[b];
  t = t < 0 ? 0 : (t >= a.T ? a.T - 1 : t);
  const int bs = a.per_band ? 8 : 0;
  const float* cf = a.coef + t * (a.per_band ? 64 * 8 : 8);
  float* row = tile + tid * S2P;
  float m[64];
  // (planar x_t: the voxel's own channels, loads in flight during the model_out staging)
  float xr[CL ? 1 : 64];
  if constexpr (!CL) {
    const float* src = a.x_t + b * xt.b + v;
#pragma unroll
    for (int q = 0; q < 64; ++q) xr[q] = live ? src[q * xt.c] : 0.f;
  }
  stage_in(a.model_out, mo);
  __syncthreads();
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float4 u = *reinterpret_cast<const float4*>(row + 4 * g);
    m[4 * g] = u.x; m[4 * g + 1] = u.y; m[4 * g + 2] = u.z; m[4 * g + 3] = u.w;
  }
  __syncthreads();
  if constexpr (CL) {
    stage_in(a.x_t, xt);
  } else {
#pragma unroll
    for (int g = 0; g < 16; ++g)
      *reinterpret_cast<float4*>(row + 4 * g) = make_float4(xr[4 * g], xr[4 * g + 1], xr[4 * g + 2], xr[4 * g + 3]);
  }
  __syncthreads();
  if (a.mean_type == 1) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 u = *reinterpret_cast<const float4*>(row + 4 * g);
      const float xq[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = 4 * g + k;
        m[q] = sb(mr(cf[q * bs + 3], xq[k]), mr(cf[q * bs + 4], m[q]));
      }
    }
  }
  float pred[64];
  if (a.clip_denoised) {
    float img[64];
    wav2_inv(m, img);
#pragma unroll
    for (int q = 0; q < 64; ++q) img[q] = fminf(fmaxf(img[q], 0.0f), 1.0f);
    wav2_fwd(img, pred);
  } else {
#pragma unroll
    for (int q = 0; q < 64; ++q) pred[q] = m[q];
  }
  const bool noisy = a.update != 1 && t != 0 && a.noise_philox;
  // x_{t-1} over the x_t row (each thread owns its row)
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float4 u = *reinterpret_cast<const float4*>(row + 4 * g);
    const float xq[4] = {u.x, u.y, u.z, u.w};
    float nq[4] = {0.f, 0.f, 0.f, 0.f};
    if (noisy) philox_normal4(a.noise_seed, v, b, t, g, nq);
    float r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = 4 * g + k;
      const float* c = cf + q * bs;
      if (a.update == 1) {
        const float eps = __fdiv_rn(sb(mr(c[3], xq[k]), pred[q]), c[4]);
        r[k] = ad(mr(pred[q], c[5]), mr(c[6], eps));
      } else {
        r[k] = ad(mr(c[0], pred[q]), mr(c[1], xq[k]));
        if (noisy) r[k] = ad(r[k], mr(c[2], nq[k]));
      }
    }
    *reinterpret_cast<float4*>(row + 4 * g) = make_float4(r[0], r[1], r[2], r[3]);
    if constexpr (!CL) {
      if (live) {
        float* dst = a.x_prev + b * xp.b + v + (4 * g) * xp.c;
        dst[0] = r[0]; dst[xp.c] = r[1]; dst[2 * xp.c] = r[2]; dst[3 * xp.c] = r[3];
      }
    }
  }
  if (!CL && !a.mirror) return;
  __syncthreads();
  // rows out: x_prev (fp32) and the mirror (the next step's U-Net input channels)
#pragma unroll 4
  for (int k = 0; k < S2V / 16; ++k) {
    const int lv = 16 * k + (tid >> 4), g = tid & 15;
    const int64_t j = i0 + lv;
    if (j >= total) continue;
    const int64_t bb = j / nvox, vv = j - bb * nvox;
    const float4 u = *reinterpret_cast<const float4*>(tile + lv * S2P + 4 * g);
    if constexpr (CL) *reinterpret_cast<float4*>(a.x_prev + bb * xp.b + vv * xp.v + 4 * g) = u;
    if (a.mirror) {
      MirT* o = reinterpret_cast<MirT*>(a.mirror) + bb * mi.b + vv * mi.v + 4 * g;
      if constexpr (sizeof(MirT) == 2) {
        uint2 q2;
        q2.x = pack2<MirT>(u.x, u.y);
        q2.y = pack2<MirT>(u.z, u.w);
        *reinterpret_cast<uint2*>(o) = q2;
      } else {
        *reinterpret_cast<float4*>(o) = u;
      }
    }
  }
}

}  // namespace

int sampler2_launch(const cwdm_sampler_args* a, hipStream_t s) {
  auto s3 = [](const int64_t* p) { return S3w{p[0], p[1], p[2]}; };
  const S3w mo = s3(a->mo_s), xt = s3(a->xt_s), xp = s3(a->xp_s), nz = s3(a->nz_s), px = s3(a->px_s),
            mi = s3(a->mr_s);
  auto ok = [](const void* p, S3w st, int esz) {
    return p && st.c == 1 && ((uintptr_t)p % 16) == 0 && (st.b * esz) % 16 == 0 && (st.v * esz) % 16 == 0;
  };
  const int mesz = dtype_size(a->mirror_dtype);
  int vec = 0;
  if (ok(a->model_out, mo, 4)) vec |= 1;
  if (ok(a->x_t, xt, 4)) vec |= 2;
  if (ok(a->x_prev, xp, 4)) vec |= 4;
  if (ok(a->noise, nz, 4)) vec |= 8;
  if (ok(a->pred_xstart, px, 4)) vec |= 16;
  if (a->mirror && mi.c == 1 && ((uintptr_t)a->mirror % 8) == 0 && (mi.b * mesz) % 8 == 0 && (mi.v * mesz) % 8 == 0)
    vec |= 32;
  // the staged kernel: every tensor channels-last (channel stride 1), 16-byte
  // aligned rows, Philox noise (or none), no pred_xstart output
  static const bool lds_on = [] { const char* e = std::getenv("CWDM_SAMPLER2_LDS"); return !(e && e[0] == '0'); }();
  const bool mir_ok = !a->mirror || ((vec & 32) && (a->mirror_dtype == CWDM_F32 ? ok(a->mirror, mi, 4) : true));
  // (or x_t / x_prev channel-planar: voxel stride 1, 4-byte aligned)
  const bool planar = xt.v == 1 && xp.v == 1 && a->x_t && a->x_prev;
  const bool cl = (vec & 6) == 6;
  if (lds_on && (vec & 1) && (cl || planar) && !a->pred_xstart && !a->noise && mir_ok) {
    const dim3 g2((unsigned)ceil_div(a->B * a->d * a->h * a->w, S2V));
    const size_t sm = (size_t)S2V * S2P * 4;
    auto go = [&](auto k) -> int {
      CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
      hipLaunchKernelGGL(k, g2, dim3(256), sm, s, *a, mo, xt, xp, mi);
      return (int)CWDM_OK;
    };
    int rc;
    if (a->mirror && a->mirror_dtype == CWDM_BF16) rc = cl ? go(sampler2_lds_kernel<bf16_t, true>) : go(sampler2_lds_kernel<bf16_t, false>);
    else if (a->mirror && a->mirror_dtype == CWDM_F16) rc = cl ? go(sampler2_lds_kernel<f16_t, true>) : go(sampler2_lds_kernel<f16_t, false>);
    else if (!a->mirror || a->mirror_dtype == CWDM_F32) rc = cl ? go(sampler2_lds_kernel<float, true>) : go(sampler2_lds_kernel<float, false>);
    else return fail(CWDM_E_INVALID, "cwdm_sampler_step: bad mirror dtype");
    if (rc) return rc;
    CWDM_LAUNCHED();
    return CWDM_OK;
  }
  const dim3 grid((unsigned)ceil_div(a->B * a->d * a->h * a->w, 256));
  if (a->mirror && a->mirror_dtype == CWDM_BF16)
    hipLaunchKernelGGL(sampler2_kernel<bf16_t>, grid, dim3(256), 0, s, *a, mo, xt, xp, nz, px, mi, vec);
  else if (a->mirror && a->mirror_dtype == CWDM_F16)
    hipLaunchKernelGGL(sampler2_kernel<f16_t>, grid, dim3(256), 0, s, *a, mo, xt, xp, nz, px, mi, vec);
  else if (!a->mirror || a->mirror_dtype == CWDM_F32)
    hipLaunchKernelGGL(sampler2_kernel<float>, grid, dim3(256), 0, s, *a, mo, xt, xp, nz, px, mi, vec);
  else
    return fail(CWDM_E_INVALID, "cwdm_sampler_step: bad mirror dtype");
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_wavelet2_analysis(const float* x, int64_t B, int64_t D, int64_t H, int64_t W, void* out,
                                      int out_dtype, int64_t out_bs, int64_t out_vs, int out_c0,
                                      cwdm_stream_t stream) {
  CWDM_REQUIRE(x && out, CWDM_E_INVALID, "cwdm_wavelet2_analysis: null pointer");
  CWDM_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0 && D % 4 == 0 && H % 4 == 0 && W % 4 == 0, CWDM_E_SHAPE,
               "cwdm_wavelet2_analysis: every edge must be a positive multiple of 4");
  CWDM_REQUIRE(((uintptr_t)x % 16) == 0, CWDM_E_INVALID, "cwdm_wavelet2_analysis: input not 16-byte aligned");
  const int64_t d = D / 4, h = H / 4, w = W / 4;
  const dim3 grid((unsigned)ceil_div(B * d * h * w, 256));
  hipStream_t s = (hipStream_t)stream;
  if (out_dtype == CWDM_BF16)
    hipLaunchKernelGGL(wav2_analysis_kernel<bf16_t>, grid, dim3(256), 0, s, x, B, d, h, w,
                       reinterpret_cast<bf16_t*>(out), out_bs, out_vs, out_c0);
  else if (out_dtype == CWDM_F16)
    hipLaunchKernelGGL(wav2_analysis_kernel<f16_t>, grid, dim3(256), 0, s, x, B, d, h, w,
                       reinterpret_cast<f16_t*>(out), out_bs, out_vs, out_c0);
  else if (out_dtype == CWDM_F32)
    hipLaunchKernelGGL(wav2_analysis_kernel<float>, grid, dim3(256), 0, s, x, B, d, h, w,
                       reinterpret_cast<float*>(out), out_bs, out_vs, out_c0);
  else
    return fail(CWDM_E_INVALID, "cwdm_wavelet2_analysis: bad output dtype");
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int cwdm_wavelet2_synthesis(const float* coef, int64_t B, int64_t d, int64_t h, int64_t w,
                                       int64_t c_bs, int64_t c_vs, int c_c0, float* out, cwdm_stream_t stream) {
  CWDM_REQUIRE(coef && out, CWDM_E_INVALID, "cwdm_wavelet2_synthesis: null pointer");
  CWDM_REQUIRE(B > 0 && d > 0 && h > 0 && w > 0, CWDM_E_SHAPE, "cwdm_wavelet2_synthesis: empty grid");
  CWDM_REQUIRE(((uintptr_t)out % 16) == 0, CWDM_E_INVALID, "cwdm_wavelet2_synthesis: output not 16-byte aligned");
  const dim3 grid((unsigned)ceil_div(B * d * h * w, 256));
  hipLaunchKernelGGL(wav2_synthesis_kernel, grid, dim3(256), 0, (hipStream_t)stream, coef, B, d, h, w, c_bs, c_vs,
                     c_c0, out);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int cwdm_prepare_batch2(const float* target, const float* c1, const float* c2, const float* c3,
                                   const float* eps_img, int64_t B, int64_t D, int64_t H, int64_t W,
                                   const float* coef, int per_band, const int64_t* t, int64_t T, float* x_in,
                                   float* x0, cwdm_stream_t stream) {
  CWDM_REQUIRE(target && c1 && c2 && c3 && eps_img && coef && t && x_in && x0, CWDM_E_INVALID,
               "cwdm_prepare_batch2: null pointer");
  CWDM_REQUIRE(B > 0 && D > 0 && H > 0 && W > 0 && T > 0, CWDM_E_SHAPE, "cwdm_prepare_batch2: empty shape");
  CWDM_REQUIRE(D % 4 == 0 && H % 4 == 0 && W % 4 == 0, CWDM_E_SHAPE,
               "cwdm_prepare_batch2: D, H, W must be multiples of 4");
  Prep2Args a{{target, c1, c2, c3, eps_img}, x_in, x0, coef, t, T, B, D / 4, H / 4, W / 4, per_band ? 1 : 0};
  for (int s = 0; s < 5; ++s)
    CWDM_REQUIRE(((uintptr_t)a.img[s] & 15) == 0, CWDM_E_INVALID, "cwdm_prepare_batch2: volumes must be 16-byte aligned");
  const int64_t n = B * a.d * a.h * a.w;
  hipLaunchKernelGGL(prepare_batch2_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, a);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
