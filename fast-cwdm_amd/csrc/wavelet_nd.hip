// Channels-last, multi-channel Haar analysis / synthesis for the frequency-aware
// U-Net (WavUNetModel, guided_diffusion/wunet.py): Downsample(use_freq) =
// DWT of a feature map, LLL / 3 kept, 7 high bands returned as the skip
// (:120-128); Upsample(use_freq) = IDWT(3 LLL, skip bands) (:62-80);
// WaveletDownsample = cat(8 bands) / 3 as a conv input (:131-145).  Each
// output may get a per-(b, c) bias (the ResBlock's emb projection, added right
// after the resampling, :252) and per-part (sum, sum^2) statistics for the
// GroupNorm that consumes it (same [B][parts][C][2] contract as the conv
// epilogue).  One thread = one coarse voxel x 8 channels; a workgroup covers
// 64 coarse voxels of one batch index (one statistics part).
#include "common.hpp"
#include "haar8.hpp"

namespace cwdm {
namespace {

constexpr int kVox = 64;  // coarse voxels per workgroup (= per statistics part)

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* f) {
  if constexpr (sizeof(T) == 2) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = lo2f<T>(u[i]);
      f[2 * i + 1] = hi2f<T>(u[i]);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
}

template <typename T>
__device__ __forceinline__ void store8(T* p, const float* f) {
  if constexpr (sizeof(T) == 2) {
    uint4 q;
    q.x = pack2<T>(f[0], f[1]);
    q.y = pack2<T>(f[2], f[3]);
    q.z = pack2<T>(f[4], f[5]);
    q.w = pack2<T>(f[6], f[7]);
    *reinterpret_cast<uint4*>(p) = q;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
}

template <typename T, bool INV>
__global__ void __launch_bounds__(256) haar_nd_kernel(cwdm_haar_nd_desc a, int parts) {
  __shared__ float red[256 * 16];
  const int C = a.C, G = C / 8;
  const int tid = threadIdx.x, g = tid % G, vl = tid / G, VB = 256 / G;
  const int64_t b = blockIdx.x / parts, part = blockIdx.x % parts;
  const int64_t nv = a.d * a.h * a.w;
  const int64_t W2 = 2 * a.w, H2 = 2 * a.h;
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = a.bias ? a.bias[b * a.bias_bstride + g * 8 + e] : 0.f;
  float ssum[8], ssq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { ssum[e] = 0.f; ssq[e] = 0.f; }
  const T* src = reinterpret_cast<const T*>(a.src);
  T* out = reinterpret_cast<T*>(a.out);
  for (int vv = vl; vl < VB && vv < kVox; vv += VB) {  // threads past G x VB idle (C / 8 not a power of two)
    const int64_t v = part * kVox + vv;
    if (v >= nv) break;
    const int64_t x = v % a.w, y = (v / a.w) % a.h, z = v / (a.w * a.h);
    // fine voxel (a, bb, c) of this coarse voxel, channel group g
    auto fine = [&](int i) {
      const int pa = i >> 2, pb = (i >> 1) & 1, pc = i & 1;
      return (((b * 2 * a.d + 2 * z + pa) * H2 + 2 * y + pb) * W2 + 2 * x + pc) * C + g * 8;
    };
    if constexpr (!INV) {
      float blk[8][8];  // [fine voxel][channel]
#pragma unroll
      for (int i = 0; i < 8; ++i) load8(src + fine(i), blk[i]);
      float band[8][8];  // [band][channel]
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float vin[8], o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) vin[i] = blk[i][e];
        haar_fwd8(vin, o);
#pragma unroll
        for (int k = 0; k < 8; ++k) band[k][e] = k == 0 ? __fmul_rn(o[0], a.lll_scale) : __fmul_rn(o[k], a.high_scale);
      }
      const int64_t cv = b * nv + v;
      if (a.all8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) store8(out + (cv * 8 + k) * C + g * 8, band[k]);
      } else {
        float l[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          l[e] = band[0][e] + bias[e];
          ssum[e] += l[e];
          ssq[e] += l[e] * l[e];
        }
        store8(out + cv * C + g * 8, l);
      }
      if (a.high_out) {
        T* ho = reinterpret_cast<T*>(a.high_out);
#pragma unroll
        for (int k = 1; k < 8; ++k) store8(ho + (cv * 7 + (k - 1)) * C + g * 8, band[k]);
      }
    } else {
      const int64_t cv = b * nv + v;
      float band[8][8];
      load8(src + cv * C + g * 8, band[0]);
      const T* hi = reinterpret_cast<const T*>(a.high_in);
#pragma unroll
      for (int k = 1; k < 8; ++k) load8(hi + (cv * 7 + (k - 1)) * C + g * 8, band[k]);
      float blk[8][8];  // [fine voxel][channel]
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o[8], r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = band[k][e];
        o[0] = __fmul_rn(o[0], a.lll_scale);
        haar_inv8(o, r);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float val = r[i] + bias[e];
          blk[i][e] = val;
          ssum[e] += val;
          ssq[e] += val * val;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) store8(out + fine(i), blk[i]);
    }
  }
  if (!a.stats) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = ssum[e]; red[tid * 16 + 8 + e] = ssq[e]; }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int gg = c / 8, e = c % 8;
    float sm = 0.f, sq = 0.f;
    for (int k = 0; k < VB; ++k) { sm += red[(k * G + gg) * 16 + e]; sq += red[(k * G + gg) * 16 + 8 + e]; }
    const int64_t pidx = (b * parts + part) * C + c;
    a.stats[pidx * 2 + 0] = sm;
    a.stats[pidx * 2 + 1] = sq;
  }
}

// ---- adjoints for the backward (WavUNetModel training) ---------------------
// One thread = one coarse voxel x 8 channels.  Haar is orthonormal, so the
// adjoint of the analysis is the synthesis and vice versa; the scales of the
// forward (LLL x lll, highs x high) carry over.  Band k (1..7) of a high-band
// tensor sits at H + v * h_vs + (k - 1) * C (band-major channels, as
// cwdm_haar_nd writes them); L / H voxel strides in elements (the pyramid's
// all-band conv input is L = g, H = g + C with stride 8 C).
template <typename T>
__global__ void __launch_bounds__(256) haar_nd_synth_kernel(int64_t n, int C, int64_t d, int64_t h, int64_t w,
                                                           const T* __restrict__ L, int64_t l_vs, float lll,
                                                           const T* __restrict__ H, int64_t h_vs, float high,
                                                           T* __restrict__ fine, int acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int G = C / 8, g = (int)(i % G);
  const int64_t cv = i / G, nv = d * h * w;
  const int64_t b = cv / nv, v = cv - b * nv;
  const int64_t x = v % w, y = (v / w) % h, z = v / (w * h);
  float band[8][8];
  load8(L + cv * l_vs + g * 8, band[0]);
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    if (H) load8(H + cv * h_vs + (k - 1) * C + g * 8, band[k]);
    else {
#pragma unroll
      for (int e = 0; e < 8; ++e) band[k][e] = 0.f;
    }
  }
  float blk[8][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float o[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = band[k][e] * (k == 0 ? lll : high);
    haar_inv8(o, r);
#pragma unroll
    for (int q = 0; q < 8; ++q) blk[q][e] = r[q];
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int pa = q >> 2, pb = (q >> 1) & 1, pc = q & 1;
    T* f = fine + (((b * 2 * d + 2 * z + pa) * 2 * h + 2 * y + pb) * 2 * w + 2 * x + pc) * C + g * 8;
    if (acc) {
      float o[8];
      load8(f, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) blk[q][e] += o[e];
    }
    store8(f, blk[q]);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) haar_nd_anal_kernel(int64_t n, int C, int64_t d, int64_t h, int64_t w,
                                                          const T* __restrict__ fine, T* __restrict__ L, int64_t l_vs,
                                                          float lll, int accL, T* __restrict__ H, int64_t h_vs,
                                                          float high, int accH) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int G = C / 8, g = (int)(i % G);
  const int64_t cv = i / G, nv = d * h * w;
  const int64_t b = cv / nv, v = cv - b * nv;
  const int64_t x = v % w, y = (v / w) % h, z = v / (w * h);
  float blk[8][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int pa = q >> 2, pb = (q >> 1) & 1, pc = q & 1;
    load8(fine + (((b * 2 * d + 2 * z + pa) * 2 * h + 2 * y + pb) * 2 * w + 2 * x + pc) * C + g * 8, blk[q]);
  }
  float band[8][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float vin[8], o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) vin[q] = blk[q][e];
    haar_fwd8(vin, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) band[k][e] = o[k] * (k == 0 ? lll : high);
  }
  if (L) {
    T* p = L + cv * l_vs + g * 8;
    if (accL) {
      float o[8];
      load8(p, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) band[0][e] += o[e];
    }
    store8(p, band[0]);
  }
  if (H) {
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      T* p = H + cv * h_vs + (k - 1) * C + g * 8;
      if (accH) {
        float o[8];
        load8(p, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) band[k][e] += o[e];
      }
      store8(p, band[k]);
    }
  }
}

}  // namespace

int haar_nd_synth_add(int dtype, int64_t B, int64_t d, int64_t h, int64_t w, int C, const void* L, int64_t l_vs,
                      float lll, const void* H, int64_t h_vs, float high, void* fine, int acc, hipStream_t s) {
  CWDM_REQUIRE(L && fine && C % 8 == 0 && dtype_compute(dtype), CWDM_E_INVALID, "haar_nd_synth_add: bad argument");
  const int64_t n = B * d * h * w * (C / 8);
  return dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL(haar_nd_synth_kernel<T>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, n, C, d, h, w,
                       reinterpret_cast<const T*>(L), l_vs, lll, reinterpret_cast<const T*>(H), h_vs, high,
                       reinterpret_cast<T*>(fine), acc);
    CWDM_LAUNCHED();
    return CWDM_OK;
  });
}

int haar_nd_anal_add(int dtype, int64_t B, int64_t d, int64_t h, int64_t w, int C, const void* fine, void* L,
                     int64_t l_vs, float lll, int accL, void* H, int64_t h_vs, float high, int accH, hipStream_t s) {
  CWDM_REQUIRE(fine && (L || H) && C % 8 == 0 && dtype_compute(dtype), CWDM_E_INVALID,
               "haar_nd_anal_add: bad argument");
  const int64_t n = B * d * h * w * (C / 8);
  return dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL(haar_nd_anal_kernel<T>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, n, C, d, h, w,
                       reinterpret_cast<const T*>(fine), reinterpret_cast<T*>(L), l_vs, lll, accL,
                       reinterpret_cast<T*>(H), h_vs, high, accH);
    CWDM_LAUNCHED();
    return CWDM_OK;
  });
}

}  // namespace cwdm

using namespace cwdm;

extern "C" int64_t cwdm_haar_nd_parts(int64_t d, int64_t h, int64_t w) { return ceil_div(d * h * w, kVox); }

extern "C" int cwdm_haar_nd(const cwdm_haar_nd_desc* a, cwdm_stream_t stream) {
  CWDM_REQUIRE(a && a->src && a->out, CWDM_E_INVALID, "cwdm_haar_nd: null pointer");
  CWDM_REQUIRE(dtype_compute(a->dtype), CWDM_E_INVALID, "cwdm_haar_nd: bad dtype");
  CWDM_REQUIRE(a->B > 0 && a->d > 0 && a->h > 0 && a->w > 0, CWDM_E_SHAPE, "cwdm_haar_nd: empty grid");
  CWDM_REQUIRE(a->C > 0 && a->C % 8 == 0 && a->C <= 2048, CWDM_E_UNSUPPORTED,
               "cwdm_haar_nd: channels must be a multiple of 8, at most 2048");
  CWDM_REQUIRE(!a->inverse || a->high_in, CWDM_E_INVALID, "cwdm_haar_nd: synthesis needs the 7 high bands");
  CWDM_REQUIRE(!(a->all8 && (a->stats || a->bias)), CWDM_E_UNSUPPORTED,
               "cwdm_haar_nd: all-band output takes no bias / statistics");
  const int parts = (int)cwdm_haar_nd_parts(a->d, a->h, a->w);
  const dim3 grid((unsigned)(a->B * parts));
  hipStream_t s = (hipStream_t)stream;
  dispatch_dtype(a->dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if (a->inverse) hipLaunchKernelGGL((haar_nd_kernel<T, true>), grid, dim3(256), 0, s, *a, parts);
    else hipLaunchKernelGGL((haar_nd_kernel<T, false>), grid, dim3(256), 0, s, *a, parts);
    return CWDM_OK;
  });
  CWDM_LAUNCHED();
  return CWDM_OK;
}
