// GroupNorm32 finalize: per-tile (sum, sum^2) partials from the producing
// conv epilogue(s) -> per-(b, c) (scale, shift) so that the consumer's
// prologue computes SiLU(GN(x)) = SiLU(x * scale + shift)
// (guided_diffusion/nn.py:17-19 + torch.nn.GroupNorm, eps inside the sqrt,
// biased variance).  Reduction over tiles is done in fp64.
#include "common.hpp"

namespace cwdm {
namespace {

// One workgroup per (group, batch).  The group's (part, channel) items are
// flattened so consecutive threads read consecutive channels of one part row
// and every thread has up to 8 independent loads in flight: a small tensor
// finishes in one load latency, a 128^3 one (4096 parts x 2 channels per
// group) in one round too.
constexpr int FIN_THREADS = 1024;
constexpr int FIN_LOADS = 8;

__device__ __forceinline__ void fin_segment(const float2* __restrict__ base, long long parts, int cs, int lo, int w,
                                            double& s, double& q) {
  // items i = pi * w + ci, channel lo + ci of part pi at base[pi * cs + lo + ci]
  // (32-bit item indices: parts * w is far below 2^32 for any grid the plan admits)
  const unsigned n = (unsigned)(parts * w), uw = (unsigned)w;
  unsigned i = threadIdx.x;
  for (; i + (FIN_LOADS - 1) * FIN_THREADS < n; i += FIN_LOADS * FIN_THREADS) {
    float2 u[FIN_LOADS];
#pragma unroll
    for (int k = 0; k < FIN_LOADS; ++k) {
      const unsigned j = i + k * FIN_THREADS;
      u[k] = base[(long long)(j / uw) * cs + lo + (int)(j % uw)];
    }
#pragma unroll
    for (int k = 0; k < FIN_LOADS; ++k) {
      s += (double)u[k].x;
      q += (double)u[k].y;
    }
  }
  for (; i < n; i += FIN_THREADS) {
    const float2 u = base[(long long)(i / uw) * cs + lo + (int)(i % uw)];
    s += (double)u.x;
    q += (double)u.y;
  }
}

__global__ void __launch_bounds__(FIN_THREADS) gn_finalize_kernel(const float* __restrict__ s0, long long p0, int c0,
                                                                 const float* __restrict__ s1, long long p1, int c1,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, int groups,
                                                                 long long voxels, float eps, float* __restrict__ out,
                                                                 float* __restrict__ mean_rstd) {
  const int g = blockIdx.x, b = blockIdx.y;
  const int C = c0 + c1, cpg = C / groups;
  const int glo = g * cpg, ghi = glo + cpg;
  double s = 0.0, q = 0.0;
  if (glo < c0)  // the group's channels in the first source
    fin_segment(reinterpret_cast<const float2*>(s0) + (long long)b * p0 * c0, p0, c0, glo, min(ghi, c0) - glo, s, q);
  if (ghi > c0)  // ... and in the second (a concatenated input)
    fin_segment(reinterpret_cast<const float2*>(s1) + (long long)b * p1 * c1, p1, c1, max(glo, c0) - c0,
                ghi - max(glo, c0), s, q);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  __shared__ double rs[FIN_THREADS / 64], rq[FIN_THREADS / 64];
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 1; k < FIN_THREADS / 64; ++k) {
      rs[0] += rs[k];
      rq[0] += rq[k];
    }
  }
  __syncthreads();
  const double n = (double)cpg * (double)voxels;
  const double mean = rs[0] / n;
  double var = rq[0] / n - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float meanf = (float)mean;
  if (mean_rstd && threadIdx.x == 0) {
    mean_rstd[((long long)b * groups + g) * 2 + 0] = meanf;
    mean_rstd[((long long)b * groups + g) * 2 + 1] = rstd;
  }
  for (int ci = threadIdx.x; ci < cpg; ci += FIN_THREADS) {
    const int c = g * cpg + ci;
    const float sc = gamma[c] * rstd;
    out[((long long)b * C + c) * 2 + 0] = sc;
    out[((long long)b * C + c) * 2 + 1] = beta[c] - meanf * sc;
  }
}

}  // namespace
}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_gn_finalize(const float* s0, int64_t p0, int c0, const float* s1, int64_t p1, int c1,
                                const float* gamma, const float* beta, int groups, int64_t B, int64_t voxels,
                                float eps, float* out, float* mean_rstd, cwdm_stream_t stream) {
  CWDM_REQUIRE(s0 && gamma && beta && out, CWDM_E_INVALID, "cwdm_gn_finalize: null pointer");
  CWDM_REQUIRE(c1 == 0 || s1, CWDM_E_INVALID, "cwdm_gn_finalize: second source missing");
  CWDM_REQUIRE(groups > 0 && (c0 + c1) % groups == 0, CWDM_E_SHAPE,
               "cwdm_gn_finalize: channels must be divisible by num_groups");
  CWDM_REQUIRE(B > 0 && B < 65536 && voxels > 0, CWDM_E_SHAPE, "cwdm_gn_finalize: bad batch/voxels");
  CWDM_REQUIRE(p0 > 0 && p0 * c0 < (1LL << 31) && (c1 == 0 || (p1 > 0 && p1 * c1 < (1LL << 31))), CWDM_E_SHAPE,
               "cwdm_gn_finalize: bad part count");
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(groups, (unsigned)B), dim3(FIN_THREADS), 0, (hipStream_t)stream, s0,
                     (long long)p0, c0, s1, (long long)p1, c1, gamma, beta, groups, (long long)voxels, eps, out,
                     mean_rstd);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

// Down-ResBlock pre-pass (unet.py:286-291 with Downsample, :73-100):
//   h = AvgPool2(SiLU(GN(x))),  x_upd = AvgPool2(x)
// one thread per (low-res voxel, 8-channel group); the consumer conv then
// runs at the low resolution with no prologue transform.
namespace cwdm {
namespace {
template <typename T> __device__ __forceinline__ void pool_load8(const T* p, float* f);
template <> __device__ __forceinline__ void pool_load8<float>(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
template <> __device__ __forceinline__ void pool_load8<bf16_t>(const bf16_t* p, float* f) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const unsigned u[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(u[i] << 16); f[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u); }
}
template <> __device__ __forceinline__ void pool_load8<f16_t>(const f16_t* p, float* f) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const unsigned u[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = lo2f<f16_t>(u[i]); f[2 * i + 1] = hi2f<f16_t>(u[i]); }
}
template <typename T> __device__ __forceinline__ void pool_store8(T* p, const float* f);
template <> __device__ __forceinline__ void pool_store8<float>(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}
template <> __device__ __forceinline__ void pool_store8<bf16_t>(bf16_t* p, const float* f) {
  uint4 a;
  a.x = (unsigned)f2bf(f[0]) | ((unsigned)f2bf(f[1]) << 16);
  a.y = (unsigned)f2bf(f[2]) | ((unsigned)f2bf(f[3]) << 16);
  a.z = (unsigned)f2bf(f[4]) | ((unsigned)f2bf(f[5]) << 16);
  a.w = (unsigned)f2bf(f[6]) | ((unsigned)f2bf(f[7]) << 16);
  *reinterpret_cast<uint4*>(p) = a;
}
template <> __device__ __forceinline__ void pool_store8<f16_t>(f16_t* p, const float* f) {
  uint4 a;
  a.x = pack2<f16_t>(f[0], f[1]);
  a.y = pack2<f16_t>(f[2], f[3]);
  a.z = pack2<f16_t>(f[4], f[5]);
  a.w = pack2<f16_t>(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = a;
}

// one thread = one 8-channel group of one pooled voxel: 8 16-byte loads (the
// 2x2x2 sources), GroupNorm + SiLU (hardware exp2 / reciprocal, as the conv
// kernels' GroupNorm prologue), 16-byte stores; 32-bit indices with magic
// divisors (host-checked: B * d * h * w * C / 8 < 2^31)
template <typename T>
__global__ void __launch_bounds__(256) gn_silu_pool_kernel(const T* __restrict__ x, int C,
                                                          const float* __restrict__ gn, unsigned n, FastDiv dg8,
                                                          FastDiv dw, FastDiv dh, FastDiv dd, T* __restrict__ oh,
                                                          T* __restrict__ ox) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned v = fdiv(i, dg8);
  const int g = (int)(i - v * dg8.d);
  const unsigned vy = fdiv(v, dw), xx = v - vy * dw.d;
  const unsigned vz = fdiv(vy, dh), yy = vy - vz * dh.d;
  const unsigned b = fdiv(vz, dd), zz = vz - b * dd.d;
  float sc[8], sh[8], ah[8], ax[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = gn[((size_t)b * C + g * 8 + e) * 2];
    sh[e] = gn[((size_t)b * C + g * 8 + e) * 2 + 1];
    ah[e] = 0.f;
    ax[e] = 0.f;
  }
  const unsigned H = 2 * dh.d, W = 2 * dw.d, D = 2 * dd.d;
  float xv[8][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const size_t src = ((((size_t)b * D + 2 * zz + (k >> 2)) * H + 2 * yy + ((k >> 1) & 1)) * W + 2 * xx + (k & 1)) * C +
                       g * 8;
    pool_load8<T>(x + src, xv[k]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float y = xv[k][e] * sc[e] + sh[e];
      ah[e] += y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(y * -1.4426950408889634f));
      ax[e] += xv[k][e];
    }
#pragma unroll
  for (int e = 0; e < 8; ++e) { ah[e] *= 0.125f; ax[e] *= 0.125f; }
  const size_t dst = (size_t)v * C + g * 8;
  pool_store8<T>(oh + dst, ah);
  pool_store8<T>(ox + dst, ax);
}
}  // namespace
}  // namespace cwdm

extern "C" int cwdm_gn_silu_pool(const void* x, int C, const float* gn, int64_t B, int64_t d, int64_t h, int64_t w,
                                 int dtype, void* out_h, void* out_x, cwdm_stream_t stream) {
  CWDM_REQUIRE(x && gn && out_h && out_x, CWDM_E_INVALID, "cwdm_gn_silu_pool: null pointer");
  CWDM_REQUIRE(C > 0 && C % 8 == 0 && B > 0 && d > 0 && h > 0 && w > 0, CWDM_E_SHAPE,
               "cwdm_gn_silu_pool: bad shape (channels must be a multiple of 8)");
  // 16-byte accesses (pool_load8 / pool_store8): every 8-channel group starts on a 16-byte boundary
  CWDM_REQUIRE(((uintptr_t)x | (uintptr_t)out_h | (uintptr_t)out_x) % 16 == 0, CWDM_E_INVALID,
               "cwdm_gn_silu_pool: x, out_h and out_x must be 16-byte aligned");
  const int64_t n = B * d * h * w * (C / 8);
  CWDM_REQUIRE(n < (1LL << 31) - 256, CWDM_E_UNSUPPORTED, "cwdm_gn_silu_pool: more than 2^31 channel groups");
  dim3 grid((unsigned)ceil_div(n, 256));
  const FastDiv dg8 = make_fastdiv((unsigned)(C / 8)), dw = make_fastdiv((unsigned)w), dh = make_fastdiv((unsigned)h),
                dd = make_fastdiv((unsigned)d);
  if (dtype == CWDM_BF16)
    hipLaunchKernelGGL(gn_silu_pool_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const bf16_t*>(x), C, gn, (unsigned)n, dg8, dw, dh, dd,
                       reinterpret_cast<bf16_t*>(out_h), reinterpret_cast<bf16_t*>(out_x));
  else if (dtype == CWDM_F16)
    hipLaunchKernelGGL(gn_silu_pool_kernel<f16_t>, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const f16_t*>(x), C, gn, (unsigned)n, dg8, dw, dh, dd,
                       reinterpret_cast<f16_t*>(out_h), reinterpret_cast<f16_t*>(out_x));
  else if (dtype == CWDM_F32)
    hipLaunchKernelGGL(gn_silu_pool_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float*>(x), C, gn, (unsigned)n, dg8, dw, dh, dd,
                       reinterpret_cast<float*>(out_h), reinterpret_cast<float*>(out_x));
  else
    return fail(CWDM_E_INVALID, "cwdm_gn_silu_pool: bad dtype");
  CWDM_LAUNCHED();
  return CWDM_OK;
}
