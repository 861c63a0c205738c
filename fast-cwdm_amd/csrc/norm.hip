// GroupNorm32 finalize: per-tile (sum, sum^2) partials from the producing
// conv epilogue(s) -> per-(b, c) (scale, shift) so that the consumer's
// prologue computes SiLU(GN(x)) = SiLU(x * scale + shift)
// (guided_diffusion/nn.py:17-19 + torch.nn.GroupNorm, eps inside the sqrt,
// biased variance).  Reduction over tiles is done in fp64.
#include "common.hpp"

namespace cwdm {
namespace {

__global__ void __launch_bounds__(256) gn_finalize_kernel(const float* __restrict__ s0, long long p0, int c0,
                                                         const float* __restrict__ s1, long long p1, int c1,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, int groups,
                                                         long long voxels, float eps, float* __restrict__ out,
                                                         float* __restrict__ mean_rstd) {
  const int g = blockIdx.x, b = blockIdx.y;
  const int C = c0 + c1, cpg = C / groups;
  __shared__ double rs[256], rq[256];
  double s = 0.0, q = 0.0;
  // items: (channel-in-group, part)
  for (int ci = 0; ci < cpg; ++ci) {
    const int c = g * cpg + ci;
    const float* src;
    long long parts;
    int cc, cs;
    if (c < c0) { src = s0; parts = p0; cc = c; cs = c0; }
    else { src = s1; parts = p1; cc = c - c0; cs = c1; }
    // (sum, sum^2) pairs of part pi at base[pi * cs]; four parts per thread in
    // flight per iteration (the loads are independent, the adds are fp64)
    const float2* base = reinterpret_cast<const float2*>(src) + (long long)b * parts * cs + cc;
    long long pi = threadIdx.x;
    for (; pi + 768 < parts; pi += 1024) {
      const float2 u0 = base[pi * cs], u1 = base[(pi + 256) * cs], u2 = base[(pi + 512) * cs],
                   u3 = base[(pi + 768) * cs];
      s += ((double)u0.x + (double)u1.x) + ((double)u2.x + (double)u3.x);
      q += ((double)u0.y + (double)u1.y) + ((double)u2.y + (double)u3.y);
    }
    for (; pi < parts; pi += 256) {
      const float2 u = base[pi * cs];
      s += (double)u.x;
      q += (double)u.y;
    }
  }
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      rs[threadIdx.x] += rs[threadIdx.x + o];
      rq[threadIdx.x] += rq[threadIdx.x + o];
    }
    __syncthreads();
  }
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
  for (int ci = threadIdx.x; ci < cpg; ci += 256) {
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
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(groups, (unsigned)B), dim3(256), 0, (hipStream_t)stream, s0,
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
template <typename T>
__global__ void __launch_bounds__(256) gn_silu_pool_kernel(const T* __restrict__ x, int C,
                                                          const float* __restrict__ gn, long long B, int d, int h,
                                                          int w, T* __restrict__ oh, T* __restrict__ ox) {
  const int G8 = C / 8;
  const long long n = B * (long long)d * h * w * G8;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int g = (int)(i % G8);
  long long v = i / G8;
  const int xx = (int)(v % w), yy = (int)((v / w) % h), zz = (int)((v / ((long long)w * h)) % d);
  const long long b = v / ((long long)w * h * d);
  float sc[8], sh[8], ah[8], ax[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = gn[(b * C + g * 8 + e) * 2];
    sh[e] = gn[(b * C + g * 8 + e) * 2 + 1];
    ah[e] = 0.f;
    ax[e] = 0.f;
  }
  const int H = 2 * h, W = 2 * w, D = 2 * d;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const long long src = (((b * D + 2 * zz + (k >> 2)) * H + 2 * yy + ((k >> 1) & 1)) * W + 2 * xx + (k & 1)) * C + g * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xv = Elem<T>::to_f(x[src + e]);
      const float y = xv * sc[e] + sh[e];
      ah[e] += y / (1.0f + __expf(-y));
      ax[e] += xv;
    }
  }
  const long long dst = v * C + g * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    oh[dst + e] = Elem<T>::from_f(ah[e] * 0.125f);
    ox[dst + e] = Elem<T>::from_f(ax[e] * 0.125f);
  }
}
}  // namespace
}  // namespace cwdm

extern "C" int cwdm_gn_silu_pool(const void* x, int C, const float* gn, int64_t B, int64_t d, int64_t h, int64_t w,
                                 int dtype, void* out_h, void* out_x, cwdm_stream_t stream) {
  CWDM_REQUIRE(x && gn && out_h && out_x, CWDM_E_INVALID, "cwdm_gn_silu_pool: null pointer");
  CWDM_REQUIRE(C > 0 && C % 8 == 0 && B > 0 && d > 0 && h > 0 && w > 0, CWDM_E_SHAPE,
               "cwdm_gn_silu_pool: bad shape (channels must be a multiple of 8)");
  const int64_t n = B * d * h * w * (C / 8);
  dim3 grid((unsigned)ceil_div(n, 256));
  if (dtype == CWDM_BF16)
    hipLaunchKernelGGL(gn_silu_pool_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const bf16_t*>(x), C, gn, (long long)B, (int)d, (int)h, (int)w,
                       reinterpret_cast<bf16_t*>(out_h), reinterpret_cast<bf16_t*>(out_x));
  else if (dtype == CWDM_F32)
    hipLaunchKernelGGL(gn_silu_pool_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float*>(x), C, gn, (long long)B, (int)d, (int)h, (int)w,
                       reinterpret_cast<float*>(out_h), reinterpret_cast<float*>(out_x));
  else
    return fail(CWDM_E_INVALID, "cwdm_gn_silu_pool: bad dtype");
  CWDM_LAUNCHED();
  return CWDM_OK;
}
