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
                                                         long long voxels, float eps, float* __restrict__ out) {
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
    for (long long pi = threadIdx.x; pi < parts; pi += 256) {
      const long long idx = (((long long)b * parts + pi) * cs + cc) * 2;
      s += (double)src[idx];
      q += (double)src[idx + 1];
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
                                float eps, float* out, cwdm_stream_t stream) {
  CWDM_REQUIRE(s0 && gamma && beta && out, CWDM_E_INVALID, "cwdm_gn_finalize: null pointer");
  CWDM_REQUIRE(c1 == 0 || s1, CWDM_E_INVALID, "cwdm_gn_finalize: second source missing");
  CWDM_REQUIRE(groups > 0 && (c0 + c1) % groups == 0, CWDM_E_SHAPE,
               "cwdm_gn_finalize: channels must be divisible by num_groups");
  CWDM_REQUIRE(B > 0 && B < 65536 && voxels > 0, CWDM_E_SHAPE, "cwdm_gn_finalize: bad batch/voxels");
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(groups, (unsigned)B), dim3(256), 0, (hipStream_t)stream, s0,
                     (long long)p0, c0, s1, (long long)p1, c1, gamma, beta, groups, (long long)voxels, eps, out);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
