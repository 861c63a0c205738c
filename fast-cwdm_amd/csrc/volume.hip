// BraTS volume front end on the device, the step
// before the wavelet path:
//   clip_and_normalize (guided_diffusion/bratsloader.py:116-120): np.quantile
//   ('linear') at 0.001 / 0.999 from exact order statistics, np.clip, min-max
//   normalisation in float64; then the fp32 cast, the z pad 155 -> 160 and
//   the 8-voxel x/y crop of BRATSVolumes.__getitem__ (bratsloader.py:44-50).
//
// Order statistics: LSD-free radix select over 64-bit order-preserving keys
// of the float64 values, 11-bit digits (6 passes), up to 4 ranks at once.
// Per pass one histogram launch (LDS histograms of the elements still
// matching each rank's prefix, merged with global atomics) and one
// single-workgroup scan launch that fixes the next digit of every rank.  All
// state lives in the caller's workspace, so the sequence is graph-capturable.
// Byte work: 6 reads of the volume (8.9 M float64 = 71 MB for BraTS); HBM-bound.
#include <algorithm>

#include "common.hpp"

namespace cwdm {
namespace {

constexpr int RS_BITS = 11, RS_BINS = 1 << RS_BITS, RS_PASSES = 6;
constexpr int RS_MAXR = 4;

struct SelState {
  unsigned long long prefix[RS_MAXR];
  unsigned long long mask[RS_MAXR];
  long long k[RS_MAXR];
};

__device__ __forceinline__ unsigned long long okey(double v) {
  const unsigned long long b = __double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unkey(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double(b);
}

template <typename T>
__device__ __forceinline__ double ldd(const T* x, long long i) { return (double)x[i]; }

__device__ __forceinline__ void digit_of(int pass, int* shift, int* width) {
  const int top = 64 - RS_BITS * pass;  // bits [top - width, top)
  *width = top < RS_BITS ? top : RS_BITS;
  *shift = top - *width;
}

__global__ void sel_init_kernel(SelState* st, unsigned* hist, int nr, long long k0, long long k1, long long k2,
                                long long k3) {
  const long long ks[4] = {k0, k1, k2, k3};
  for (int i = threadIdx.x; i < nr * RS_BINS; i += blockDim.x) hist[i] = 0u;
  if (threadIdx.x < RS_MAXR) {
    st->prefix[threadIdx.x] = 0ull;
    st->mask[threadIdx.x] = 0ull;
    st->k[threadIdx.x] = ks[threadIdx.x];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) sel_hist_kernel(const T* __restrict__ x, long long n, int nr, int pass,
                                                       const SelState* __restrict__ st, unsigned* __restrict__ hist) {
  __shared__ unsigned h[RS_MAXR * RS_BINS];
  for (int i = threadIdx.x; i < nr * RS_BINS; i += 256) h[i] = 0u;
  unsigned long long pre[RS_MAXR], msk[RS_MAXR];
#pragma unroll
  for (int r = 0; r < RS_MAXR; ++r) {
    pre[r] = st->prefix[r];
    msk[r] = st->mask[r];
  }
  int shift, width;
  digit_of(pass, &shift, &width);
  const unsigned dmask = (1u << width) - 1u;
  __syncthreads();
  // per-lane run-length of the last bin hit: the zero background of a brain
  // volume would otherwise serialise on one LDS address
  unsigned last[RS_MAXR], cnt[RS_MAXR];
#pragma unroll
  for (int r = 0; r < RS_MAXR; ++r) { last[r] = 0u; cnt[r] = 0u; }
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const unsigned long long k = okey(ldd(x, i));
    const unsigned dg = (unsigned)(k >> shift) & dmask;
#pragma unroll
    for (int r = 0; r < RS_MAXR; ++r) {
      if (r < nr && (k & msk[r]) == pre[r]) {
        if (dg == last[r]) {
          ++cnt[r];
        } else {
          if (cnt[r]) atomicAdd(&h[r * RS_BINS + last[r]], cnt[r]);
          last[r] = dg;
          cnt[r] = 1u;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RS_MAXR; ++r)
    if (cnt[r]) atomicAdd(&h[r * RS_BINS + last[r]], cnt[r]);
  __syncthreads();
  for (int i = threadIdx.x; i < nr * RS_BINS; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// one workgroup per rank: the bin holding rank k, then k -= elements below it
__global__ void __launch_bounds__(256) sel_scan_kernel(SelState* st, unsigned* hist, int pass) {
  const int r = blockIdx.x, t = threadIdx.x;
  __shared__ unsigned long long part[256];
  __shared__ unsigned c[RS_BINS];
  unsigned* hr = hist + r * RS_BINS;
  unsigned long long s = 0;
  for (int j = 0; j < RS_BINS / 256; ++j) {
    const unsigned v = hr[t * (RS_BINS / 256) + j];
    c[t * (RS_BINS / 256) + j] = v;
    s += v;
  }
  part[t] = s;
  __syncthreads();
  for (int i = t; i < RS_BINS; i += 256) hr[i] = 0u;  // ready for the next pass
  if (t == 0) {
    long long k = st->k[r];
    int seg = 0;
    while (seg < 255 && (long long)part[seg] <= k) { k -= (long long)part[seg]; ++seg; }
    int bin = seg * (RS_BINS / 256);
    while (bin < (seg + 1) * (RS_BINS / 256) - 1 && (long long)c[bin] <= k) { k -= (long long)c[bin]; ++bin; }
    int shift, width;
    digit_of(pass, &shift, &width);
    st->prefix[r] |= (unsigned long long)bin << shift;
    st->mask[r] |= (unsigned long long)((1u << width) - 1u) << shift;
    st->k[r] = k;
  }
}

// numpy's 'linear' interpolation between the order statistics (lo, hi) of
// each quantile: _lerp (numpy/lib/_function_base_impl.py) in float64
__global__ void sel_lerp_kernel(const SelState* st, int nq, double g0, double g1, double* out) {
  const int i = threadIdx.x;
  if (i >= nq) return;
  const double g = i == 0 ? g0 : g1;
  const double a = unkey(st->prefix[2 * i]), b = unkey(st->prefix[2 * i + 1]);
  const double diff = b - a;
  double r = a + diff * g;
  if (g >= 0.5) r = b - diff * (1.0 - g);
  out[i] = r;
}

// out[i][j][k] = k < Z ? (clip(x[i + crop][j + crop][k], lo, hi) - lo) / (hi - lo) : 0
template <typename T, typename O>
__global__ void __launch_bounds__(256) prepare_kernel(const T* __restrict__ x, long long X, long long Y, long long Z,
                                                      const double* __restrict__ lohi, long long crop,
                                                      long long OZ, O* __restrict__ out) {
  const long long OX = X - 2 * crop, OY = Y - 2 * crop;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= OX * OY * OZ) return;
  const long long k = i % OZ, j = (i / OZ) % OY, a = i / (OZ * OY);
  double r = 0.0;
  if (k < Z) {
    const double lo = lohi[0], hi = lohi[1];
    double v = ldd(x, ((a + crop) * Y + (j + crop)) * Z + k);
    v = v > lo ? v : lo;   // np.clip = minimum(maximum(x, lo), hi)
    v = v < hi ? v : hi;
    r = (v - lo) / (hi - lo);
  }
  out[i] = (O)r;
}

}  // namespace
}  // namespace cwdm

using namespace cwdm;

extern "C" int64_t cwdm_quantile_workspace_bytes(void) {
  return (int64_t)sizeof(SelState) + 256 + (int64_t)RS_MAXR * RS_BINS * 4;
}

extern "C" int cwdm_quantiles(const void* x, int dtype, int64_t n, const int64_t* ranks, int nranks,
                              const double* gammas, double* out, void* workspace, int64_t ws_bytes,
                              cwdm_stream_t stream) {
  CWDM_REQUIRE(x && ranks && gammas && out && workspace, CWDM_E_INVALID, "cwdm_quantiles: null pointer");
  CWDM_REQUIRE(dtype == CWDM_F32 || dtype == CWDM_F64, CWDM_E_INVALID, "cwdm_quantiles: fp32 or fp64 input");
  CWDM_REQUIRE(n > 0 && (nranks == 2 || nranks == 4), CWDM_E_SHAPE, "cwdm_quantiles: 1 or 2 quantiles");
  CWDM_REQUIRE(ws_bytes >= cwdm_quantile_workspace_bytes(), CWDM_E_WORKSPACE, "cwdm_quantiles: workspace too small");
  for (int r = 0; r < nranks; ++r)
    CWDM_REQUIRE(ranks[r] >= 0 && ranks[r] < n, CWDM_E_INDEX, "cwdm_quantiles: rank out of range");
  hipStream_t s = (hipStream_t)stream;
  SelState* st = reinterpret_cast<SelState*>(workspace);
  unsigned* hist = reinterpret_cast<unsigned*>(reinterpret_cast<unsigned char*>(workspace) + sizeof(SelState) + 256);
  long long k[4] = {0, 0, 0, 0};
  for (int r = 0; r < nranks; ++r) k[r] = ranks[r];
  hipLaunchKernelGGL(sel_init_kernel, dim3(1), dim3(256), 0, s, st, hist, nranks, k[0], k[1], k[2], k[3]);
  CWDM_LAUNCHED();
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(n, 256 * 16), 1024));
  for (int pass = 0; pass < RS_PASSES; ++pass) {
    if (dtype == CWDM_F64)
      hipLaunchKernelGGL(sel_hist_kernel<double>, grid, dim3(256), 0, s, reinterpret_cast<const double*>(x),
                         (long long)n, nranks, pass, st, hist);
    else
      hipLaunchKernelGGL(sel_hist_kernel<float>, grid, dim3(256), 0, s, reinterpret_cast<const float*>(x),
                         (long long)n, nranks, pass, st, hist);
    CWDM_LAUNCHED();
    hipLaunchKernelGGL(sel_scan_kernel, dim3(nranks), dim3(256), 0, s, st, hist, pass);
    CWDM_LAUNCHED();
  }
  hipLaunchKernelGGL(sel_lerp_kernel, dim3(1), dim3(64), 0, s, st, nranks / 2, gammas[0],
                     nranks == 4 ? gammas[1] : 0.0, out);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int cwdm_volume_prepare(const void* x, int dtype, int64_t X, int64_t Y, int64_t Z, const double* lohi,
                                   int64_t crop, int64_t out_z, void* out, int out_dtype, cwdm_stream_t stream) {
  CWDM_REQUIRE(x && lohi && out, CWDM_E_INVALID, "cwdm_volume_prepare: null pointer");
  CWDM_REQUIRE(dtype == CWDM_F32 || dtype == CWDM_F64, CWDM_E_INVALID, "cwdm_volume_prepare: fp32 or fp64 input");
  CWDM_REQUIRE(out_dtype == CWDM_F32 || out_dtype == CWDM_F64, CWDM_E_INVALID,
               "cwdm_volume_prepare: fp32 or fp64 output");
  CWDM_REQUIRE(X > 2 * crop && Y > 2 * crop && Z > 0 && crop >= 0 && out_z >= Z, CWDM_E_SHAPE,
               "cwdm_volume_prepare: bad crop / pad");
  const int64_t n = (X - 2 * crop) * (Y - 2 * crop) * out_z;
  const dim3 grid((unsigned)ceil_div(n, 256));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CWDM_F64 && out_dtype == CWDM_F32)
    hipLaunchKernelGGL((prepare_kernel<double, float>), grid, dim3(256), 0, s, reinterpret_cast<const double*>(x),
                       (long long)X, (long long)Y, (long long)Z, lohi, (long long)crop, (long long)out_z,
                       reinterpret_cast<float*>(out));
  else if (dtype == CWDM_F64)
    hipLaunchKernelGGL((prepare_kernel<double, double>), grid, dim3(256), 0, s, reinterpret_cast<const double*>(x),
                       (long long)X, (long long)Y, (long long)Z, lohi, (long long)crop, (long long)out_z,
                       reinterpret_cast<double*>(out));
  else if (out_dtype == CWDM_F32)
    hipLaunchKernelGGL((prepare_kernel<float, float>), grid, dim3(256), 0, s, reinterpret_cast<const float*>(x),
                       (long long)X, (long long)Y, (long long)Z, lohi, (long long)crop, (long long)out_z,
                       reinterpret_cast<float*>(out));
  else
    hipLaunchKernelGGL((prepare_kernel<float, double>), grid, dim3(256), 0, s, reinterpret_cast<const float*>(x),
                       (long long)X, (long long)Y, (long long)Z, lohi, (long long)crop, (long long)out_z,
                       reinterpret_cast<double*>(out));
  CWDM_LAUNCHED();
  return CWDM_OK;
}
