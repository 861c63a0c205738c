// Strided (b, c, v) copy with dtype conversion, tiled through LDS so that
// both the channel-planar (NCDHW) and the channels-last (NDHWC) side are
// accessed with consecutive lanes on consecutive addresses.
#include "common.hpp"

namespace cwdm {
namespace {

constexpr int TV = 64;  // voxels per tile
constexpr int TC = 32;  // channels per tile

template <typename T>
__device__ __forceinline__ float ldf(const void* p, int64_t o) {
  return Elem<T>::to_f(reinterpret_cast<const T*>(p)[o]);
}
template <typename T>
__device__ __forceinline__ void stf(void* p, int64_t o, float v) {
  reinterpret_cast<T*>(p)[o] = Elem<T>::from_f(v);
}

template <typename SrcT, typename DstT>
__global__ void __launch_bounds__(256) copy3_kernel(const void* __restrict__ src, int64_t sb, int64_t sc,
                                                   int64_t sv, void* __restrict__ dst, int64_t db, int64_t dc,
                                                   int64_t dv, int64_t C, int64_t V) {
  __shared__ float tile[TC][TV + 1];
  const int64_t v0 = (int64_t)blockIdx.x * TV, c0 = (int64_t)blockIdx.y * TC, b = blockIdx.z;
  const int tid = threadIdx.x;
  // read: lanes along v (channel-planar friendly)
  {
    int vl = tid & (TV - 1);
    for (int cl = tid >> 6; cl < TC; cl += 4) {
      int64_t c = c0 + cl, v = v0 + vl;
      float x = 0.f;
      if (c < C && v < V) x = ldf<SrcT>(src, b * sb + c * sc + v * sv);
      tile[cl][vl] = x;
    }
  }
  __syncthreads();
  // write: lanes along c (channels-last friendly)
  {
    int cl = tid & (TC - 1);
    for (int vl = tid >> 5; vl < TV; vl += 8) {
      int64_t c = c0 + cl, v = v0 + vl;
      if (c < C && v < V) stf<DstT>(dst, b * db + c * dc + v * dv, tile[cl][vl]);
    }
  }
}

template <typename SrcT>
int launch_dst(const void* src, const int64_t* s, void* dst, int ddt, const int64_t* d, int64_t B, int64_t C,
               int64_t V, hipStream_t st) {
  dim3 grid((unsigned)ceil_div(V, TV), (unsigned)ceil_div(C, TC), (unsigned)B);
  if (ddt == CWDM_F32)
    hipLaunchKernelGGL((copy3_kernel<SrcT, float>), grid, dim3(256), 0, st, src, s[0], s[1], s[2], dst, d[0], d[1],
                       d[2], C, V);
  else if (ddt == CWDM_BF16)
    hipLaunchKernelGGL((copy3_kernel<SrcT, bf16_t>), grid, dim3(256), 0, st, src, s[0], s[1], s[2], dst, d[0], d[1],
                       d[2], C, V);
  else if (ddt == CWDM_F16)
    hipLaunchKernelGGL((copy3_kernel<SrcT, f16_t>), grid, dim3(256), 0, st, src, s[0], s[1], s[2], dst, d[0], d[1],
                       d[2], C, V);
  else
    return fail(CWDM_E_INVALID, "cwdm_copy3: bad dst dtype");
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace
}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_copy3(const void* src, int sdt, const int64_t* s, void* dst, int ddt, const int64_t* d,
                          int64_t B, int64_t C, int64_t V, cwdm_stream_t stream) {
  CWDM_REQUIRE(src && dst && s && d, CWDM_E_INVALID, "cwdm_copy3: null pointer");
  if (B <= 0 || C <= 0 || V <= 0) return CWDM_OK;
  CWDM_REQUIRE(B < 65536 && ceil_div(C, TC) < 65536, CWDM_E_UNSUPPORTED, "cwdm_copy3: grid too large");
  if (sdt == CWDM_F32) return launch_dst<float>(src, s, dst, ddt, d, B, C, V, (hipStream_t)stream);
  if (sdt == CWDM_BF16) return launch_dst<bf16_t>(src, s, dst, ddt, d, B, C, V, (hipStream_t)stream);
  if (sdt == CWDM_F16) return launch_dst<f16_t>(src, s, dst, ddt, d, B, C, V, (hipStream_t)stream);
  return fail(CWDM_E_INVALID, "cwdm_copy3: bad src dtype");
}
