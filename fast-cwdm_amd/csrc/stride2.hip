// Stride-2 Conv3d (Downsample(use_conv=True), guided_diffusion/unet.py:73-100:
// conv_nd(3, C, C_out, 3, stride=2, padding=1)) on the stride-1 implicit-GEMM
// kernels, by space-to-depth:
//   X'[b][o][ph C + c] = x[b][2 o + p][c],   ph = 4 pz + 2 py + px
// Per axis the stride-2 taps k = 0, 1, 2 read x[2o - 1], x[2o], x[2o + 1] =
// phase 1 of coarse voxel o - 1, phase 0 and phase 1 of voxel o, i.e. a
// stride-1 3x3x3 conv over X' whose tap (d' + 1) and phase p carry weight
// k = 2 d' + p + 1 (d' = 0: k = 1 + p; d' = -1, p = 1: k = 0; zero otherwise).
// The backward reuses the same algebra: dgrad = the stride-1 dgrad over X'
// followed by depth-to-space; wgrad = the stride-1 wgrad over X' folded back
// onto the 27 original taps (each original weight sits at exactly one
// (phase, tap) of the expanded kernel).
#include "common.hpp"

namespace cwdm {
namespace {

// 16-byte (8 bf16 / fp16 or 4 fp32 channels) copies; C * esize % 16 == 0
template <bool TO_DEPTH, bool ACC, typename T>
__global__ void __launch_bounds__(256) s2d_kernel(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst,
                                                 int C, int64_t B, int64_t d, int64_t h, int64_t w) {
  const int q16 = C * (int)sizeof(T) / 16;        // quads per channel row of one phase
  const int64_t nvox = d * h * w;
  const int64_t n = B * nvox * 8 * q16;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int q = (int)(i % q16);
  int64_t r = i / q16;
  const int ph = (int)(r % 8);
  r /= 8;
  const int64_t o = r % nvox, b = r / nvox;
  const int64_t ox = o % w, oy = (o / w) % h, oz = o / (w * h);
  const int pz = ph >> 2, py = (ph >> 1) & 1, px = ph & 1;
  const int64_t fine = ((b * 2 * d + 2 * oz + pz) * 2 * h + 2 * oy + py) * 2 * w + 2 * ox + px;
  const int64_t coarse_off = ((b * nvox + o) * 8 + ph) * (int64_t)q16 + q;   // in quads
  const int64_t fine_off = fine * q16 + q;
  const int64_t so = TO_DEPTH ? fine_off : coarse_off, dofs = TO_DEPTH ? coarse_off : fine_off;
  uint4 v = reinterpret_cast<const uint4*>(src)[so];
  if (ACC) {
    const uint4 a = reinterpret_cast<const uint4*>(dst)[dofs];
    if constexpr (sizeof(T) == 2) {
      unsigned* pv = reinterpret_cast<unsigned*>(&v);
      const unsigned* pa = reinterpret_cast<const unsigned*>(&a);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pv[k] = pack2<T>(lo2f<T>(pv[k]) + lo2f<T>(pa[k]), hi2f<T>(pv[k]) + hi2f<T>(pa[k]));
    } else {
      float* pv = reinterpret_cast<float*>(&v);
      const float* pa = reinterpret_cast<const float*>(&a);
#pragma unroll
      for (int k = 0; k < 4; ++k) pv[k] += pa[k];
    }
  }
  reinterpret_cast<uint4*>(dst)[dofs] = v;
}

// dw[co][ci][kz ky kx] (+)= dwe[co][ph cin + ci][tz ty tx] at the one (ph, t) that holds each weight
__global__ void __launch_bounds__(256) s2_fold_kernel(const float* __restrict__ dwe, int cout, int cin,
                                                     float* __restrict__ dw, int acc) {
  const int64_t n = (int64_t)cout * cin * 27;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = (int)(i % 27);
  const int ci = (int)((i / 27) % cin), co = (int)(i / (27LL * cin));
  int ph = 0, t = 0;
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) {  // z, y, x
    const int kk = ax == 0 ? k / 9 : (ax == 1 ? (k / 3) % 3 : k % 3);
    const int p = kk == 1 ? 0 : 1, tt = kk == 0 ? 0 : 1;
    ph = ph * 2 + p;
    t = t * 3 + tt;
  }
  const float v = dwe[((int64_t)co * 8 * cin + (int64_t)ph * cin + ci) * 27 + t];
  dw[i] = acc ? dw[i] + v : v;
}

}  // namespace

}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_space_to_depth(const void* x, int C, int64_t B, int64_t d, int64_t h, int64_t w, int dtype,
                                   void* out, int to_depth, int accumulate, cwdm_stream_t stream) {
  CWDM_REQUIRE(x && out, CWDM_E_INVALID, "cwdm_space_to_depth: null pointer");
  CWDM_REQUIRE(dtype_compute(dtype), CWDM_E_INVALID, "cwdm_space_to_depth: bad dtype");
  const int es = dtype_size(dtype);
  CWDM_REQUIRE(C > 0 && (C * es) % 16 == 0 && B > 0 && d > 0 && h > 0 && w > 0, CWDM_E_SHAPE,
               "cwdm_space_to_depth: channels must fill 16-byte rows");
  const int64_t n = B * d * h * w * 8 * (C * es / 16);
  const dim3 grid((unsigned)ceil_div(n, 256));
  auto src = reinterpret_cast<const unsigned char*>(x);
  auto dst = reinterpret_cast<unsigned char*>(out);
  hipStream_t s = (hipStream_t)stream;
#define S2D(TD, AC)                                                                                         \
  if (dtype == CWDM_BF16) hipLaunchKernelGGL((s2d_kernel<TD, AC, bf16_t>), grid, dim3(256), 0, s, src, dst, C, B, d, h, w); \
  else if (dtype == CWDM_F16) hipLaunchKernelGGL((s2d_kernel<TD, AC, f16_t>), grid, dim3(256), 0, s, src, dst, C, B, d, h, w); \
  else hipLaunchKernelGGL((s2d_kernel<TD, AC, float>), grid, dim3(256), 0, s, src, dst, C, B, d, h, w);
  if (to_depth) {
    if (accumulate) { S2D(true, true) } else { S2D(true, false) }
  } else {
    if (accumulate) { S2D(false, true) } else { S2D(false, false) }
  }
#undef S2D
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int cwdm_conv3d_s2_fold_dw(const float* dwe, int cout, int cin, float* dw, int accumulate,
                                      cwdm_stream_t stream) {
  CWDM_REQUIRE(dwe && dw && cout > 0 && cin > 0, CWDM_E_INVALID, "cwdm_conv3d_s2_fold_dw: bad argument");
  const int64_t n = (int64_t)cout * cin * 27;
  hipLaunchKernelGGL(s2_fold_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, dwe, cout,
                     cin, dw, accumulate);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
