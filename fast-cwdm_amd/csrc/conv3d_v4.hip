// Host side of the DMA-staged conv3d (conv3d_v4.hpp) and its pre-passes:
//   * cwdm_gn_apply: SiLU(GroupNorm(x)) of one or two channels-last sources
//     written once into a workspace tensor (the conv then stages raw copies),
//   * the 1x1 skip segment (ResBlock skip_connection) runs first as a B-only
//     conv into a workspace tensor that the 3x3x3 conv adds as its residual.
#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "conv3d_v4.hpp"

namespace cwdm {

template __global__ void conv3d_v4_kernel<bf16_t, 0, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 1, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 0, false>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 1, false>(V4Params);
template __global__ void conv3d_v4_kernel<float, 0, false>(V4Params);
template __global__ void conv3d_v4_kernel<float, 1, false>(V4Params);

namespace {

// one thread per (voxel, 8-channel group): out[v][c] = SiLU(x[v][c] * sc[b][c] + sh[b][c])
// cm: write the chunk-major layout [B][C / CK][V][CK] the DMA-staged conv reads
// as contiguous halo rows (CK = 16 bf16 / 8 fp32 channels = 32 bytes per voxel)
template <typename T>
__global__ void __launch_bounds__(256) gn_apply_kernel(const T* __restrict__ x0, int c0, const T* __restrict__ x1,
                                                      int c1, const float* __restrict__ gn, long long vpb,
                                                      long long n8, T* __restrict__ out, int cm) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int C = c0 + c1, G8 = C >> 3;
  const int g = (int)(i % G8);
  const long long v = i / G8;
  const long long b = v / vpb;
  const int c = g * 8;
  const T* src = c < c0 ? x0 + v * c0 + c : x1 + v * c1 + (c - c0);
  float xv[8];
  if constexpr (sizeof(T) == 2) {
    unpack<bf16_t>(*reinterpret_cast<const u32x4*>(src), xv);
  } else {
    unpack<float>(*reinterpret_cast<const u32x4*>(src), xv);
    unpack<float>(*reinterpret_cast<const u32x4*>(src + 4), xv + 4);
  }
  const float4* g4 = reinterpret_cast<const float4*>(gn + (b * C + c) * 2);
  float y[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float4 s = g4[e];  // (sc, sh) of channels c + 2e, c + 2e + 1
    y[2 * e] = silu(xv[2 * e] * s.x + s.y);
    y[2 * e + 1] = silu(xv[2 * e + 1] * s.z + s.w);
  }
  constexpr int CK = 32 / sizeof(T);
  T* dst = cm ? out + ((b * (C / CK) + c / CK) * vpb + (v - b * vpb)) * CK + (c % CK) : out + v * C + c;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<u32x4*>(dst) = pack<bf16_t>(y);
  } else {
    *reinterpret_cast<u32x4*>(dst) = pack<float>(y);
    *reinterpret_cast<u32x4*>(dst + 4) = pack<float>(y + 4);
  }
}

inline int64_t align256(int64_t n) { return (n + 255) & ~(int64_t)255; }

int64_t src_voxels(const cwdm_conv3d_desc* d) {
  const int64_t V = d->D * d->H * d->W;
  return d->a_mode == 1 ? V / 8 : V;
}

}  // namespace

// kernel-path policy (cwdm_conv3d_set_path): 0 auto, 1 legacy only, 2 DMA kernel wherever the shape allows
std::atomic<int> g_conv_path{[] {
  const char* e = std::getenv("CWDM_CONV_PATH");
  return e ? std::atoi(e) : 0;
}()};

std::atomic<unsigned long long*> g_stamps{nullptr};

bool v4_eligible(const cwdm_conv3d_desc* d) {
  const int path = g_conv_path.load(std::memory_order_relaxed);
  if (path == 1) return false;
  if (d->dtype != CWDM_BF16 && d->dtype != CWDM_F32) return false;
  if (!d->a_w || d->W % 32 || d->H % 4 || d->D % 4 || d->cout % 64) return false;
  if (d->a_mode != 0 && d->a_mode != 1) return false;
  if (d->res_mode < -1 || d->res_mode > 1) return false;
  if (d->out1 && d->out_c0 % 8) return false;
  const int64_t nblk = d->B * (d->W / 32) * (d->H / 4) * (d->D / 4) * (d->cout / 64);
  if (nblk < 512 && path != 2) return false;  // small grids: the split-K brick kernels fill the chip better
  const int esz = d->dtype == CWDM_BF16 ? 2 : 4;
  const int64_t sv = src_voxels(d);
  // the DMA range check works on 32-bit byte offsets per batch
  const int64_t lim = 0xFFFFE000LL;
  if (d->a_gn) return sv * (d->a_c0 + d->a_c1) * esz < lim;
  return sv * d->a_c0 * esz < lim && sv * d->a_c1 * esz < lim;
}

int64_t v4_workspace_bytes(const cwdm_conv3d_desc* d) {
  const int esz = d->dtype == CWDM_BF16 ? 2 : 4;
  int64_t ws = 0;
  if (d->a_gn) ws += align256(d->B * src_voxels(d) * (d->a_c0 + d->a_c1) * esz);
  if (d->b_w) ws += align256(d->B * d->D * d->H * d->W * d->cout * esz);
  return ws;
}

int legacy_conv3d_forward(const cwdm_conv3d_desc* d, cwdm_stream_t stream);

int gn_apply(const void* x0, int c0, const void* x1, int c1, const float* gn, int64_t B, int64_t vpb, int dtype,
             void* out, hipStream_t s, int cm = 0) {
  const int64_t n8 = B * vpb * ((c0 + c1) / 8);
  const dim3 grid((unsigned)ceil_div(n8, 256));
  if (dtype == CWDM_BF16)
    hipLaunchKernelGGL(gn_apply_kernel<bf16_t>, grid, dim3(256), 0, s, reinterpret_cast<const bf16_t*>(x0), c0,
                       reinterpret_cast<const bf16_t*>(x1), c1, gn, (long long)vpb, (long long)n8,
                       reinterpret_cast<bf16_t*>(out), cm);
  else
    hipLaunchKernelGGL(gn_apply_kernel<float>, grid, dim3(256), 0, s, reinterpret_cast<const float*>(x0), c0,
                       reinterpret_cast<const float*>(x1), c1, gn, (long long)vpb, (long long)n8,
                       reinterpret_cast<float*>(out), cm);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

int conv3d_v4_forward(const cwdm_conv3d_desc* d, hipStream_t s) {
  const int esz = d->dtype == CWDM_BF16 ? 2 : 4;
  const int ck = d->dtype == CWDM_BF16 ? 16 : 8;
  unsigned char* ws = reinterpret_cast<unsigned char*>(d->workspace);
  const int64_t SV = src_voxels(d);
  const void* a0 = d->a0;
  const void* a1 = d->a1;
  int c0 = d->a_c0, c1 = d->a_c1;
  int a0_cm = 0;
  int rc;
  if (d->a_gn) {
    void* act = ws;
    ws += align256(d->B * SV * (c0 + c1) * esz);
    if ((rc = gn_apply(a0, c0, a1, c1, d->a_gn, d->B, SV, d->dtype, act, s, 1))) return rc;
    a0 = act; c0 = c0 + c1; a1 = nullptr; c1 = 0;
    a0_cm = 1;
  }
  const void* res = d->res;
  int rmode = d->res_mode;
  if (d->b_w) {
    void* skip = ws;
    cwdm_conv3d_desc e = *d;
    e.a0 = nullptr; e.a1 = nullptr; e.a_c0 = 0; e.a_c1 = 0; e.a_gn = nullptr; e.a_w = nullptr; e.a_mode = 0;
    e.bias = nullptr; e.bias_bstride = 0; e.stats = nullptr;
    e.out = skip; e.out_dtype = d->dtype; e.out1 = nullptr; e.out_c0 = 0; e.accumulate = 0;
    e.workspace = nullptr; e.ws_bytes = 0;
    if ((rc = legacy_conv3d_forward(&e, (cwdm_stream_t)s))) return rc;
    res = skip; rmode = 0;
  }
  V4Params p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W;
  p.tx = p.W / 32; p.ty = p.H / 4; p.tz = p.D / 4;
  p.cout = d->cout; p.nct = d->cout / 64;
  p.nch0 = c0 / ck; p.nch = (c0 + c1) / ck;
  p.a0 = a0; p.ac0 = c0; p.a1 = a1; p.ac1 = c1;
  p.a0_bstride = SV * c0 * esz; p.a1_bstride = SV * c1 * esz;
  p.a0_bytes = (unsigned)(SV * c0 * esz); p.a1_bytes = (unsigned)(SV * c1 * esz);
  p.amode = d->a_mode;
  p.a0_cm = a0_cm;
  p.a0_cvox = (int)SV;
  p.aw = reinterpret_cast<const unsigned char*>(d->a_w);
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.res = res; p.rmode = rmode;
  p.out = d->out;
  p.out_f32 = (d->out_dtype == CWDM_F32 && d->dtype != CWDM_F32) ? 1 : 0;
  p.stats = d->stats;
  p.out1 = d->out1; p.out_c0 = d->out_c0;
  p.accumulate = d->accumulate;
  p.stamps = g_stamps.load(std::memory_order_relaxed);
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz * p.nct;
  p.nblk = (int)nblk;
  // persistent: two workgroups per CU (80 KB LDS, <= 256 registers per lane each)
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  const dim3 grid((unsigned)std::min<long long>(nblk, 2LL * ncu));
  // half a tile: ~17k cycles per chunk and ~12k for the epilogue when shared (tools/conv_stamps.py)
  static const int stagger_env = [] { const char* e = std::getenv("CWDM_CONV_STAGGER"); return e ? std::atoi(e) : -1; }();
  p.stagger_cycles = nblk > 2LL * ncu ? (stagger_env >= 0 ? stagger_env : (p.nch * 17000 + 12000) / 2) : 0;
  const bool fast = !p.out_f32 && !p.accumulate && !p.out1;
  if (d->dtype == CWDM_BF16) {
    if (fast) {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<bf16_t, 1, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v4_kernel<bf16_t, 0, true>), grid, dim3(256), 0, s, p);
    } else {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<bf16_t, 1, false>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v4_kernel<bf16_t, 0, false>), grid, dim3(256), 0, s, p);
    }
  } else {
    if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<float, 1, false>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_v4_kernel<float, 0, false>), grid, dim3(256), 0, s, p);
  }
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_gn_apply(const void* x0, int c0, const void* x1, int c1, const float* gn, int64_t B,
                             int64_t voxels, int dtype, void* out, cwdm_stream_t stream) {
  CWDM_REQUIRE(x0 && gn && out && (c1 == 0 || x1), CWDM_E_INVALID, "cwdm_gn_apply: null pointer");
  CWDM_REQUIRE(c0 > 0 && c0 % 8 == 0 && c1 % 8 == 0 && B > 0 && voxels > 0, CWDM_E_SHAPE,
               "cwdm_gn_apply: channels must be multiples of 8");
  CWDM_REQUIRE(dtype == CWDM_BF16 || dtype == CWDM_F32, CWDM_E_INVALID, "cwdm_gn_apply: bad dtype");
  return gn_apply(x0, c0, x1, c1, gn, B, voxels, dtype, out, (hipStream_t)stream);
}

extern "C" int cwdm_conv3d_set_path(int path) {
  CWDM_REQUIRE(path >= 0 && path <= 2, CWDM_E_INVALID, "cwdm_conv3d_set_path: path must be 0, 1 or 2");
  return g_conv_path.exchange(path);
}

// diagnostics: the DMA-staged conv kernel writes 24 u64 per workgroup (s_memtime
// at start / after the prologue / after each of the first 16 chunks / at the end,
// and HW_ID, XCC_ID) into buf (device memory, >= 24 * workgroups); null disables
extern "C" int cwdm_debug_conv_stamps(void* buf) {
  g_stamps.store(reinterpret_cast<unsigned long long*>(buf));
  return CWDM_OK;
}
