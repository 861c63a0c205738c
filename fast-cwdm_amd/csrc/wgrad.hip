// Conv3d weight gradient on MFMA (the backward of nn.Conv3d's weight,
// guided_diffusion/nn.py:22-32, as torch autograd computes it for
// TrainLoop.forward_backward, guided_diffusion/train_util.py:396-462):
//
//   dW[co][ci][tap] = sum_{b, v} dY[b, v, co] * U[b, v + tap - 1, ci]
//
// a GEMM with M = cout, N = cin (x 27 taps), K = B * voxels.  U is the conv's
// INPUT as the forward saw it -- recomputed on the fly from the saved
// activations by the forward's staging code (GroupNorm scale/shift + SiLU,
// nearest-x2 upsample, two-source concat, zero padding), so nothing but the
// raw activations is kept for the backward.
//
// Work decomposition (one 512-thread workgroup = 8 waves, 1 per CU):
//   * tile = 32*MC output channels x 32 input channels x all taps; K is walked
//     in bricks of 16x4x4 voxels (a range of bricks per workgroup, split over
//     the grid; partial tiles are combined with fp32 atomics).
//   * per brick: waves 0-3 / 4-7 stage the halo of input-channel chunks into
//     LDS (one image per 16-channel chunk, 32-B rows), all threads stage the
//     brick's dY rows [voxel][co].
//   * both MFMA operands need K (voxels) along the lane's 8 elements while
//     LDS rows hold channels: bf16 reads them with the gfx950 transposed LDS
//     read ds_read_b64_tr_b16 (4 voxel rows x 16 channels per 16-lane group),
//     so no transposed copy is ever written.
//   * 3x3x3: wave w owns taps {w, w+8, w+16, w+24}; the dY fragments of a
//     K-step are read once and reused for all its taps.  1x1: the 8 waves split
//     the K-steps instead.
// fp32 (parity mode) runs the same structure on exact-fp32 v_mfma_f32_32x32x2_f32.
#include "conv3d_kernels.hpp"

namespace cwdm {
namespace {

typedef short v4s __attribute__((ext_vector_type(4)));

struct WgradParams {
  ConvParams cp;          // grid + U sources (a* for 3x3x3, b* for 1x1)
  const void* dy;
  int dy_cs, cout, cin, taps;
  float* dw;
  int tx, ty, tz;         // bricks per axis
  long long nbricks;      // B * tx * ty * tz
  long long per;          // bricks per workgroup
  int nco;                // output-channel tiles
};

constexpr int WBX = 16, WBY = 4, WBZ = 4;
constexpr int WHX = WBX + 2, WHY = WBY + 2, WHV = WHX * WHY * (WBZ + 2);
constexpr int WIMG = WHV * 32 + 128;  // +128 B: the two images of a half-wave sit on complementary banks

template <typename T, int MC>
struct WgCfg {
  static constexpr int CK = ConvTr<T>::CK;
  static constexpr int NCH = 32 / CK;                 // chunk images per 32-channel input tile
  static constexpr int CO = 32 * MC;
  static constexpr int DYP = CO * (int)sizeof(T);      // dY row pitch (bytes)
  static constexpr int DY_OFF = NCH * WIMG;
  static constexpr int SMEM = DY_OFF + 256 * DYP;
};

__device__ __forceinline__ v4s tr_read(const unsigned char* lds) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds));
}

__device__ __forceinline__ bf16x8 join(v4s a, v4s b) {
  typedef short v8s __attribute__((ext_vector_type(8)));
  v8s r = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// dY quad swizzle (bf16, 128-B rows): rows 2,3 of every 4 use the other half
// of the row so the 4-row transposed reads of a half-wave hit all 64 banks.
template <typename T, int MC>
__device__ __forceinline__ int dy_quad(int qd, int v) {
  if constexpr (sizeof(T) == 2 && MC == 2) return qd ^ (((v >> 1) & 1) << 2);
  else return qd;
}

template <typename T, int MC>
__device__ __forceinline__ void stage_dy(const WgradParams& p, unsigned char* dyl, int b, int x0, int y0, int z0,
                                         int co0, int tid) {
  using C = WgCfg<T, MC>;
  constexpr int QPV = C::DYP / 16;  // quads per voxel row
  constexpr int EPQ = 16 / (int)sizeof(T);
  constexpr int NQ = 256 * QPV;
#pragma unroll
  for (int j = 0; j < NQ / 512; ++j) {
    const int q = tid + 512 * j;
    const int v = q / QPV, qd = q % QPV;
    const int x = x0 + (v & 15), y = y0 + ((v >> 4) & 3), z = z0 + (v >> 6);
    const int c = co0 + qd * EPQ;
    u32x4 val = u32x4{0u, 0u, 0u, 0u};
    if (x < p.cp.W && y < p.cp.H && z < p.cp.D && c < p.dy_cs) {
      const long long vox = (((long long)b * p.cp.D + z) * p.cp.H + y) * p.cp.W + x;
      val = ldg16(reinterpret_cast<const T*>(p.dy) + vox * p.dy_cs + c);
    }
    *reinterpret_cast<u32x4*>(dyl + v * C::DYP + dy_quad<T, MC>(qd, v) * 16) = val;
  }
}

// halo offset (in rows) of tap t = (kz, ky, kx)
__device__ __forceinline__ int tap_rows(int t) {
  const int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;
  return (kz * WHY + ky) * WHX + kx;
}

template <typename T, int MC, int MODE, bool GN, int TAPS>
__global__ void __launch_bounds__(512) wgrad_kernel(WgradParams p) {
  using C = WgCfg<T, MC>;
  constexpr int CK = C::CK, NCH = C::NCH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* halo = smem;
  unsigned char* dyl = smem + C::DY_OFF;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int half = tid >> 8, htid = tid & 255;
  const int ct = blockIdx.y % p.nco, it = blockIdx.y / p.nco;
  const int co0 = ct * C::CO, ci0 = it * 32;
  const long long bb = (long long)blockIdx.x * p.per;
  const long long be = bb + p.per < p.nbricks ? bb + p.per : p.nbricks;
  constexpr bool SEGA = TAPS == 27;

  // this wave's taps (3x3x3) or K-steps (1x1)
  int ntap, toff[4];
  if constexpr (TAPS == 27) {
    ntap = wv < 3 ? 4 : 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) toff[k] = tap_rows(wv + 8 * k < 27 ? wv + 8 * k : 0);
  } else {
    ntap = 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) toff[k] = tap_rows(13);
  }

  f32x16 acc[4][MC];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int m = 0; m < MC; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[k][m][i] = 0.f;

  Stager<T, WBX, WBY, WBZ, MODE, GN> sg;
  const int nb_vol = p.tx * p.ty * p.tz;
  for (long long bi = bb; bi < be; ++bi) {
    const int b = (int)(bi / nb_vol);
    int r = (int)(bi % nb_vol);
    const int x0 = (r % p.tx) * WBX;
    r /= p.tx;
    const int y0 = (r % p.ty) * WBY;
    const int z0 = (r / p.ty) * WBZ;
    __syncthreads();  // previous brick's reads are done
    sg.cached = false;
#pragma unroll
    for (int c = half; c < NCH; c += 2) {
      sg.fetch(p.cp, SEGA, ci0 / CK + c, b, x0, y0, z0, htid);
      sg.template store<false>(halo + c * WIMG, p.cp, b, x0, y0, z0, htid);
    }
    stage_dy<T, MC>(p, dyl, b, x0, y0, z0, co0, tid);
    __syncthreads();

    if constexpr (sizeof(T) == 2) {
      // lane roles in the transposed reads
      const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = g >> 1;
      const unsigned char* bimg = halo + (g & 1) * WIMG + 8 * pp;
      constexpr int S0 = TAPS == 27 ? 0 : 0;
      const int s_begin = TAPS == 27 ? 0 : 2 * wv, s_end = TAPS == 27 ? 16 : 2 * wv + 2;
      (void)S0;
      for (int s = s_begin; s < s_end; ++s) {
        const int y = s & 3, z = s >> 2;
        bf16x8 a[MC];
#pragma unroll
        for (int m = 0; m < MC; ++m) {
          const int v0 = 16 * s + 8 * h + q, v1 = v0 + 4;
          const int qd = 4 * m + 2 * (g & 1) + (pp >> 1);
          const v4s lo = tr_read(dyl + v0 * C::DYP + dy_quad<T, MC>(qd, v0) * 16 + 8 * (pp & 1));
          const v4s hi = tr_read(dyl + v1 * C::DYP + dy_quad<T, MC>(qd, v1) * 16 + 8 * (pp & 1));
          a[m] = join(lo, hi);
        }
        const int hrow = (z * WHY + y) * WHX + 8 * h + q;  // halo row of voxel (x=8h+q, y, z) at tap (0,0,0)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < ntap) {
            const unsigned char* bp = bimg + (hrow + toff[k]) * 32;
            const bf16x8 bf = join(tr_read(bp), tr_read(bp + 4 * 32));
#pragma unroll
            for (int m = 0; m < MC; ++m)
              acc[k][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m], bf, acc[k][m], 0, 0, 0);
          }
        }
      }
    } else {
      // fp32: lane holds one K element (voxel 2s + (lane >> 5)) of one row/column
      const int col = lane & 31, hh = lane >> 5;
      const int s_begin = TAPS == 27 ? 0 : 16 * wv, s_end = TAPS == 27 ? 128 : 16 * wv + 16;
      const unsigned char* bimg = halo + (col >> 3) * WIMG + (col & 7) * 4;
      for (int s = s_begin; s < s_end; ++s) {
        const int v = 2 * s + hh;
        const int x = v & 15, y = (v >> 4) & 3, z = v >> 6;
        float a[MC];
#pragma unroll
        for (int m = 0; m < MC; ++m) a[m] = *reinterpret_cast<const float*>(dyl + v * C::DYP + (32 * m + col) * 4);
        const int hrow = (z * WHY + y) * WHX + x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < ntap) {
            const float bv = *reinterpret_cast<const float*>(bimg + (hrow + toff[k]) * 32);
#pragma unroll
            for (int m = 0; m < MC; ++m)
              acc[k][m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m], bv, acc[k][m], 0, 0, 0);
          }
        }
      }
    }
  }

  // combine: fp32 atomics into dW[co][ci][tap]
  const int ci = ci0 + (lane & 31);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < ntap) {
      const int tap = TAPS == 27 ? wv + 8 * k : 0;
#pragma unroll
      for (int m = 0; m < MC; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int co = co0 + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          if (co < p.cout && ci < p.cin)
            atomicAdd(p.dw + ((long long)co * p.cin + ci) * TAPS + tap, acc[k][m][i]);
        }
    }
  }
}

template <typename T, int MC, int MODE, bool GN, int TAPS>
int launch_wg(const WgradParams& p, dim3 grid, hipStream_t s) {
  constexpr int smem = WgCfg<T, MC>::SMEM;
  static_assert(smem <= 160 * 1024, "wgrad LDS");
  auto k = wgrad_kernel<T, MC, MODE, GN, TAPS>;
  CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  hipLaunchKernelGGL(k, grid, dim3(512), smem, s, p);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

template <typename T, int MC>
int dispatch_wg(const WgradParams& p, int mode, bool gn, dim3 grid, hipStream_t s) {
  if (p.taps == 1) return launch_wg<T, MC, 0, false, 1>(p, grid, s);
  if (mode == 1) return gn ? launch_wg<T, MC, 1, true, 27>(p, grid, s) : launch_wg<T, MC, 1, false, 27>(p, grid, s);
  return gn ? launch_wg<T, MC, 0, true, 27>(p, grid, s) : launch_wg<T, MC, 0, false, 27>(p, grid, s);
}

}  // namespace
}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_conv3d_wgrad(const cwdm_wgrad_desc* d, cwdm_stream_t stream) {
  CWDM_REQUIRE(d, CWDM_E_INVALID, "cwdm_conv3d_wgrad: null desc");
  CWDM_REQUIRE(d->u0 && d->dy && d->dw, CWDM_E_INVALID, "cwdm_conv3d_wgrad: null pointer");
  CWDM_REQUIRE(d->dtype == CWDM_F32 || d->dtype == CWDM_BF16, CWDM_E_INVALID, "cwdm_conv3d_wgrad: bad dtype");
  CWDM_REQUIRE(d->ksize == 1 || d->ksize == 3, CWDM_E_UNSUPPORTED, "cwdm_conv3d_wgrad: ksize must be 1 or 3");
  CWDM_REQUIRE(d->B > 0 && d->D > 0 && d->H > 0 && d->W > 0, CWDM_E_SHAPE, "cwdm_conv3d_wgrad: empty grid");
  CWDM_REQUIRE(d->u_c1 == 0 || d->u1, CWDM_E_INVALID, "cwdm_conv3d_wgrad: second source missing");
  const int cin = d->u_c0 + d->u_c1;
  const int epq = d->dtype == CWDM_BF16 ? 8 : 4;
  CWDM_REQUIRE(cin > 0 && cin % 32 == 0 && d->u_c0 % epq == 0, CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_wgrad: input channels must be a multiple of 32 (split on a quad)");
  CWDM_REQUIRE(d->cout > 0 && d->dy_cs >= d->cout && d->dy_cs % epq == 0, CWDM_E_SHAPE,
               "cwdm_conv3d_wgrad: dy channel stride must cover cout and be a multiple of the quad");
  CWDM_REQUIRE(d->u_mode == 0 || (d->u_mode == 1 && d->ksize == 3), CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_wgrad: u_mode must be 0 or 1 (upsample, 3x3x3)");
  CWDM_REQUIRE(d->ksize == 3 || !d->u_gn, CWDM_E_UNSUPPORTED, "cwdm_conv3d_wgrad: GroupNorm prologue needs ksize 3");
  if (d->u_mode == 1)
    CWDM_REQUIRE(d->D % 2 == 0 && d->H % 2 == 0 && d->W % 2 == 0, CWDM_E_SHAPE,
                 "cwdm_conv3d_wgrad: upsampled grid must be even");
  WgradParams p{};
  ConvParams& c = p.cp;
  c.B = (int)d->B; c.D = (int)d->D; c.H = (int)d->H; c.W = (int)d->W;
  if (d->ksize == 3) {
    c.a0 = d->u0; c.ac0 = d->u_c0; c.a1 = d->u1; c.ac1 = d->u_c1; c.amode = d->u_mode; c.agn = d->u_gn;
  } else {
    c.b0 = d->u0; c.bc0 = d->u_c0; c.b1 = d->u1; c.bc1 = d->u_c1;
  }
  p.dy = d->dy; p.dy_cs = d->dy_cs; p.cout = d->cout; p.cin = cin; p.taps = d->ksize == 3 ? 27 : 1; p.dw = d->dw;
  p.tx = (int)ceil_div(d->W, WBX); p.ty = (int)ceil_div(d->H, WBY); p.tz = (int)ceil_div(d->D, WBZ);
  p.nbricks = d->B * (long long)p.tx * p.ty * p.tz;
  // MC = 2 (64-channel tiles) spills at 2 waves/SIMD with the staging state
  // live; 32-channel tiles for now
  const int mc = 1;
  p.nco = (int)ceil_div(d->cout, 32 * mc);
  const long long tiles = (long long)p.nco * (cin / 32);
  long long S = ceil_div(512, tiles);
  if (S > p.nbricks) S = p.nbricks;
  if (S < 1) S = 1;
  p.per = ceil_div(p.nbricks, S);
  S = ceil_div(p.nbricks, p.per);
  CWDM_REQUIRE(tiles < 65536, CWDM_E_SHAPE, "cwdm_conv3d_wgrad: too many channel tiles");
  dim3 grid((unsigned)S, (unsigned)tiles);
  hipStream_t s = (hipStream_t)stream;
  const bool gn = d->u_gn != nullptr;
  if (d->dtype == CWDM_BF16) return dispatch_wg<bf16_t, 1>(p, d->u_mode, gn, grid, s);
  return dispatch_wg<float, 1>(p, d->u_mode, gn, grid, s);
}
