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
// Work decomposition (one 256-thread workgroup = 4 waves, one wave per SIMD
// so each wave holds its 7 taps x 64 x 32 fp32 accumulators in AGPRs):
//   * tile = 32*MC output channels x 32 input channels x all taps; K is walked
//     in bricks of 16x4x4 voxels (a range of bricks per workgroup, split over
//     the grid; partial tiles are combined with fp32 atomics).
//   * per brick: the halo of the two 16-channel input chunks (one LDS image
//     each, 32-B rows) and the brick's dY rows [voxel][co] are committed from
//     registers that were loaded while the previous brick's MFMAs ran.
//   * both MFMA operands need K (voxels) along the lane's 8 elements while
//     LDS rows hold channels: bf16 / fp16 read them with the gfx950 transposed LDS
//     read ds_read_b64_tr_b16 (4 voxel rows x 16 channels per 16-lane group),
//     so no transposed copy is ever written.
//   * 3x3x3: wave w owns taps {w, w+4, ..., <27}; the dY fragments of a
//     K-step are read once and reused for all its taps.  1x1: the 4 waves split
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

// two transposed 64-bit reads -> one 8 x 16-bit operand (bf16 or fp16), as
// whole dwords (an element-wise shuffle of the 16-bit lanes made the compiler
// repack every dword with v_lshrrev + v_perm: 48 VALU per K-step)
__device__ __forceinline__ u32x4 join(v4s a, v4s b) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 lo = __builtin_bit_cast(u32x2, a), hi = __builtin_bit_cast(u32x2, b);
  return u32x4{lo.x, lo.y, hi.x, hi.y};
}

// dY quad swizzle (bf16, 128-B rows): rows 2,3 of every 4 use the other half
// of the row so the 4-row transposed reads of a half-wave hit all 64 banks.
template <typename T, int MC>
__device__ __forceinline__ int dy_quad(int qd, int v) {
  if constexpr (sizeof(T) == 2 && MC == 2) return qd ^ (((v >> 1) & 1) << 2);
  else return qd;
}

// halo offset (in rows) of tap t = (kz, ky, kx)
__device__ __forceinline__ int tap_rows(int t) {
  const int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;
  return (kz * WHY + ky) * WHX + kx;
}

template <typename T, int MC, int MODE, bool GN, int TAPS>
__global__ void __launch_bounds__(256) wgrad_kernel(WgradParams p) {
  using C = WgCfg<T, MC>;
  constexpr int CK = C::CK, NCH = C::NCH;
  constexpr int QPV = C::DYP / 16;          // dY quads per voxel row
  constexpr int EPQ = 16 / (int)sizeof(T);
  constexpr bool PF = sizeof(T) == 2;       // register prefetch of the next brick (16-bit types)
  constexpr int NT = TAPS == 27 ? 7 : 1;    // taps per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* halo = smem;
  unsigned char* dyl = smem + C::DY_OFF;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int ct = blockIdx.y % p.nco, it = blockIdx.y / p.nco;
  const int co0 = ct * C::CO, ci0 = it * 32;
  const long long bb = (long long)blockIdx.x * p.per;
  const long long be = bb + p.per < p.nbricks ? bb + p.per : p.nbricks;
  constexpr bool SEGA = TAPS == 27;

  // taps of this wave: w, w+4, w+8, ... (7/7/7/6); 1x1: the waves split the K-steps
  const int ntap = TAPS == 27 ? (wv < 3 ? 7 : 6) : 1;
  int toff[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) toff[k] = TAPS == 27 ? tap_rows(wv + 4 * k < 27 ? wv + 4 * k : 0) : tap_rows(13);

  f32x16 acc[NT][MC];
#pragma unroll
  for (int k = 0; k < NT; ++k)
#pragma unroll
    for (int m = 0; m < MC; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[k][m][i] = 0.f;

  Stager<T, WBX, WBY, WBZ, MODE, GN> sg[NCH];
  u32x4 dyr[QPV];
  const int nb_vol = p.tx * p.ty * p.tz;
  int fb = 0;  // batch index of the fetched brick

  // global -> registers for brick bi (nothing waits here)
  auto fetch = [&](long long bi) {
    const int b = (int)(bi / nb_vol);
    fb = b;
    int r = (int)(bi % nb_vol);
    const int x0 = (r % p.tx) * WBX;
    r /= p.tx;
    const int y0 = (r % p.ty) * WBY;
    const int z0 = (r / p.ty) * WBZ;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      sg[c].cached = false;
      sg[c].template fetch<false>(p.cp, SEGA, ci0 / CK + c, b, x0, y0, z0, tid);
    }
#pragma unroll
    for (int j = 0; j < QPV; ++j) {
      const int q = tid + 256 * j;
      const int v = q / QPV, qd = q % QPV;
      const int x = x0 + (v & 15), y = y0 + ((v >> 4) & 3), z = z0 + (v >> 6);
      const int cc = co0 + qd * EPQ;
      const bool in = x < p.cp.W && y < p.cp.H && z < p.cp.D && cc < p.dy_cs;
      const long long vox = in ? (((long long)b * p.cp.D + z) * p.cp.H + y) * p.cp.W + x : 0;
      const u32x4 val = ldg16(reinterpret_cast<const T*>(p.dy) + vox * p.dy_cs + (in ? cc : 0));
      const unsigned keep = in ? ~0u : 0u;
      dyr[j] = u32x4{val[0] & keep, val[1] & keep, val[2] & keep, val[3] & keep};
    }
  };
  // registers -> LDS (GroupNorm + SiLU / zero padding applied here)
  auto commit = [&]() {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (GN && SEGA) sg[c].load_gn(p.cp, ci0 / CK + c, fb, tid);
      sg[c].transform();
      sg[c].template write<false>(halo + c * WIMG, tid);
    }
#pragma unroll
    for (int j = 0; j < QPV; ++j) {
      const int q = tid + 256 * j;
      const int v = q / QPV, qd = q % QPV;
      *reinterpret_cast<u32x4*>(dyl + v * C::DYP + dy_quad<T, MC>(qd, v) * 16) = dyr[j];
    }
  };

  if (PF && bb < be) fetch(bb);
  for (long long bi = bb; bi < be; ++bi) {
    __syncthreads();  // previous brick's LDS reads are done
    if (!PF) fetch(bi);
    commit();
    __syncthreads();
    if (PF && bi + 1 < be) fetch(bi + 1);  // next brick's loads fly during the MFMAs

    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = g >> 1;
      const unsigned char* bimg = halo + (g & 1) * WIMG + 8 * pp;
      constexpr int NS = TAPS == 27 ? 16 : 4;   // K-steps of this wave
      const int s0 = TAPS == 27 ? 0 : 4 * wv;
      // fragments of K-step s: dY (A) for every co sub-tile, U (B) for every tap
      auto load_frags = [&](int s, u32x4* a, u32x4* bfr) {
        const int y = s & 3, z = s >> 2;
#pragma unroll
        for (int m = 0; m < MC; ++m) {
          const int v0 = 16 * s + 8 * h + q, v1 = v0 + 4;
          const int qd = 4 * m + 2 * (g & 1) + (pp >> 1);
          const v4s lo = tr_read(dyl + v0 * C::DYP + dy_quad<T, MC>(qd, v0) * 16 + 8 * (pp & 1));
          const v4s hi = tr_read(dyl + v1 * C::DYP + dy_quad<T, MC>(qd, v1) * 16 + 8 * (pp & 1));
          a[m] = join(lo, hi);
        }
        const int hrow = (z * WHY + y) * WHX + 8 * h + q;
        // every wave reads NT fragments (a wave with 6 taps reads a valid
        // dummy 7th, toff = tap 0, and skips its MFMAs): no divergent phi on
        // the operand registers
#pragma unroll
        for (int k = 0; k < NT; ++k) {
          const unsigned char* bp = bimg + (hrow + toff[k]) * 32;
          bfr[k] = join(tr_read(bp), tr_read(bp + 4 * 32));
        }
      };
      // software pipeline: K-step s+1's LDS reads are in flight during K-step s's MFMAs
      u32x4 fa0[MC], fb0[NT], fa1[MC], fb1[NT];
      auto mfmas = [&](const u32x4* a, const u32x4* bfr) {
#pragma unroll
        for (int k = 0; k < NT; ++k) {
          if (k + 1 < NT || k < ntap) {
#pragma unroll
            for (int m = 0; m < MC; ++m) mfma_acc(acc[k][m], a[m], bfr[k], (T*)nullptr);
          }
        }
      };
      // the next K-step's transposed reads interleaved with this step's MFMAs
      // (2 reads per MFMA pair): at most 15 LDS reads may be tracked by
      // lgkmcnt, so a block of 18 reads ahead of the MFMAs made every step wait
      auto interleave = [&]() {
#pragma unroll
        for (int r = 0; r < (2 * MC + 2 * NT + 1) / 2; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        }
      };
      load_frags(s0, fa0, fb0);
#pragma unroll 1
      for (int i = 0; i < NS - 2; i += 2) {
        load_frags(s0 + i + 1, fa1, fb1);
        mfmas(fa0, fb0);
        interleave();
        load_frags(s0 + i + 2, fa0, fb0);
        mfmas(fa1, fb1);
        interleave();
      }
      load_frags(s0 + NS - 1, fa1, fb1);
      mfmas(fa0, fb0);
      interleave();
      mfmas(fa1, fb1);
    } else {
      const int col = lane & 31, hh = lane >> 5;
      const int s_begin = TAPS == 27 ? 0 : 32 * wv, s_end = TAPS == 27 ? 128 : 32 * wv + 32;
      const unsigned char* bimg = halo + (col >> 3) * WIMG + (col & 7) * 4;
      for (int s = s_begin; s < s_end; ++s) {
        const int v = 2 * s + hh;
        const int x = v & 15, y = (v >> 4) & 3, z = v >> 6;
        float a[MC];
#pragma unroll
        for (int m = 0; m < MC; ++m) a[m] = *reinterpret_cast<const float*>(dyl + v * C::DYP + (32 * m + col) * 4);
        const int hrow = (z * WHY + y) * WHX + x;
#pragma unroll
        for (int k = 0; k < NT; ++k) {
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

  // combine: fp32 atomics into the [tap][co][ci] scratch -- one accumulator
  // register is two 128-B row segments (ci contiguous), the full-rate atomic
  // shape; OIDHW order would scatter the 64 lanes over 64 rows (~17x slower)
  const int ci = ci0 + (lane & 31);
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    if (k < ntap) {
      const int tap = TAPS == 27 ? wv + 4 * k : 0;
#pragma unroll
      for (int m = 0; m < MC; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int co = co0 + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          if (co < p.cout && ci < p.cin)
            atomicAdd(p.dw + ((long long)tap * p.cout + co) * p.cin + ci, acc[k][m][i]);
        }
    }
  }
}

// dW[co][ci][tap] += scratch[tap][co][ci]
__global__ void __launch_bounds__(256) wgrad_finish_kernel(const float* __restrict__ scr, float* __restrict__ dw,
                                                          int cout, int cin, int taps) {
  const long long n = (long long)cout * cin * taps;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int tap = (int)(i % taps);
  const long long oc = i / taps;  // co * cin + ci
  dw[i] += scr[(long long)tap * cout * cin + oc];
}

template <typename T, int MC, int MODE, bool GN, int TAPS>
int launch_wg(const WgradParams& p, dim3 grid, hipStream_t s) {
  constexpr int smem = WgCfg<T, MC>::SMEM;
  static_assert(smem <= 160 * 1024, "wgrad LDS");
  auto k = wgrad_kernel<T, MC, MODE, GN, TAPS>;
  CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  hipLaunchKernelGGL(k, grid, dim3(256), smem, s, p);
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
  CWDM_REQUIRE(dtype_compute(d->dtype), CWDM_E_INVALID, "cwdm_conv3d_wgrad: bad dtype");
  CWDM_REQUIRE(d->ksize == 1 || d->ksize == 3, CWDM_E_UNSUPPORTED, "cwdm_conv3d_wgrad: ksize must be 1 or 3");
  CWDM_REQUIRE(d->B > 0 && d->D > 0 && d->H > 0 && d->W > 0, CWDM_E_SHAPE, "cwdm_conv3d_wgrad: empty grid");
  CWDM_REQUIRE(d->u_c1 == 0 || d->u1, CWDM_E_INVALID, "cwdm_conv3d_wgrad: second source missing");
  const int cin = d->u_c0 + d->u_c1;
  const int epq = 16 / dtype_size(d->dtype);
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
  CWDM_REQUIRE(d->workspace, CWDM_E_WORKSPACE, "cwdm_conv3d_wgrad: workspace (cwdm_conv3d_wgrad_workspace_bytes) missing");
  WgradParams p{};
  ConvParams& c = p.cp;
  c.B = (int)d->B; c.D = (int)d->D; c.H = (int)d->H; c.W = (int)d->W;
  if (d->ksize == 3) {
    c.a0 = d->u0; c.ac0 = d->u_c0; c.a1 = d->u1; c.ac1 = d->u_c1; c.amode = d->u_mode; c.agn = d->u_gn;
  } else {
    c.b0 = d->u0; c.bc0 = d->u_c0; c.b1 = d->u1; c.bc1 = d->u_c1;
  }
  p.dy = d->dy; p.dy_cs = d->dy_cs; p.cout = d->cout; p.cin = cin; p.taps = d->ksize == 3 ? 27 : 1;
  p.dw = reinterpret_cast<float*>(d->workspace);
  p.tx = (int)ceil_div(d->W, WBX); p.ty = (int)ceil_div(d->H, WBY); p.tz = (int)ceil_div(d->D, WBZ);
  p.nbricks = d->B * (long long)p.tx * p.ty * p.tz;
  const int mc = d->cout > 32 ? 2 : 1;
  p.nco = (int)ceil_div(d->cout, 32 * mc);
  const long long tiles = (long long)p.nco * (cin / 32);
  long long S = ceil_div(256, tiles);
  if (S > p.nbricks) S = p.nbricks;
  if (S < 1) S = 1;
  p.per = ceil_div(p.nbricks, S);
  S = ceil_div(p.nbricks, p.per);
  CWDM_REQUIRE(tiles < 65536, CWDM_E_SHAPE, "cwdm_conv3d_wgrad: too many channel tiles");
  dim3 grid((unsigned)S, (unsigned)tiles);
  hipStream_t s = (hipStream_t)stream;
  const bool gn = d->u_gn != nullptr;
  const long long nw = (long long)d->cout * cin * p.taps;
  CWDM_HIP(hipMemsetAsync(d->workspace, 0, nw * 4, s));
  int rc;
  rc = dispatch_dtype(d->dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    return mc == 2 ? dispatch_wg<T, 2>(p, d->u_mode, gn, grid, s) : dispatch_wg<T, 1>(p, d->u_mode, gn, grid, s);
  });
  if (rc) return rc;
  hipLaunchKernelGGL(wgrad_finish_kernel, dim3((unsigned)ceil_div(nw, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float*>(d->workspace), d->dw, d->cout, cin, p.taps);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int64_t cwdm_conv3d_wgrad_workspace_bytes(int cout, int cin, int ksize) {
  if (cout <= 0 || cin <= 0 || (ksize != 1 && ksize != 3)) return -1;
  return (int64_t)cout * cin * ksize * ksize * ksize * 4;
}
