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
//     the grid).  Every (brick range, tile) unit stores its partial tile into
//     the range's slab of the workspace; wg_reduce_kernel then adds the slabs
//     into dw in range order -- the result does not depend on which workgroup
//     finishes first (no fp32 atomics: two runs are bitwise identical).
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
  float* part;            // [S = gridDim.x][taps][cout][cin] partial slabs
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
__host__ __device__ constexpr int tap_rows(int t) {
  const int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;
  return (kz * WHY + ky) * WHX + kx;
}

// The MFMAs of one brick (16-bit types): the halo images (NCH x WIMG) and the
// brick's dY rows (256 x DYP) are in LDS; every wave accumulates its taps.
template <typename T, int MC, int TAPS>
__device__ __forceinline__ void wg_brick_mfma(const unsigned char* halo, const unsigned char* dyl,
                                              f32x16 (&acc)[TAPS == 27 ? 7 : 1][MC], const int (&toff)[TAPS == 27 ? 7 : 1],
                                              int ntap, int wv, int lane) {
  using C = WgCfg<T, MC>;
  constexpr int NT = TAPS == 27 ? 7 : 1;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = g >> 1;
  const unsigned char* bimg = halo + (g & 1) * WIMG + 8 * pp;
  constexpr int NS = TAPS == 27 ? 16 : 4;   // K-steps of this wave
  const int s0 = TAPS == 27 ? 0 : 4 * wv;
  // per-lane LDS addresses without the K-step part, which is wave-uniform (one
  // address add per fragment and K-step; the hi halves are immediate offsets).
  // dY row v = 16 s + 8 h + q (+ 4): the quad swizzle reads bit 1 of v, = bit 1 of q
  const unsigned char* abase[MC];
  const unsigned char* bbase[NT];
#pragma unroll
  for (int m = 0; m < MC; ++m) {
    const int qd = 4 * m + 2 * (g & 1) + (pp >> 1);
    abase[m] = dyl + (8 * h + q) * C::DYP + dy_quad<T, MC>(qd, q) * 16 + 8 * (pp & 1);
  }
#pragma unroll
  for (int k = 0; k < NT; ++k) bbase[k] = bimg + (8 * h + q + toff[k]) * 32;
  // fragments of K-step s: dY (A) for every co sub-tile, U (B) for every tap
  auto load_frags = [&](int s, u32x4* a, u32x4* bfr) {
    const int y = s & 3, z = s >> 2;
    const int aoff = 16 * s * C::DYP, boff = (z * WHY + y) * WHX * 32;
#pragma unroll
    for (int m = 0; m < MC; ++m) {
      const unsigned char* ap = abase[m] + aoff;
      a[m] = join(tr_read(ap), tr_read(ap + 4 * C::DYP));
    }
    // every wave reads NT fragments (a wave with 6 taps reads a valid
    // dummy 7th, toff = tap 0, and skips its MFMAs): no divergent phi on
    // the operand registers
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const unsigned char* bp = bbase[k] + boff;
      bfr[k] = join(tr_read(bp), tr_read(bp + 4 * 32));
    }
  };
  // software pipeline: K-step s+1's LDS reads are in flight during K-step s's MFMAs
  u32x4 fa0[MC], fb0[NT], fa1[MC], fb1[NT];
  // every wave runs NT taps: the wave with 6 real taps accumulates a dummy 7th
  // (tap 0 again, dropped by wg_combine) -- it would wait for the 7-tap waves at
  // the next barrier anyway, and a conditional MFMA makes the accumulators phis
  // (~190 v_accvgpr_mov per brick)
  (void)ntap;
  auto mfmas = [&](const u32x4* a, const u32x4* bfr) {
#pragma unroll
    for (int k = 0; k < NT; ++k)
#pragma unroll
      for (int m = 0; m < MC; ++m) mfma_acc(acc[k][m], a[m], bfr[k], (T*)nullptr);
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
}

// the unit's partial tile -> its slab [tap][co][ci] (plain stores: one
// accumulator register is two 128-B row segments, ci contiguous; OIDHW order
// would scatter the 64 lanes over 64 rows); wg_reduce_kernel transposes
template <int MC, int TAPS>
__device__ __forceinline__ void wg_combine(float* slab, const f32x16 (&acc)[TAPS == 27 ? 7 : 1][MC], int cout, int cin,
                                           int co0, int ci0, int ntap, int wv, int lane) {
  constexpr int NT = TAPS == 27 ? 7 : 1;
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
          if (co < cout && ci < cin) slab[((long long)tap * cout + co) * cin + ci] = acc[k][m][i];
        }
    }
  }
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
      wg_brick_mfma<T, MC, TAPS>(halo, dyl, acc, toff, ntap, wv, lane);
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

  if constexpr (TAPS == 1) {
    // 1x1: the four waves hold partial sums of the same tile (they split the
    // K-steps): waves 1-3 hand theirs over through LDS and wave 0 adds them in
    // wave order before the store
    __syncthreads();   // the last brick's operand reads are done
    float* xs = reinterpret_cast<float*>(smem);
    if (wv > 0) {
#pragma unroll
      for (int m = 0; m < MC; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) xs[(((wv - 1) * MC + m) * 16 + i) * 64 + lane] = acc[0][m][i];
    }
    __syncthreads();
    if (wv > 0) return;
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int m = 0; m < MC; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[0][m][i] += xs[((w * MC + m) * 16 + i) * 64 + lane];
  }
  wg_combine<MC, TAPS>(p.part + (long long)blockIdx.x * p.taps * p.cout * p.cin, acc, p.cout, p.cin, co0, ci0, ntap,
                       wv, lane);
}

// ---------------------------------------------------------------------------
// DMA-staged variant (16-bit types, 3x3x3): U is the forward's activated input
// kept chunk-major ([B][cin / 16][SV][16], cwdm_gn_apply's output, retained by
// the training forward), so staging is a pure copy -- every byte of the halo
// images and of the brick's dY rows reaches LDS by LDS-DMA (buffer loads with
// an LDS destination; out-of-volume voxels get an out-of-range offset and land
// as zeros), double-buffered: brick i+1's DMA flies during brick i's MFMAs, with
// no VGPRs and no VALU spent on it.  The same LDS images and MFMA loop as
// wgrad_kernel, so the products are identical.
struct WgDmaParams {
  int D, H, W;                 // conv (output) grid
  int SD, SH, SW;              // source grid of U (half of D, H, W for MODE 1)
  int tx, ty, tz;
  long long nbricks, per;
  int nco, cin, cout, dy_cs;
  int units, upx;              // (brick range, channel tile) units; units per XCD
  const unsigned char* act; long long act_bs;  // per-batch bytes of U (cin * SV * esz)
  const unsigned char* dy; long long dy_bs;    // per-batch bytes of dY (V * dy_cs * esz)
  float* part;                 // [S][cout][cin][27] partial slabs (dw's OIDHW order), one per brick range
#ifdef CWDM_WG_DIAG
  int diag;                    // timing-only decomposition (make WGDIAG=1, env CWDM_WG_DIAGMASK): 1 no MFMA loop, 2 no DMA after the first two bricks
#endif
};

// One LDS-DMA of 16 B per lane (lane l -> lds + 16 l), issued by inline asm so
// the compiler does not track it: its waitcnt pass cannot prove the transposed
// LDS reads (ds_read_b64_tr_b16) disjoint from an LDS-DMA and would drain every
// in-flight DMA (vmcnt(0)) before the first of them -- the prefetch would be
// serial.  Completion is the explicit vmcnt(0) + barrier at the next brick.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; nothing else in these kernels uses it
__device__ __forceinline__ void wg_dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff) {
  const unsigned la =
      __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(la), "v"(voff), "s"(r)
               : "memory", "m0");
}
// (the same with the LDS destination as a wave-uniform LDS byte address: no
// generic-pointer cast and null check per DMA)
__device__ __forceinline__ void wg_dma16(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff) {
  const unsigned la = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(la), "v"(voff), "s"(r)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// WS (warp-specialised, r05): 512 threads -- waves 0-3 run the MFMAs (MC = 1: their 7 taps x 32 co
// x 32 ci = 112 accumulators fit two waves per SIMD), waves 4-7 issue and wait for the LDS-DMA of
// the next brick.  Issued by the MFMA waves themselves (WS = false) the DMA cost them ~180 cycles per
// instruction at every brick start (r05 decomposition): here it runs beside the MFMAs.
template <typename T, int MC, int MODE, bool WS = false>
__global__ void __launch_bounds__(WS ? 512 : 256) wgrad_dma_kernel(WgDmaParams p) {
  using C = WgCfg<T, MC>;
  constexpr int NCH = C::NCH, EPQ = 16 / (int)sizeof(T), QPV = C::DYP / 16;
  constexpr int BUF = C::SMEM;           // one stage: the halo images + the dY rows
  constexpr int HP = WHV * 2;            // halo pieces (16 B) per chunk image
  constexpr int HI = (HP + 63) / 64;     // ... = wave instructions per chunk (21)
  constexpr int DI = 256 * QPV / 64;     // dY wave instructions per brick
  constexpr int ESZ = (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // (wv wave-uniform in an SGPR: the DMAs' LDS destinations are scalar adds)
  const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const bool mw = !WS || wv < 4;     // this wave runs MFMAs
  const bool dw = !WS || wv >= 4;    // this wave issues the DMA
  const int iw = WS ? (wv & 3) : wv;  // its index among the issuing waves
  constexpr int NT = WS ? 512 : 256;
  // XCD-aware map of the 1-D grid: workgroups are dealt to the 8 XCDs round
  // robin, so the k-th workgroup of XCD j takes unit j * upx + k of the
  // range-major (brick range, channel tile) list -- the channel tiles of a
  // brick range run on one XCD (two at a seam) and the range's dY rows (and
  // halo) are fetched into one L2, not into up to 8 (cin 192: 1.7x the time
  // per flop with the plain 2-D grid); upx <= 32 keeps every XCD to one round
  // of its 32 CUs (ranges dealt j + 8 k put 36 on XCD 0 at cin 192: 2.5x)
  const int ntiles = p.nco * (p.cin / 32);
  const int xj = (int)(blockIdx.x & 7), xk = (int)(blockIdx.x >> 3);
  const int u = xj * p.upx + xk;
  if (xk >= p.upx || u >= p.units) return;
  const long long sx = u / ntiles;
  const int tile = u % ntiles;
  if (sx * p.per >= p.nbricks) return;
  const int ct = tile % p.nco, it = tile / p.nco;
  const int co0 = ct * C::CO, ci0 = it * 32;
  const long long bb = sx * p.per;
  const long long be = bb + p.per < p.nbricks ? bb + p.per : p.nbricks;
  const int ntap = wv < 3 ? 7 : 6;
  int toff[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) toff[k] = tap_rows(wv + 4 * k < 27 ? wv + 4 * k : 0);
  f32x16 acc[7][MC];
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int m = 0; m < MC; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[k][m][i] = 0.f;
  const int nb_vol = p.tx * p.ty * p.tz;
  const long long sv_n = (long long)p.SD * p.SH * p.SW;
  // per-lane DMA offsets relative to the brick origin, for the bricks whose
  // halo lies inside the volume and whose dY rows are all in range (interior
  // bricks: two thirds at 128^3): their issue is one add per DMA instead of the
  // coordinate arithmetic below, which the MFMA waves ran serially before every
  // brick (~280 VALU + ~390 SALU ahead of the first MFMA).  MODE 1: x0, y0, z0
  // are even, so (x0 + d) >> 1 = x0 / 2 + (d >> 1) (arithmetic shift: -1 -> -1).
  constexpr int HJ = (HI + 3) / 4, DJ = DI / 4;
  int hrel[HJ], drel[DJ];
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int pc = (iw + 4 * j) * 64 + lane, hv = pc >> 1, q = pc & 1;
    int hx = hv % WHX - 1, hy = (hv / WHX) % WHY - 1, hz = hv / (WHX * WHY) - 1;
    if (MODE == 1) { hx >>= 1; hy >>= 1; hz >>= 1; }
    hrel[j] = ((hz * p.SH + hy) * p.SW + hx) * 32 + q * 16;
  }
#pragma unroll
  for (int j = 0; j < DJ; ++j) {
    const int pc = (iw + 4 * j) * 64 + lane, v = pc / QPV, pos = pc % QPV;
    const int qd = dy_quad<T, MC>(pos, v);
    drel[j] = ((((v >> 6) * p.H + ((v >> 4) & 3)) * p.W + (v & 15)) * p.dy_cs + qd * EPQ) * ESZ;
  }

  // brick coordinates of the next brick to issue, advanced in brick order (a
  // 64-bit division per brick was ~130 SALU ahead of the MFMAs)
  int nb_b = (int)(bb / nb_vol), nb_x, nb_y, nb_z;
  {
    const int r0 = (int)(bb % nb_vol);
    nb_x = r0 % p.tx; nb_y = (r0 / p.tx) % p.ty; nb_z = r0 / (p.tx * p.ty);
  }
  auto issue = [&](unsigned lb) {
    const int b = nb_b, x0 = nb_x * WBX, y0 = nb_y * WBY, z0 = nb_z * WBZ;
    if (++nb_x == p.tx) {
      nb_x = 0;
      if (++nb_y == p.ty) {
        nb_y = 0;
        if (++nb_z == p.tz) { nb_z = 0; ++nb_b; }
      }
    }
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.act + (long long)b * p.act_bs), (short)0, (int)p.act_bs, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.dy + (long long)b * p.dy_bs), (short)0, (int)p.dy_bs, 0x00020000);
    if (x0 >= 1 && y0 >= 1 && z0 >= 1 && x0 + WBX < p.W && y0 + WBY < p.H && z0 + WBZ < p.D &&
        co0 + C::CO <= p.dy_cs) {
      const int hbase = MODE == 1 ? (((z0 >> 1) * p.SH + (y0 >> 1)) * p.SW + (x0 >> 1)) * 32
                                  : ((z0 * p.SH + y0) * p.SW + x0) * 32;
      const int dbase = (((z0 * p.H + y0) * p.W + x0) * p.dy_cs + co0) * ESZ;
#pragma unroll
      for (int j = 0; j < HJ; ++j) {
        const int k = iw + 4 * j;
        if (k < HI && (k * 64 + lane) / 2 < WHV) {
#pragma unroll
          for (int c = 0; c < NCH; ++c)
            wg_dma16(ra, lb + c * WIMG + k * 1024,
                     (unsigned)(hbase + hrel[j]) + (unsigned)((long long)(ci0 / 16 + c) * sv_n * 32));
        }
      }
#pragma unroll
      for (int j = 0; j < DJ; ++j) wg_dma16(rd, lb + C::DY_OFF + (iw + 4 * j) * 1024, (unsigned)(dbase + drel[j]));
      return;
    }
    // halo: instruction k of a chunk image covers pieces 64 k .. +63 = voxel slots 32 k .. +31, both quads
#pragma unroll
    for (int j = 0; j < (HI + 3) / 4; ++j) {
      const int k = iw + 4 * j;
      if (k < HI) {
        const int pc = k * 64 + lane, hv = pc >> 1, q = pc & 1;
        unsigned vb = 0xFFFFFFF0u;
        const int hx = hv % WHX, hy = (hv / WHX) % WHY, hz = hv / (WHX * WHY);
        int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
        if (ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) {
          if (MODE == 1) { ox >>= 1; oy >>= 1; oz >>= 1; }
          vb = (unsigned)(((oz * p.SH + oy) * p.SW + ox) * 32 + q * 16);
        }
        if (hv < WHV) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            const unsigned cofs = (unsigned)((long long)(ci0 / 16 + c) * sv_n * 32);  // chunk ci0 / 16 + c
            const unsigned voff = vb == 0xFFFFFFF0u ? vb : vb + cofs;
            wg_dma16(ra, lb + c * WIMG + k * 1024, voff);
          }
        }
      }
    }
    // dY rows: instruction k covers pieces 64 k .. +63 = (voxel v, LDS quad position pos)
#pragma unroll
    for (int j = 0; j < DI / 4; ++j) {
      const int k = iw + 4 * j;
      const int pc = k * 64 + lane, v = pc / QPV, pos = pc % QPV;
      const int qd = dy_quad<T, MC>(pos, v);  // the swizzle is an involution
      const int x = x0 + (v & 15), y = y0 + ((v >> 4) & 3), z = z0 + (v >> 6);
      const int cc = co0 + qd * EPQ;
      const bool in = x < p.W && y < p.H && z < p.D && cc < p.dy_cs;
      const unsigned voff =
          in ? ((unsigned)((z * p.H + y) * p.W + x) * (unsigned)p.dy_cs + (unsigned)cc) * (unsigned)ESZ : 0xFFFFFFF0u;
      wg_dma16(rd, lb + C::DY_OFF + k * 1024, voff);
    }
  };

  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)smem;
#ifdef CWDM_WG_DIAG
  const bool no_mfma = p.diag & 1, no_dma = p.diag & 2;
#else
  constexpr bool no_mfma = false, no_dma = false;
#endif
  // (no_dma: both stages are filled once, so the MFMAs run on real data -- their clock depends on it)
  if (bb < be && dw) issue(lds0);
  for (long long bi = bb; bi < be; ++bi) {
    unsigned char* cur = smem + ((bi - bb) & 1) * BUF;
    if (dw) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this brick's DMA (issued one brick ago) landed
    __syncthreads();                                  // ... for every wave; the other stage is free
    if (dw && bi + 1 < be && (!no_dma || bi == bb)) issue(lds0 + (unsigned)(((bi - bb + 1) & 1) * BUF));   // brick bi + 1
    if (mw && !no_mfma) wg_brick_mfma<T, MC, 27>(cur, cur + C::DY_OFF, acc, toff, ntap, wv, lane);
  }
  // the partial tile -> the brick range's slab in dw's OIDHW order: per 32-channel
  // half m of the tile the four waves' taps meet in LDS as [co 32][ci 32][tap 27]
  // (the stages are free now), then every row co -- 32 ci x 27 taps = 864
  // contiguous floats -- goes out as coalesced stores (wg_reduce_kernel adds the
  // slabs in range order: deterministic)
  float* T3 = reinterpret_cast<float*>(smem);
  const int cil = lane & 31;
#pragma unroll
  for (int m = 0; m < MC; ++m) {
    __syncthreads();  // the previous half's rows are out (m = 0: the last brick's reads are done)
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (mw && k < ntap) {
        const int tap = wv + 4 * k;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int col = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          T3[(col * 32 + cil) * 27 + tap] = acc[k][m][i];
        }
      }
    }
    __syncthreads();
    const int ncol = min(32, p.cout - co0 - 32 * m), nci = min(32, p.cin - ci0);
    float* slab = p.part + sx * ((long long)p.cout * p.cin * 27);
    for (int r = 0; r < ncol; ++r) {
      float* row = slab + ((long long)(co0 + 32 * m + r) * p.cin + ci0) * 27;
      for (int e = tid; e < nci * 27; e += NT) row[e] = T3[r * 864 + e];
    }
  }
}

// ---------------------------------------------------------------------------
// 1x1 weight gradient (the ResBlock skip_connection conv, unet.py:264-271;
// 16-bit types): dW[co][ci] = sum_v dY[v][co] U[v][ci] with U the raw
// concat(u0, u1).  A GEMM with K = B * V voxels and a 64 x 128 output tile, so
// HBM-bound (R0 of the run.sh U-Net: 192 -> 64 channels over 2 M voxels reads
// 1.07 GB for 0.05 TFLOP).  The brick kernel staged a 3^3 halo per 16x4x4
// brick (2.5x the voxels) and re-read dY once per 32-channel input tile
// (386-607 us per R0 call, ~2.2 ms per training step); here a unit = a range of
// 64-voxel stages x one (64 co, 128 ci) tile, every stage -- 8 chunk images of
// U (16 channels, 32-B rows) + the 64 dY rows -- lands in LDS by LDS-DMA,
// double-buffered, and feeds the transposed-read MFMA operands of the 3x3x3
// kernels (tap offset 0).  Wave w owns input channels [32 w, +32) of the tile.
// Partial tiles go to the stage range's slab; wg_reduce_kernel adds the slabs.
struct Wg1Params {
  const unsigned char* u0; const unsigned char* u1;
  int c0, c1, cin;
  const unsigned char* dy; int dy_cs, cout;
  long long rows;   // B * V voxel rows (u0 / u1 / dy are row-contiguous over the batch)
  long long nst;    // 64-row stages = ceil(rows / 64)
  long long per;    // stages per unit
  int nco, nci;     // 64-channel co tiles x 128-channel ci tiles
  int units, upx;   // (stage range, tile) units; units per XCD
  float* part;      // [S][cout][cin] partial slabs, one per stage range
};
constexpr int W1_NV = 64;
constexpr int W1_IMG = W1_NV * 32 + 128;         // one 16-channel chunk image (+128 B: complementary banks)
constexpr int W1_DY = 8 * W1_IMG;                // the 64 dY rows (128 B, quad-swizzled) after the 8 images
constexpr int W1_BUF = W1_DY + W1_NV * 128;      // one stage: 25.6 KB (three workgroups per CU double-buffered)

template <typename T>
__global__ void __launch_bounds__(256) wgrad1_kernel(Wg1Params p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the DMA descriptors are SGPRs
  const int ntiles = p.nco * p.nci;
  // XCD-aware: the k-th workgroup of XCD j takes unit j * upx + k of the
  // range-major list, so the tiles of one stage range share an L2
  const int xj = (int)(blockIdx.x & 7), xk = (int)(blockIdx.x >> 3);
  const int u = xj * p.upx + xk;
  if (xk >= p.upx || u >= p.units) return;
  const long long sr = u / ntiles;
  const int tile = u % ntiles;
  const long long sb = sr * p.per, se = min(sb + p.per, p.nst);
  if (sb >= se) return;
  const int co0 = (tile % p.nco) * 64, ci0 = (tile / p.nco) * 128;
  const bool wact = ci0 + 32 * wv < p.cin;   // this wave's 32 input channels exist
  f32x16 acc[2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[m][i] = 0.f;

  // DMA of stage st into buf: 16 image instructions (chunk c, half k) + 8 dY
  // instructions, 6 per wave; rows past the end read zeros (buffer range check)
  auto issue = [&](long long st, unsigned char* buf) {
    const long long r0 = st * W1_NV;
    const int nr = (int)min((long long)W1_NV, p.rows - r0);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int k = wv + 4 * j;   // instruction 0..23
      if (k < 16) {
        const int c = k >> 1, half = k & 1;
        const int gc = ci0 + 16 * c;
        if (gc < p.cin) {
          const bool s0 = gc < p.c0;
          const int cs = s0 ? p.c0 : p.c1;
          const unsigned char* base = (s0 ? p.u0 : p.u1) + r0 * cs * 2;
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nr * cs * 2, 0x00020000);
          const int row = 32 * half + (lane >> 1);
          const unsigned voff = (unsigned)(row * cs + (s0 ? gc : gc - p.c0)) * 2u + (unsigned)(lane & 1) * 16u;
          wg_dma16(rs, buf + c * W1_IMG + half * 1024, voff);
        }
      } else {
        const int kk = k - 16;
        const int pc = kk * 64 + lane, v = pc >> 3, pos = pc & 7;
        const int qd = dy_quad<T, 2>(pos, v);   // the swizzle is an involution
        const int cc = co0 + qd * 8;
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.dy + r0 * p.dy_cs * 2), (short)0, nr * p.dy_cs * 2, 0x00020000);
        const unsigned voff = cc < p.dy_cs ? (unsigned)(v * p.dy_cs + cc) * 2u : 0xFFFFFFF0u;
        wg_dma16(rd, buf + W1_DY + kk * 1024, voff);
      }
    }
  };

  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = g >> 1;
  issue(sb, smem);
  for (long long st = sb; st < se; ++st) {
    unsigned char* cur = smem + ((st - sb) & 1) * W1_BUF;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this stage's DMA (issued one stage ago) landed
    __syncthreads();                                  // ... for every wave; the other buffer is free
    if (st + 1 < se) issue(st + 1, smem + ((st - sb + 1) & 1) * W1_BUF);
    if (wact) {
      const unsigned char* dyl = cur + W1_DY;
      const unsigned char* bimg = cur + (2 * wv + (g & 1)) * W1_IMG + 8 * pp;
#pragma unroll
      for (int s = 0; s < W1_NV / 16; ++s) {
        const int v0 = 16 * s + 8 * h + q, v1 = v0 + 4;
        u32x4 a[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int qd = 4 * m + 2 * (g & 1) + (pp >> 1);
          a[m] = join(tr_read(dyl + v0 * 128 + dy_quad<T, 2>(qd, v0) * 16 + 8 * (pp & 1)),
                      tr_read(dyl + v1 * 128 + dy_quad<T, 2>(qd, v1) * 16 + 8 * (pp & 1)));
        }
        const u32x4 b = join(tr_read(bimg + v0 * 32), tr_read(bimg + v1 * 32));
#pragma unroll
        for (int m = 0; m < 2; ++m) mfma_acc(acc[m], a[m], b, (T*)nullptr);
      }
    }
  }
  if (!wact) return;
  const int ci = ci0 + 32 * wv + (lane & 31);
  if (ci >= p.cin) return;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = co0 + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      if (co < p.cout) p.part[(sr * p.cout + co) * p.cin + ci] = acc[m][i];
    }
}

// dw += sum over the S partial slabs, in slab order.  A 256-thread block is
// (256 / R) columns x R row groups; column c owns 4 consecutive slab elements
// (16-byte loads), row group r sums slabs r, r + R, ... in increasing order (8
// loads in flight), and the R group sums are added in group order -- the same
// sum on every run for a given S.  R = min(16, ceil(S / 8)) (host): few slabs
// (the small levels) -> one row group and 1024 elements per block; many (the
// 128^3 level's 128) -> 16 groups of 8 slabs.  perm: the slabs are
// [taps][cout][cin] (wgrad_kernel) and dw is OIDHW.
template <int R>
__global__ void __launch_bounds__(256) wg_reduce_kernel(const float* __restrict__ part, int S, long long n,
                                                       float* __restrict__ dw, int cout, int cin, int taps, int perm) {
  constexpr int NC = 256 / R;
  const int c = threadIdx.x % NC, r = threadIdx.x / NC;
  const long long j = ((long long)blockIdx.x * NC + c) * 4;   // n % 4 == 0 (cin % 32 == 0)
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < n) {
    const float* p = part + j;
    int k = r;
    for (; k + 7 * R < S; k += 8 * R) {
      float4 u[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = *reinterpret_cast<const float4*>(p + (long long)(k + e * R) * n);
#pragma unroll
      for (int e = 0; e < 8; ++e) { a.x += u[e].x; a.y += u[e].y; a.z += u[e].z; a.w += u[e].w; }
    }
    for (; k < S; k += R) {
      const float4 u = *reinterpret_cast<const float4*>(p + (long long)k * n);
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
  }
  if constexpr (R > 1) {
    __shared__ float4 red[256];
    red[threadIdx.x] = a;
    __syncthreads();
    if (r) return;
#pragma unroll
    for (int q = 1; q < R; ++q) {
      const float4 u = red[q * NC + c];
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
  }
  if (j >= n) return;
  const float t[4] = {a.x, a.y, a.z, a.w};
  const long long cc = (long long)cout * cin;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long jj = j + e;
    const long long o = perm ? (jj % cc) * taps + jj / cc : jj;   // [tap][co][ci] -> [co][ci][tap]
    dw[o] += t[e];
  }
}

int launch_wg_reduce(const float* part, long long S, long long n, float* dw, int cout, int cin, int taps, bool perm,
                     hipStream_t s) {
  CWDM_REQUIRE(S > 0 && S < (1LL << 31) && n % 4 == 0, CWDM_E_SHAPE, "cwdm_conv3d_wgrad: bad partial slab count");
  const int R = S >= 128 ? 16 : S >= 64 ? 8 : S >= 32 ? 4 : S >= 16 ? 2 : 1;
  const long long nb = ceil_div(n / 4, (long long)(256 / R));
  CWDM_REQUIRE(nb < (1LL << 31), CWDM_E_SHAPE, "cwdm_conv3d_wgrad: weight gradient too large");
  const int pm = perm ? 1 : 0;
  const dim3 g((unsigned)nb), b(256);
  switch (R) {
    case 16: hipLaunchKernelGGL(wg_reduce_kernel<16>, g, b, 0, s, part, (int)S, n, dw, cout, cin, taps, pm); break;
    case 8: hipLaunchKernelGGL(wg_reduce_kernel<8>, g, b, 0, s, part, (int)S, n, dw, cout, cin, taps, pm); break;
    case 4: hipLaunchKernelGGL(wg_reduce_kernel<4>, g, b, 0, s, part, (int)S, n, dw, cout, cin, taps, pm); break;
    case 2: hipLaunchKernelGGL(wg_reduce_kernel<2>, g, b, 0, s, part, (int)S, n, dw, cout, cin, taps, pm); break;
    default: hipLaunchKernelGGL(wg_reduce_kernel<1>, g, b, 0, s, part, (int)S, n, dw, cout, cin, taps, pm); break;
  }
  CWDM_LAUNCHED();
  return CWDM_OK;
}

template <typename T>
int launch_wg1(const cwdm_wgrad_desc* d, hipStream_t s) {
  Wg1Params q{};
  q.u0 = reinterpret_cast<const unsigned char*>(d->u0);
  q.u1 = reinterpret_cast<const unsigned char*>(d->u1);
  q.c0 = d->u_c0; q.c1 = d->u_c1; q.cin = d->u_c0 + d->u_c1;
  q.dy = reinterpret_cast<const unsigned char*>(d->dy); q.dy_cs = d->dy_cs; q.cout = d->cout;
  q.rows = d->B * d->D * d->H * d->W;
  q.nst = ceil_div(q.rows, (int64_t)W1_NV);
  q.nco = (int)ceil_div(d->cout, 64);
  q.nci = (int)ceil_div(q.cin, 128);
  const long long ntiles = (long long)q.nco * q.nci;
  // ~3 workgroups per CU slot (51 KB of LDS each): stage ranges x tiles ~ 768
  long long S = std::max<long long>(1, 768 / ntiles);
  if (S > q.nst) S = q.nst;
  q.per = ceil_div(q.nst, S);
  S = ceil_div(q.nst, q.per);
  q.units = (int)(S * ntiles);
  q.upx = (q.units + 7) / 8;
  q.part = reinterpret_cast<float*>(d->workspace);
  constexpr int smem = 2 * W1_BUF;
  auto k = wgrad1_kernel<T>;
  CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  hipLaunchKernelGGL(k, dim3((unsigned)(8LL * q.upx)), dim3(256), smem, s, q);
  CWDM_LAUNCHED();
  return launch_wg_reduce(q.part, S, (long long)q.cout * q.cin, d->dw, q.cout, q.cin, 1, false, s);
}

// the 1x1 kernel's shapes: 16-bit, source boundary on a 16-channel chunk, < 2 GB per stage row block
bool wg1_eligible(const cwdm_wgrad_desc* d) {
  if (d->ksize != 1 || !dtype_half(d->dtype) || d->u_gn || d->u_mode != 0 || d->u_cm) return false;
  if (d->u_c0 % 16 || (d->u_c0 + d->u_c1) % 32 || d->dy_cs % 8) return false;
  return d->B * d->D * d->H * d->W * (int64_t)(d->u_c0 + d->u_c1) * 2 < (1LL << 40);
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

template <typename T, int MC, int MODE, bool WS = false>
int launch_wg_dma(const WgDmaParams& p, dim3, hipStream_t s) {
  constexpr int smem = 2 * WgCfg<T, MC>::SMEM;
  static_assert(smem <= 160 * 1024, "wgrad DMA LDS");
  auto k = wgrad_dma_kernel<T, MC, MODE, WS>;
  CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  // 1-D: 8 XCDs x upx units of (brick range grid.x, channel tile grid.y)
  const long long n = 8LL * p.upx;
  CWDM_REQUIRE(n < (1LL << 31), CWDM_E_UNSUPPORTED, "cwdm_conv3d_wgrad: grid too large");
  hipLaunchKernelGGL(k, dim3((unsigned)n), dim3(WS ? 512 : 256), smem, s, p);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

// ---------------------------------------------------------------------------
// Output-head weight gradient (the 64 -> out_channels conv of out[2], unet.py:
// 793-797, with its GroupNorm+SiLU; 16-bit, 3x3x3, cout <= 8, cin 64):
//
//   dW[co][ci][t] = sum_u dY[u - (t - 1)][co] U[u][ci],   U = SiLU(GN(x))
//
// The brick kernel put cout on the MFMA's M side (a 32-row tile, 8 used) and
// staged U's 3^3 halo for every 32-channel tile (the transform on 2.5x the
// voxels, twice): 486 us at 128^3.  Here M = (tap, co) = 216 rows (7 tiles of 4
// taps x 8 channels), N = ci (2 tiles), K = voxels: the SHIFT moves to dY (8
// channels, its halo is small) and U is staged once per brick, without halo.
// Both operands need 8 consecutive voxels per lane, so both LDS images are
// channel-major: U [ci][z][y][16 x] (ci pitch 528 B: 16-lane groups of the B
// reads hit distinct bank quads) and dY [x shift][co][6 z][6 y][16 x] (three
// x-shifted copies keep every A read 16-byte aligned; co pitch 1168 B).  Wave w:
// N tile w & 1, M tiles 0-3 (w < 2) or 4-6; per 16-voxel K step one B read and
// 4 A reads feed 4 v_mfma_f32_32x32x16, software-pipelined one step ahead.  Two workgroups per CU (61.8 KB of
// LDS each) overlap one's staging with the other's MFMAs, and a brick's global loads are
// issued before the previous brick's MFMAs (register prefetch).  Partial tiles go to
// the workgroup's slab [27][cout][64]; wg_reduce_kernel adds the slabs in order.
struct HwParams {
  const void* x; const float* gn; const void* dy;
  int dy_cs, cout;
  int D, H, W, tx, ty, tz;
  long long nbricks, per;
  float* part;
};
constexpr int HW_CS = 16 * 32 + 16;          // U image: bytes per input channel
constexpr int HW_UIMG = 64 * HW_CS;
constexpr int HW_COS = 36 * 32 + 16;         // dY image: bytes per output channel (6 x 6 rows)
constexpr int HW_KXS = 8 * HW_COS;           // one x-shifted copy
constexpr int HW_ZOFF = HW_UIMG + 3 * HW_KXS;  // zeros: the A rows of taps >= 27 read them (branch-free K loop)
constexpr int HW_SMEM = HW_ZOFF + 704;
constexpr long long HW_SMAX = 512;           // brick ranges (workgroups)

template <typename T, bool GN>
__global__ void __launch_bounds__(256, 2) head_wgrad_kernel(HwParams p) {
  constexpr int EPQ = 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* uimg = smem;
  unsigned char* dimg = smem + HW_UIMG;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, col = lane & 31, kh = lane >> 5;
  const long long bb = (long long)blockIdx.x * p.per;
  const long long be = bb + p.per < p.nbricks ? bb + p.per : p.nbricks;
  const int nt = wv & 1, mt0 = (wv >> 1) * 4, nmt = (wv >> 1) ? 3 : 4;   // M tiles 0-3 / 4-6
  // A rows: lane row m = col -> tap 4 mt + col / 8, co = col % 8; its dY row for K step
  // (zz, yy) is (hz, hy) = (zz + 2 - kz, yy + 2 - ky) of copy kx
  // (every wave runs 4 M tiles: waves 2-3's fourth is taps 28-31, all zero rows -- the same MFMA
  // count as waves 0-1 and no branch in the K loop)
  int aoff[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int tap = 4 * (mt0 + k) + (col >> 3);
    const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
    aoff[k] = tap < 27 ? kx * HW_KXS + (col & 7) * HW_COS + ((2 - kz) * 6 + (2 - ky)) * 32 + kh * 16
                       : HW_ZOFF - HW_UIMG + kh * 16;
  }
  for (int i = tid; i < 704 / 16; i += 256) *reinterpret_cast<u32x4*>(smem + HW_ZOFF + 16 * i) = u32x4{0u, 0u, 0u, 0u};
  const int boff = (32 * nt + col) * HW_CS + kh * 16;
  f32x16 acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[k][i] = 0.f;
  const int nb_vol = p.tx * p.ty * p.tz;
  const int g = tid & 7, pr = tid >> 3;   // U staging: channels 8 g .. + 8 of voxel pairs pr + 32 j
  const T* xs = reinterpret_cast<const T*>(p.x);
  const T* ds = reinterpret_cast<const T*>(p.dy);

  // global -> registers for brick bi (U's 8 16-byte pieces, dY's up to 3 halo voxels): issued
  // before the previous brick's MFMAs, so a brick's loads fly under them
  u32x4 ur[4][2], dr[3];
  int fb = 0;
  auto fetch = [&](long long bi) {
    const int b = (int)(bi / nb_vol);
    int r = (int)(bi % nb_vol);
    const int x0 = (r % p.tx) * 16;
    r /= p.tx;
    const int y0 = (r % p.ty) * 4, z0 = (r / p.ty) * 4;
    fb = b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = pr + 32 * j, x = 2 * (q & 7), yy = (q >> 3) & 3, zz = q >> 5;
      const long long vox = (((long long)b * p.D + z0 + zz) * p.H + y0 + yy) * p.W + x0 + x;
      ur[j][0] = ldg16(xs + vox * 64 + 8 * g);
      ur[j][1] = ldg16(xs + (vox + 1) * 64 + 8 * g);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int hv = tid + 256 * j;
      const int hx = hv % 18, hy = (hv / 18) % 6, hz = hv / 108;
      const int vx = x0 + hx - 1, vy = y0 + hy - 1, vz = z0 + hz - 1;
      const bool in = hv < 648 && vx >= 0 && vy >= 0 && vz >= 0 && vx < p.W && vy < p.H && vz < p.D;
      dr[j] = u32x4{0u, 0u, 0u, 0u};
      if (in) dr[j] = ldg16(ds + ((((long long)b * p.D + vz) * p.H + vy) * p.W + vx) * p.dy_cs);
    }
  };
  if (bb < be) fetch(bb);
  int sb = -1;
  float sc[EPQ], sh[EPQ];
  for (long long bi = bb; bi < be; ++bi) {
    const int b = fb;
    if (b != sb) {
#pragma unroll
      for (int e = 0; e < EPQ; ++e) {
        // (the head's forward transform, silu_aff: U bit-identical to what the conv saw)
        if (GN) silu_aff_coef(p.gn[((long long)b * 64 + 8 * g + e) * 2], p.gn[((long long)b * 64 + 8 * g + e) * 2 + 1],
                              sc[e], sh[e]);
      }
      sb = b;
    }
    __syncthreads();   // the previous brick's operand reads are done
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = pr + 32 * j, x = 2 * (q & 7), yy = (q >> 3) & 3, zz = q >> 5;
      u32x4 t2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (GN) {
          float f[EPQ];
          unpack<T>(ur[j][h], f);
#pragma unroll
          for (int e = 0; e < EPQ; ++e) f[e] = silu_aff(f[e], sc[e], sh[e]);
          t2[h] = pack<T>(f);
        } else {
          t2[h] = ur[j][h];
        }
      }
      // channel 8 g + e of voxels x, x + 1 -> one 32-bit word of row (ci, zz, yy)
      unsigned char* dst = uimg + (8 * g) * HW_CS + ((zz * 4 + yy) * 16 + x) * 2;
#pragma unroll
      for (int e = 0; e < EPQ; ++e)
        *reinterpret_cast<unsigned*>(dst + e * HW_CS) =
            __builtin_amdgcn_perm(t2[1][e >> 1], t2[0][e >> 1], (e & 1) ? 0x07060302u : 0x05040100u);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int hv = tid + 256 * j;
      if (hv < 648) {
        const int hx = hv % 18, hy = (hv / 18) % 6, hz = hv / 108;
        unsigned char* row = dimg + (hz * 6 + hy) * 32;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int jj = hx + kx - 2;   // element jj of copy kx is dY at halo x jj - kx + 2
          if (jj >= 0 && jj < 16) {
#pragma unroll
            for (int co = 0; co < 8; ++co)
              *reinterpret_cast<unsigned short*>(row + kx * HW_KXS + co * HW_COS + jj * 2) =
                  (unsigned short)((dr[j][co >> 1] >> (16 * (co & 1))) & 0xffffu);
          }
        }
      }
    }
    __syncthreads();
    if (bi + 1 < be) fetch(bi + 1);
    // K step st = (zz, yy): its 5 operand reads are issued before step st - 1's MFMAs
    u32x4 bv[2], av[2][4];
    auto rd = [&](int st, int q) {
      const int zz = st >> 2, yy = st & 3;
      bv[q] = *reinterpret_cast<const u32x4*>(uimg + boff + (zz * 4 + yy) * 32);
#pragma unroll
      for (int k = 0; k < 4; ++k) av[q][k] = *reinterpret_cast<const u32x4*>(dimg + aoff[k] + (zz * 6 + yy) * 32);
    };
    rd(0, 0);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      if (st + 1 < 16) rd(st + 1, (st + 1) & 1);
#pragma unroll
      for (int k = 0; k < 4; ++k) mfma_acc(acc[k], av[st & 1][k], bv[st & 1], (T*)nullptr);
    }
  }
  // acc[k][i] = dW row m = 8 (i / 4) + 4 kh + i % 4 -> (tap 4 (mt0 + k) + i / 4, co 4 kh + i % 4), ci 32 nt + col
  float* slab = p.part + (long long)blockIdx.x * 27 * p.cout * 64;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < nmt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int tap = 4 * (mt0 + k) + (i >> 2), co = 4 * kh + (i & 3);
        if (tap < 27 && co < p.cout) slab[((long long)tap * p.cout + co) * 64 + 32 * nt + col] = acc[k][i];
      }
    }
  }
}

bool hw_shape_ok(int cout, int cin, int ksize) { return ksize == 3 && cout >= 1 && cout <= 8 && cin == 64; }

// the output head's weight gradient kernel where it applies (env CWDM_HEAD_WG=0: the brick kernel, A/B)
bool hw_eligible(const cwdm_wgrad_desc* d) {
  static const bool on = [] { const char* e = std::getenv("CWDM_HEAD_WG"); return !(e && e[0] == '0'); }();
  if (!on || !hw_shape_ok(d->cout, d->u_c0 + d->u_c1, d->ksize) || !dtype_half(d->dtype)) return false;
  if (d->u_mode != 0 || d->u_cm || d->u1 || d->u_c1 != 0 || d->dy_cs < 8 || d->dy_cs % 8) return false;
  if (d->W % 16 || d->H % 4 || d->D % 4) return false;
  return d->B * d->D * d->H * d->W * 64 < (1LL << 40);
}

template <typename T>
int launch_hw(const cwdm_wgrad_desc* d, hipStream_t s) {
  HwParams q{};
  q.x = d->u0; q.gn = d->u_gn; q.dy = d->dy; q.dy_cs = d->dy_cs; q.cout = d->cout;
  q.D = (int)d->D; q.H = (int)d->H; q.W = (int)d->W;
  q.tx = q.W / 16; q.ty = q.H / 4; q.tz = q.D / 4;
  q.nbricks = d->B * (long long)q.tx * q.ty * q.tz;
  long long S = std::min(HW_SMAX, q.nbricks);
  q.per = ceil_div(q.nbricks, S);
  S = ceil_div(q.nbricks, q.per);
  q.part = reinterpret_cast<float*>(d->workspace);
  auto k = d->u_gn ? head_wgrad_kernel<T, true> : head_wgrad_kernel<T, false>;
  CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, HW_SMEM));
  hipLaunchKernelGGL(k, dim3((unsigned)S), dim3(256), HW_SMEM, s, q);
  CWDM_LAUNCHED();
  return launch_wg_reduce(q.part, S, 27LL * d->cout * 64, d->dw, d->cout, 64, 27, true, s);
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
  CWDM_REQUIRE(d->ws_bytes >= cwdm_conv3d_wgrad_workspace_bytes(d->cout, cin, d->ksize), CWDM_E_WORKSPACE,
               "cwdm_conv3d_wgrad: ws_bytes below cwdm_conv3d_wgrad_workspace_bytes(cout, cin, ksize)");
  WgradParams p{};
  ConvParams& c = p.cp;
  c.B = (int)d->B; c.D = (int)d->D; c.H = (int)d->H; c.W = (int)d->W;
  if (d->ksize == 3) {
    c.a0 = d->u0; c.ac0 = d->u_c0; c.a1 = d->u1; c.ac1 = d->u_c1; c.amode = d->u_mode; c.agn = d->u_gn;
  } else {
    c.b0 = d->u0; c.bc0 = d->u_c0; c.b1 = d->u1; c.bc1 = d->u_c1;
  }
  p.dy = d->dy; p.dy_cs = d->dy_cs; p.cout = d->cout; p.cin = cin; p.taps = d->ksize == 3 ? 27 : 1;
  p.part = reinterpret_cast<float*>(d->workspace);
  p.tx = (int)ceil_div(d->W, WBX); p.ty = (int)ceil_div(d->H, WBY); p.tz = (int)ceil_div(d->D, WBZ);
  p.nbricks = d->B * (long long)p.tx * p.ty * p.tz;
  // the DMA-staged kernel's warp-specialised form takes 32-output tiles, where it measured faster:
  // cin <= cout (r05 A/B, profiles/r05/k_wgrad_ws_ab.txt: 64->64 477 -> 440 us, 64^3 128->128 219 ->
  // 205, the upsampling 128->128 1519 -> 1489; 192->64 / 128->64 / 384->128 1-4 % slower).  Env
  // CWDM_WG_WS=0: never, 2: every kept-activation call (A/B)
  static const int ws_mode = [] { const char* e = std::getenv("CWDM_WG_WS"); return e ? std::atoi(e) : 1; }();
  const bool ws = d->u_cm && (ws_mode == 2 || (ws_mode == 1 && cin <= d->cout));
#ifdef CWDM_WG_DIAG
  static const bool force_mc1 = [] { const char* e = std::getenv("CWDM_WG_MC1"); return e && e[0] == '1'; }();
  const int mc = (d->cout > 32 && !((force_mc1 || ws) && d->u_cm)) ? 2 : 1;
#else
  const int mc = (d->cout > 32 && !ws) ? 2 : 1;
#endif
  p.nco = (int)ceil_div(d->cout, 32 * mc);
  const long long tiles = (long long)p.nco * (cin / 32);
  // one workgroup per CU (LDS / 224 accumulators): S brick ranges x tiles <= 256,
  // else the last few workgroups run as a second round (cin 192: 43 x 6 = 258 ran 2x long)
  long long S = 256 / tiles;
  if (S > p.nbricks) S = p.nbricks;
  if (S < 1) S = 1;
  p.per = ceil_div(p.nbricks, S);
  S = ceil_div(p.nbricks, p.per);
  CWDM_REQUIRE(tiles < 65536, CWDM_E_SHAPE, "cwdm_conv3d_wgrad: too many channel tiles");
  dim3 grid((unsigned)S, (unsigned)tiles);
  hipStream_t s = (hipStream_t)stream;
  const bool gn = d->u_gn != nullptr;
  const long long nw = (long long)d->cout * cin * p.taps;
  int rc;
  static const bool wg1_on = !std::getenv("CWDM_WG1_OFF");   // A/B knob: the brick kernel for 1x1
  if (hw_eligible(d)) return d->dtype == CWDM_F16 ? launch_hw<f16_t>(d, s) : launch_hw<bf16_t>(d, s);
  if (wg1_on && wg1_eligible(d)) {
    // 1x1: the streaming kernel, accumulating straight into dw (no scratch)
    return d->dtype == CWDM_F16 ? launch_wg1<f16_t>(d, s) : launch_wg1<bf16_t>(d, s);
  }
  if (d->u_cm) {
    // U kept chunk-major by the forward: the DMA-staged kernel
    CWDM_REQUIRE(dtype_half(d->dtype) && d->ksize == 3 && !d->u_gn && !d->u1 && d->u_c1 == 0, CWDM_E_UNSUPPORTED,
                 "cwdm_conv3d_wgrad: u_cm needs a 16-bit dtype, ksize 3, one source and no GroupNorm prologue");
    WgDmaParams q{};
    q.D = (int)d->D; q.H = (int)d->H; q.W = (int)d->W;
    q.SD = d->u_mode == 1 ? q.D / 2 : q.D; q.SH = d->u_mode == 1 ? q.H / 2 : q.H; q.SW = d->u_mode == 1 ? q.W / 2 : q.W;
    q.tx = p.tx; q.ty = p.ty; q.tz = p.tz; q.nbricks = p.nbricks; q.per = p.per; q.nco = p.nco;
    q.cin = cin; q.cout = d->cout; q.dy_cs = d->dy_cs;
    q.units = (int)(S * tiles); q.upx = (q.units + 7) / 8;
#ifdef CWDM_WG_DIAG
    static const int wg_diag = [] { const char* e = std::getenv("CWDM_WG_DIAGMASK"); return e ? std::atoi(e) : 0; }();
    q.diag = wg_diag;
#endif
    const long long sv = (long long)q.SD * q.SH * q.SW, V = d->D * d->H * d->W;
    q.act = reinterpret_cast<const unsigned char*>(d->u0); q.act_bs = sv * cin * 2;
    q.dy = reinterpret_cast<const unsigned char*>(d->dy); q.dy_bs = V * d->dy_cs * 2;
    q.part = p.part;
    CWDM_REQUIRE(q.act_bs < (1LL << 31) && q.dy_bs < (1LL << 31), CWDM_E_UNSUPPORTED,
                 "cwdm_conv3d_wgrad: u_cm sources above 2 GB per batch");
    if (ws) {
      rc = d->dtype == CWDM_F16
               ? (d->u_mode ? launch_wg_dma<f16_t, 1, 1, true>(q, grid, s) : launch_wg_dma<f16_t, 1, 0, true>(q, grid, s))
               : (d->u_mode ? launch_wg_dma<bf16_t, 1, 1, true>(q, grid, s) : launch_wg_dma<bf16_t, 1, 0, true>(q, grid, s));
    } else {
      rc = d->dtype == CWDM_F16
               ? (mc == 2 ? (d->u_mode ? launch_wg_dma<f16_t, 2, 1>(q, grid, s) : launch_wg_dma<f16_t, 2, 0>(q, grid, s))
                          : (d->u_mode ? launch_wg_dma<f16_t, 1, 1>(q, grid, s) : launch_wg_dma<f16_t, 1, 0>(q, grid, s)))
               : (mc == 2 ? (d->u_mode ? launch_wg_dma<bf16_t, 2, 1>(q, grid, s) : launch_wg_dma<bf16_t, 2, 0>(q, grid, s))
                          : (d->u_mode ? launch_wg_dma<bf16_t, 1, 1>(q, grid, s) : launch_wg_dma<bf16_t, 1, 0>(q, grid, s)));
    }
    if (rc) return rc;
    return launch_wg_reduce(p.part, S, nw, d->dw, d->cout, cin, 27, false, s);
  }
  rc = dispatch_dtype(d->dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    return mc == 2 ? dispatch_wg<T, 2>(p, d->u_mode, gn, grid, s) : dispatch_wg<T, 1>(p, d->u_mode, gn, grid, s);
  });
  if (rc) return rc;
  return launch_wg_reduce(p.part, S, nw, d->dw, d->cout, cin, p.taps, true, s);
}

// the partial slabs: at most S_max brick / stage ranges of cout x cin x ksize^3
// fp32 each (the launch code's S never exceeds these bounds)
extern "C" int64_t cwdm_conv3d_wgrad_workspace_bytes(int cout, int cin, int ksize) {
  if (cout <= 0 || cin <= 0 || (ksize != 1 && ksize != 3)) return -1;
  const int mc = cout > 32 ? 2 : 1;
  const int64_t tiles = ceil_div((int64_t)cout, 32 * mc) * ceil_div((int64_t)cin, 32);
  int64_t smax = std::max<int64_t>(1, 256 / tiles);                      // wgrad_kernel / wgrad_dma_kernel
  if (hw_shape_ok(cout, cin, ksize)) smax = std::max<int64_t>(smax, HW_SMAX);   // head_wgrad_kernel
  if (ksize == 1) {
    const int64_t t1 = ceil_div((int64_t)cout, 64) * ceil_div((int64_t)cin, 128);
    smax = std::max(smax, std::max<int64_t>(1, 768 / t1));                // wgrad1_kernel
  }
  return smax * cout * cin * ksize * ksize * ksize * 4;
}
