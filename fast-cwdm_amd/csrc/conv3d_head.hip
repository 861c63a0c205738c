// Output head of the U-Net (unet.py `out`: GroupNorm -> SiLU -> conv3x3x3,
// model_channels -> out_channels = 8): a narrow-output conv with its
// GroupNorm+SiLU fused into the halo staging.
//
// The general kernels tile 32 / 64 output channels per MFMA; with 8 outputs
// that wastes 4-8x of the matrix work and the head ran at ~130 TF/s
// (~0.55 ms of the 128^3 step).  Here the MFMA is v_mfma_f32_16x16x32_bf16 (/ _f16)
// with A = 16 voxels x 32 input channels (from LDS) and B = 32 input channels
// x 16 output channels (8 real + zero rows, held in registers per tap): half
// the lanes of the product are useful instead of an eighth.
//
//   * Tile 32(x) x 4(y) x 4(z) voxels, 4 waves, wave w = output z-plane w:
//     4 lines x 2 x-blocks of 16 voxels = 8 accumulators (f32x4).
//   * Input channels in halves of 32: the 34 x 6 x 6 halo of a half (64 B per
//     voxel, 78 KB, so two workgroups share a CU) is loaded with 16-byte
//     loads, GroupNorm+SiLU applied in registers, zero-padded and written to
//     LDS.  A ds_read_b128 of a wave covers 16 consecutive voxels x 64 B:
//     conflict-free.  For each (dz, dx) the 6 input lines are read once and
//     used by the 3 dy taps (24 MFMAs per 12 reads).
//   * Weights come from the standard packed layout (cwdm_conv3d_pack, NT = 32
//     rows per channel tile; rows >= cout are zero).
//
// SAMP variant (cwdm_unet_forward_step): the sampling step's epilogue runs on
// the accumulators -- the tile's 512 x 8 fp32 outputs (+ bias) go through LDS
// to one thread per voxel, which applies sampler_voxel8 (sampler.hpp; the same
// function as cwdm_sampler_step, so the bits match the unfused step) and
// stores x_{t-1}, the optional pred_xstart and the 16-bit mirror into the next
// step's U-Net input.  The fp32 model output never reaches HBM, and with
// Philox noise neither does the noise tensor.
#include <atomic>
#include <cstdlib>

#include "conv3d_kernels.hpp"
#include "sampler.hpp"

namespace cwdm {

struct HeadParams {
  int B, D, H, W, C, cout;
  int tx, ty, tz;
  const void* x;            // [B][V][C] channels-last, bf16 or fp16
  const float* gn;          // [B][C][2] scale / shift (null: no GroupNorm+SiLU)
  const unsigned char* w;   // packed, NT = 32
  const float* bias; long long bias_bs;
  void* out; int out_f32;   // [B][V][cout]
  cwdm_sampler_args samp;   // SAMP only: the step (out unused)
  int mir_vec;              // SAMP: the mirror's 8 channels are 16-byte vectors
  unsigned long long* stamps;   // diagnostics (make STAMPS=1): head2 phase stamps, 64 per workgroup
};

// head2 stamps (tools/head_stamps.py): [0] start; tile k < 8: MFMA wave 0 past
// B_k [1 + 3k], MFMAs done [2 + 3k], at B_k+1 [3 + 3k]; fill wave 4 loaded +
// transformed [32 + 3k], stored [33 + 3k], at B_k+1 [34 + 3k]; [60] / [61]
// s_memrealtime at start / end of MFMA wave 0's first column, [62] s_memtime at that end
#ifdef CWDM_CONV_STAMPS
#define H2_STAMP(k, cond)                                                                        \
  do {                                                                                           \
    if (p.stamps && (cond)) p.stamps[(long long)blockIdx.x * 64 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define H2_STAMP(k, cond) do { } while (0)
#endif

namespace {

constexpr int HHX = 34, HHY = 6, HHZ = 6, HHV = HHX * HHY * HHZ;  // 1224 halo voxels
constexpr int HEAD_LDS = HHV * 64;                                 // 78336 B

typedef __bf16 hbf16x8 __attribute__((ext_vector_type(8)));
typedef float hf32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ hf32x4 head_mfma(const u32x4& a, const u32x4& b, hf32x4 acc, bf16_t*) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hbf16x8, a), __builtin_bit_cast(hbf16x8, b), acc,
                                                 0, 0, 0);
}
__device__ __forceinline__ hf32x4 head_mfma(const u32x4& a, const u32x4& b, hf32x4 acc, f16_t*) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0,
                                                0, 0);
}

// T: the 16-bit storage type (bf16 / fp16); SAMP: run the sampler epilogue
// with mirror type MirT (T or fp32)
template <typename T, bool GN, bool SAMP = false, typename MirT = T>
__global__ void __launch_bounds__(256, 2) head_conv_kernel(HeadParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char halo[HEAD_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = lane & 15, kg = lane >> 4;
  const int tiles = p.tx * p.ty * p.tz;
  // XCD-aware: workgroups are dealt round robin to the 8 XCDs; XCD j runs one
  // contiguous run of the x-fastest tile order, so a tile's y / z neighbours
  // (whose halos overlap its own 2.25x) are fetched into the same L2 (the
  // plain order put y neighbours, tx = 4 apart, on different XCDs: 3.5x the
  // input read from HBM)
  const int nb = (int)gridDim.x, xj = (int)(blockIdx.x & 7), q8 = nb >> 3, r8 = nb & 7;
  const int bid = (xj < r8 ? xj * (q8 + 1) : r8 * (q8 + 1) + (xj - r8) * q8) + (int)(blockIdx.x >> 3);
  const int b = bid / tiles, sl = bid - b * tiles;
  const int x0 = (sl % p.tx) * 32, y0 = ((sl / p.tx) % p.ty) * 4, z0 = (sl / (p.tx * p.ty)) * 4;
  const long long V = (long long)p.D * p.H * p.W;
  const int nh = p.C / 32;

  hf32x4 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int xb = 0; xb < 2; ++xb) acc[m][xb] = hf32x4{0.f, 0.f, 0.f, 0.f};

  // fill work: item i = tid + 256 k -> halo voxel i >> 2, quad i & 3 (= tid & 3 for every k);
  // the element offset (voxel * C, within the batch) of each item, -1 outside the volume
  constexpr int NFILL = (HHV * 4 + 255) / 256;  // 20
  const int fq = tid & 3;
  const T* xb = reinterpret_cast<const T*>(p.x) + (long long)b * V * p.C;
  // (recomputed per input half: 20 registers fewer across the MFMA phase)
  auto fill_off = [&](int k) {
    const int hv = (tid + 256 * k) >> 2;
    const int hx = hv % HHX, hy = (hv / HHX) % HHY, hz = hv / (HHX * HHY);
    const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
    const bool ok = hv < HHV && ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D;
    return ok ? ((oz * p.H + oy) * p.W + ox) * p.C + fq * 8 : -1;
  };
  // this lane's A-operand base: voxel (x = n, line 0, plane wv) of the halo, K group kg
  const int abase = ((wv * HHY) * HHX + n) * 64 + kg * 16;

  // SAMP: this thread's 2 voxels of the epilogue (lv = tid, tid + 256 of the
  // tile, x fastest): their x_t loads are issued here and fly during the whole conv
  int64_t vv[2] = {0, 0};
  float xv[2][8], nzv[2][8];
  int64_t ts = 0;
  bool noisy = false, philox = false;
  if constexpr (SAMP) {
    const cwdm_sampler_args& a = p.samp;
    ts = a.t[b];
    ts = ts < 0 ? 0 : (ts >= a.T ? a.T - 1 : ts);
    noisy = a.update != 1 && ts != 0;
    philox = noisy && !a.noise && a.noise_philox;
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int lv = tid + 256 * r2;
      vv[r2] = ((int64_t)(z0 + (lv >> 7)) * p.H + y0 + ((lv >> 5) & 3)) * p.W + x0 + (lv & 31);
      const float* xp = a.x_t + b * a.xt_s[0] + vv[r2] * a.xt_s[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[r2][q] = xp[q * a.xt_s[1]];
    }
  }

  for (int h = 0; h < nh; ++h) {
    if (h) __syncthreads();  // the previous half's operand reads are done
    float sc[8], sh[8];
    if constexpr (GN) {
      const float2* g2 = reinterpret_cast<const float2*>(p.gn) + (long long)b * p.C + h * 32 + fq * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 v2 = g2[e];
        silu_aff_coef(v2.x, v2.y, sc[e], sh[e]);
      }
    }
    u32x4 v[NFILL];
    int foff[NFILL];
#pragma unroll
    for (int k = 0; k < NFILL; ++k) {
      foff[k] = fill_off(k);
      v[k] = u32x4{0u, 0u, 0u, 0u};
      if (foff[k] >= 0) v[k] = *reinterpret_cast<const u32x4*>(xb + foff[k] + h * 32);
    }
#pragma unroll
    for (int k = 0; k < NFILL; ++k) {
      const int i = tid + 256 * k;
      if ((i >> 2) < HHV) {
        u32x4 q = v[k];
        if (GN && foff[k] >= 0) {
          float f[8];
          unpack<T>(v[k], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = silu_aff(f[e], sc[e], sh[e]);
          q = pack<T>(f);
        }
        *reinterpret_cast<u32x4*>(halo + i * 16) = q;
      }
    }
    // B operands of this half: tap t, lane (n, kg) = W[co n][ci h 32 + 8 kg .. + 8][t]
    u32x4 wr[27];
    {
      const int chunk = 2 * h + (kg >> 1), q = kg & 1;
      const unsigned char* src = p.w + ((long long)chunk * 27 * 32 + n) * 32 + ((q ^ ((n >> 3) & 1)) << 4);
#pragma unroll
      for (int t = 0; t < 27; ++t) wr[t] = *reinterpret_cast<const u32x4*>(src + (long long)t * 32 * 32);
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 9; ++g) {
      const int dz = g / 3, dx = g % 3;  // 0..2 (offset - 1)
      u32x4 a[6][2];
#pragma unroll
      for (int L = 0; L < 6; ++L)
#pragma unroll
        for (int xb = 0; xb < 2; ++xb)
          a[L][xb] = *reinterpret_cast<const u32x4*>(halo + abase + (((dz * HHY) + L) * HHX + xb * 16 + dx) * 64);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const u32x4 wb = wr[dz * 9 + dy * 3 + dx];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int xb = 0; xb < 2; ++xb) acc[m][xb] = head_mfma(a[m + dy][xb], wb, acc[m][xb], (T*)nullptr);
      }
    }
  }
  // epilogue: lane (n, kg) holds output channel n of voxels x = 16 xb + 4 kg + i
  if constexpr (SAMP) {
    // this thread's 2 voxels (lv = tid, tid + 256 of the tile, x fastest): the
    // x_t (and tensor-noise) loads go out first and fly during the tile exchange
    const cwdm_sampler_args& a = p.samp;
    const int64_t t = ts;
    const int bs = a.per_band ? 8 : 0;
    const float* cf = a.coef + t * (a.per_band ? 64 : 8);
    __syncthreads();  // every wave's operand reads are done: the halo becomes the output tile
    float* tile = reinterpret_cast<float*>(halo);  // [512 voxels (z, y, x)][8]
    if (n < 8) {
      const float bn = p.bias ? p.bias[(long long)b * p.bias_bs + n] : 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int xb = 0; xb < 2; ++xb)
#pragma unroll
          for (int i = 0; i < 4; ++i) tile[(((wv * 4 + m) * 32) + xb * 16 + 4 * kg + i) * 8 + n] = acc[m][xb][i] + bn;
    }
    if (noisy && a.noise) {   // tensor noise (tests): loaded here, not held across the conv
#pragma unroll
      for (int r2 = 0; r2 < 2; ++r2) {
        const float* np = a.noise + b * a.nz_s[0] + vv[r2] * a.nz_s[2];
#pragma unroll
        for (int q = 0; q < 8; ++q) nzv[r2][q] = np[q * a.nz_s[1]];
      }
    }
    if (philox) {
#pragma unroll
      for (int r2 = 0; r2 < 2; ++r2) {
        philox_normal4(a.noise_seed, vv[r2], b, t, 0, nzv[r2]);
        philox_normal4(a.noise_seed, vv[r2], b, t, 1, nzv[r2] + 4);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int lv = tid + 256 * r2;
      const int64_t v = vv[r2];
      float m8[8], r[8], pred[8];
      const float4 u0 = *reinterpret_cast<const float4*>(tile + lv * 8);
      const float4 u1 = *reinterpret_cast<const float4*>(tile + lv * 8 + 4);
      m8[0] = u0.x; m8[1] = u0.y; m8[2] = u0.z; m8[3] = u0.w;
      m8[4] = u1.x; m8[5] = u1.y; m8[6] = u1.z; m8[7] = u1.w;
      sampler_voxel8(a, cf, bs, t, m8, xv[r2], noisy && (a.noise || philox), nzv[r2], r, pred);
      float* xo = a.x_prev + b * a.xp_s[0] + v * a.xp_s[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) xo[q * a.xp_s[1]] = r[q];
      if (a.pred_xstart) {
        float* po = a.pred_xstart + b * a.px_s[0] + v * a.px_s[2];
#pragma unroll
        for (int q = 0; q < 8; ++q) po[q * a.px_s[1]] = pred[q];
      }
      if (a.mirror) {
        MirT* o = reinterpret_cast<MirT*>(a.mirror) + b * a.mr_s[0] + v * a.mr_s[2];
        bool done = false;
        if constexpr (sizeof(MirT) == 2) {
          if (p.mir_vec) {
            uint4 q;
            q.x = pack2<MirT>(r[0], r[1]);
            q.y = pack2<MirT>(r[2], r[3]);
            q.z = pack2<MirT>(r[4], r[5]);
            q.w = pack2<MirT>(r[6], r[7]);
            *reinterpret_cast<uint4*>(o) = q;
            done = true;
          }
        }
        if (!done) {
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q * a.mr_s[1]] = Elem<MirT>::from_f(r[q]);
        }
      }
    }
    return;
  }
  if (n < p.cout) {
    const float bn = p.bias ? p.bias[(long long)b * p.bias_bs + n] : 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int xb = 0; xb < 2; ++xb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long long vox =
              (long long)b * V + ((long long)(z0 + wv) * p.H + y0 + m) * p.W + x0 + xb * 16 + 4 * kg + i;
          const float r = acc[m][xb][i] + bn;
          if (p.out_f32) reinterpret_cast<float*>(p.out)[vox * p.cout + n] = r;
          else reinterpret_cast<T*>(p.out)[vox * p.cout + n] = Elem<T>::from_f(r);
        }
  }
}


// ---------------------------------------------------------------------------
// Second-generation head (64 input channels; W % 16, H % 4, D % 4): one
// persistent 512-thread workgroup per CU walks a z column of 16 x 4 x 4-voxel
// tiles.  Waves 4-7 fill: they keep a ring of 10 halo planes (18 x 6 voxels x
// 64 channels, two 32-channel halves, 13.5 KB each) in LDS.  Consecutive tiles
// of a column share 2 of their 6 halo planes, so a tile brings 4 new planes: the
// GroupNorm+SiLU transform runs on 1.69x the tile's voxels instead of the 2.39x
// of a 32 x 4 x 4 halo per tile, and on the fill waves while the MFMA waves
// compute -- the first head serialised fill and MFMAs in every workgroup (two
// per CU by LDS).  Ring slot = plane mod 10: tile k reads planes 4k - 1 .. 4k + 4,
// tile k + 1's new planes 4k + 5 .. 4k + 8 are already in, and tile k + 2's
// (4k + 9 .. 4k + 12) take the slots of tile k's first four once its MFMAs are
// done (barrier X_k).  Per tile: [B_k] MFMAs | fill loads + transforms tile
// k + 2 [X_k] epilogue | fill stores tile k + 2 [B_k+1].
// MFMA wave w = (input half h = w & 1, output planes 2 (w >> 1) + 0 / 1): its 27
// weight fragments stay in registers for the whole launch (a per-tile reload
// from L2 stalled every tap group), and after the MFMAs it hands the partial
// sums of its partner's plane over through LDS; each wave finishes one plane as
// (half 0 sum) + (half 1 sum).  SAMP: the finished 64 voxels x 8 outputs go to
// a voxel-per-lane layout through a wave-private 2 KB LDS region (no workgroup
// barrier) and run sampler_voxel8 like the first head -- deferred to after the
// next tile's MFMAs, where the MFMA waves would otherwise wait for the fill.
// a half is 6912 B + 32 B of padding: the two halves of a voxel (written by
// neighbouring lanes of a fill wave) land on different banks
constexpr int H2X = 18, H2Y = 6, H2HALF = H2Y * H2X * 64 + 32;   // 6944 B: one 32-channel half of a plane
constexpr int H2SLOT = 2 * H2HALF, H2NS = 10;
constexpr int H2P = H2NS * H2SLOT;                           // 138880: 4 partial-sum regions (4 KB)
constexpr int H2T = H2P + 4 * 4096;                          // 155264: 4 finished-plane regions (2 KB)
constexpr int H2LDS = H2T + 4 * 2048;                        // 163456 (+ 16 B: the fill's dummy word)
constexpr int H2NI = 14;                                     // fill pieces per thread (4 planes: 3456 / 256)
static_assert(H2LDS + 16 <= 163840, "head2 LDS");

struct Head2Geo {
  int cx, cy, ntz;     // 16-voxel x blocks, 4-line y blocks, 4-plane z tiles
  int zs, per;         // z segments per column, tiles per segment
  int units;           // B * cy * cx * zs
};

template <typename T, bool GN, bool SAMP = false, typename MirT = T>
__global__ void __launch_bounds__(512) head2_kernel(HeadParams p, Head2Geo g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // wave-uniform role (readfirstlane: a scalar branch, each role's registers its own)
  const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const bool mw = wv < 4;
  const int n = lane & 15, kg = lane >> 4;
  const long long V = (long long)p.D * p.H * p.W;
  // XCD-aware unit order: workgroup j of XCD x takes unit x * (grid / 8) + j of
  // the x-fastest list, so neighbouring columns (shared halo lines) share an L2
  const int gx = (int)gridDim.x;
  const int u0 = (gx % 8 == 0) ? (int)(blockIdx.x & 7) * (gx >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;

  // the unit loop inside each role: the two roles' registers never meet
  auto unit = [&](int u, int& b, int& x0, int& y0, int& tz0, int& tz1) {
    int r = u;
    const int zsi = r % g.zs; r /= g.zs;
    const int xc = r % g.cx; r /= g.cx;
    const int yc = r % g.cy;
    b = r / g.cy;
    x0 = xc * 16; y0 = yc * 4;
    tz0 = zsi * g.per; tz1 = min(g.ntz, tz0 + g.per);
  };
  H2_STAMP(0, tid == 0);
#ifdef CWDM_CONV_STAMPS
  if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 64 + 60] = __builtin_amdgcn_s_memrealtime();
#endif
  if (mw) {
    // ------------------------------------------------------------ MFMA waves
    const int h = wv & 1, pp = wv >> 1;
    // B operands of input half h, resident: tap t, lane (n, kg) = W[co n][ci 32 h + 8 kg .. + 8][t]
    u32x4 wr[27];
    {
      const int chunk = 2 * h + (kg >> 1), q = kg & 1;
      const unsigned char* src = p.w + ((long long)chunk * 27 * 32 + n) * 32 + ((q ^ ((n >> 3) & 1)) << 4);
#pragma unroll
      for (int t = 0; t < 27; ++t) wr[t] = *reinterpret_cast<const u32x4*>(src + (long long)t * 32 * 32);
    }
    const int abase = h * H2HALF + n * 64 + kg * 16;
    hf32x4* part_mine = reinterpret_cast<hf32x4*>(smem + H2P + wv * 4096);
    const hf32x4* part_other = reinterpret_cast<const hf32x4*>(smem + H2P + (wv ^ 1) * 4096);
    const int pf = 2 * pp + h;   // the output plane this wave finishes
    float* tfin = reinterpret_cast<float*>(smem + H2T + wv * 2048);   // finished plane [64 voxels][8]
    // SAMP: the sampler step of the plane in tfin (tile tzp of the column at x0, y0):
    // lane = voxel (line lane >> 4, x lane & 15)
    auto samp_plane = [&](int b, int x0, int y0, int tzp) {
      const cwdm_sampler_args& a = p.samp;
      int64_t t = a.t[b];
      t = t < 0 ? 0 : (t >= a.T ? a.T - 1 : t);
      const int bs = a.per_band ? 8 : 0;
      const float* cf = a.coef + t * (a.per_band ? 64 : 8);
      const bool noisy = a.update != 1 && t != 0;
      const bool philox = noisy && !a.noise && a.noise_philox;
      const int64_t vv = ((int64_t)(tzp * 4 + pf) * p.H + y0 + (lane >> 4)) * p.W + x0 + (lane & 15);
      float xv[8], nzv[8];
      const float* xp = a.x_t + b * a.xt_s[0] + vv * a.xt_s[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[q] = xp[q * a.xt_s[1]];
      if (noisy && a.noise) {
        const float* np = a.noise + b * a.nz_s[0] + vv * a.nz_s[2];
#pragma unroll
        for (int q = 0; q < 8; ++q) nzv[q] = np[q * a.nz_s[1]];
      }
      if (philox) {
        philox_normal4(a.noise_seed, vv, b, t, 0, nzv);
        philox_normal4(a.noise_seed, vv, b, t, 1, nzv + 4);
      }
      float m8[8], rr[8], pred[8];
      const float4 e0 = *reinterpret_cast<const float4*>(tfin + lane * 8);
      const float4 e1 = *reinterpret_cast<const float4*>(tfin + lane * 8 + 4);
      m8[0] = e0.x; m8[1] = e0.y; m8[2] = e0.z; m8[3] = e0.w;
      m8[4] = e1.x; m8[5] = e1.y; m8[6] = e1.z; m8[7] = e1.w;
      sampler_voxel8(a, cf, bs, t, m8, xv, noisy && (a.noise || philox), nzv, rr, pred);
      float* xo = a.x_prev + b * a.xp_s[0] + vv * a.xp_s[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) xo[q * a.xp_s[1]] = rr[q];
      if (a.pred_xstart) {
        float* po = a.pred_xstart + b * a.px_s[0] + vv * a.px_s[2];
#pragma unroll
        for (int q = 0; q < 8; ++q) po[q * a.px_s[1]] = pred[q];
      }
      if (a.mirror) {
        MirT* o = reinterpret_cast<MirT*>(a.mirror) + b * a.mr_s[0] + vv * a.mr_s[2];
        bool done = false;
        if constexpr (sizeof(MirT) == 2) {
          if (p.mir_vec) {
            uint4 q;
            q.x = pack2<MirT>(rr[0], rr[1]);
            q.y = pack2<MirT>(rr[2], rr[3]);
            q.z = pack2<MirT>(rr[4], rr[5]);
            q.w = pack2<MirT>(rr[6], rr[7]);
            *reinterpret_cast<uint4*>(o) = q;
            done = true;
          }
        }
        if (!done) {
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q * a.mr_s[1]] = Elem<MirT>::from_f(rr[q]);
        }
      }
    };
    for (int u = u0; u < g.units; u += gx) {
      int b, x0, y0, tz0, tz1;
      unit(u, b, x0, y0, tz0, tz1);
      const float bn = (n < p.cout && p.bias) ? p.bias[(long long)b * p.bias_bs + n] : 0.f;
      __syncthreads();   // B_tz0: the prologue planes are in
      for (int tz = tz0; tz < tz1; ++tz) {
        const int z0 = tz * 4;
        [[maybe_unused]] const int ks = tz - tz0;
        H2_STAMP(1 + 3 * ks, tid == 0 && ks < 8 && u == u0);
        // SAMP: the previous tile's sampler step runs after this tile's MFMAs (the
        // MFMA waves wait for the fill there)
        hf32x4 acc[2][4];
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[pl][m] = hf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int dz = 0; dz < 3; ++dz)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) {
              const int pz = z0 - 1 + 2 * pp + pl + dz;
              const unsigned char* sl = smem + ((pz + H2NS) % H2NS) * H2SLOT + abase + dx * 64;
              u32x4 a[6];
#pragma unroll
              for (int L = 0; L < 6; ++L) a[L] = *reinterpret_cast<const u32x4*>(sl + L * H2X * 64);
#pragma unroll
              for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int m = 0; m < 4; ++m)
                  acc[pl][m] = head_mfma(a[m + dy], wr[dz * 9 + dy * 3 + dx], acc[pl][m], (T*)nullptr);
            }
        H2_STAMP(2 + 3 * ks, tid == 0 && ks < 8 && u == u0);
        // the partner's plane goes to it; X_k: every wave is past its ring reads too
        hf32x4 fin[4];
        if (h == 0) {
#pragma unroll
          for (int m = 0; m < 4; ++m) part_mine[m * 64 + lane] = acc[1][m];
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m) part_mine[m * 64 + lane] = acc[0][m];
        }
        // (the partner read this region before B_k: it may be rewritten any time in tile k)
        if constexpr (SAMP) {
          if (tz > tz0) samp_plane(b, x0, y0, tz - 1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (h == 0) {
#pragma unroll
          for (int m = 0; m < 4; ++m) fin[m] = acc[0][m] + part_other[m * 64 + lane];   // half 0 + half 1
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m) fin[m] = part_other[m * 64 + lane] + acc[1][m];   // half 0 + half 1
        }
        asm volatile("" ::: "memory");   // the partial reads stay ahead of the transpose writes into that region
        // epilogue: lane (n, kg) holds output channel n of voxels x = 4 kg + i, line m of plane pf
        if constexpr (SAMP) {
          // the finished plane -> this wave's region ([64 voxels][8]); its sampler
          // step runs after the next tile's MFMAs (or after the column)
          if (n < 8) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
              for (int i = 0; i < 4; ++i) tfin[(m * 16 + 4 * kg + i) * 8 + n] = fin[m][i] + bn;
          }
        } else {
          if (n < p.cout) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const long long vox = (long long)b * V + ((long long)(z0 + pf) * p.H + y0 + m) * p.W + x0 + 4 * kg + i;
                const float rv = fin[m][i] + bn;
                if (p.out_f32) reinterpret_cast<float*>(p.out)[vox * p.cout + n] = rv;
                else reinterpret_cast<T*>(p.out)[vox * p.cout + n] = Elem<T>::from_f(rv);
              }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        H2_STAMP(3 + 3 * ks, tid == 0 && ks < 8 && u == u0);
        __builtin_amdgcn_s_barrier();   // B_k+1: the partials are read, tile k + 2's planes are in
      }
      if constexpr (SAMP) {
        // the column's last tile
        samp_plane(b, x0, y0, tz1 - 1);
      }
#ifdef CWDM_CONV_STAMPS
      if (p.stamps && tid == 0 && u == u0) {
        p.stamps[(long long)blockIdx.x * 64 + 61] = __builtin_amdgcn_s_memrealtime();
        p.stamps[(long long)blockIdx.x * 64 + 62] = __builtin_amdgcn_s_memtime();
      }
#endif
    }
  } else {
    for (int u = u0; u < g.units; u += gx) {
      int b, x0, y0, tz0, tz1;
      unit(u, b, x0, y0, tz0, tz1);
      // ------------------------------------------------------------ fill waves
      const int ht = tid - 256, fq = ht & 7;   // this thread's 8 channels: 8 fq .. 8 fq + 7 (both halves: fq >> 2)
      float sa[8], sb8[8];
      if constexpr (GN) {
        const float2* g2 = reinterpret_cast<const float2*>(p.gn) + (long long)b * p.C + fq * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float2 v2 = g2[e];
          silu_aff_coef(v2.x, v2.y, sa[e], sb8[e]);
        }
      }
      const T* xb = reinterpret_cast<const T*>(p.x) + (long long)b * V * p.C;
      // piece i (16 bytes: voxel pc >> 3 of a plane group, channels 8 fq ..) of
      // this thread, decoded once per column: its element offset within a plane
      // (-1: outside the volume in x / y) and its LDS offset within a slot | the
      // plane of the group << 16.  Everything below is branch-free: a padding
      // piece loads from an out-of-range offset (zeros) and keeps them through
      // the transform (select), a piece past the group writes a dummy LDS word.
      const int pel = p.H * p.W * p.C;
      int pbase[H2NI], pinfo[H2NI];
#pragma unroll
      for (int i = 0; i < H2NI; ++i) {
        const int pc = ht + 256 * i, vox = pc >> 3;
        const int pl = vox / (H2X * H2Y), rr = vox - pl * (H2X * H2Y), yy = rr / H2X, xx = rr - yy * H2X;
        const int gy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        const bool ok = gy >= 0 && gy < p.H && gxx >= 0 && gxx < p.W;
        pbase[i] = ok ? (gy * p.W + gxx) * p.C + fq * 8 : -1;
        pinfo[i] = ((fq >> 2) * H2HALF + (yy * H2X + xx) * 64 + (fq & 3) * 16) | (pl << 16);
      }
      // 32-bit buffer offsets (no 64-bit address per piece)
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void*)xb, (short)0, (int)min((long long)V * p.C * (long long)sizeof(T), 0x7FFFFFF0LL), 0x00020000);
      unsigned okm = 0;   // pieces of the group holding volume data (bit i)
      auto load = [&](u32x4 (&R)[H2NI], int pz0, int np) {
        okm = 0;
#pragma unroll
        for (int i = 0; i < H2NI; ++i) {
          const int pl = pinfo[i] >> 16, pz = pz0 + pl;
          const bool ok = pl < np && pbase[i] >= 0 && pz >= 0 && pz < p.D;
          const unsigned vo = ok ? (unsigned)(pbase[i] + pz * pel) * (unsigned)sizeof(T) : 0xFFFFFFF0u;
          R[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo, 0, 0));
          okm |= ok ? (1u << i) : 0u;
        }
      };
      auto transform = [&](u32x4 (&R)[H2NI]) {
        if constexpr (GN) {
#pragma unroll
          for (int i = 0; i < H2NI; ++i) {
            float f[8];
            unpack<T>(R[i], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = silu_aff(f[e], sa[e], sb8[e]);
            const u32x4 y = pack<T>(f);
            const bool ok = (okm >> i) & 1u;   // zero padding stays zero (the conv pads the activated input)
            R[i] = u32x4{ok ? y[0] : 0u, ok ? y[1] : 0u, ok ? y[2] : 0u, ok ? y[3] : 0u};
          }
        }
        // the loads / transform complete here, not sunk past the next barrier
#pragma unroll
        for (int i = 0; i < H2NI; ++i) asm volatile("" ::"v"(R[i]));
      };
      auto store = [&](const u32x4 (&R)[H2NI], int pz0, int np) {
        const int s0 = (pz0 + H2NS) % H2NS;
#pragma unroll
        for (int i = 0; i < H2NI; ++i) {
          const int pl = pinfo[i] >> 16;
          int sl = s0 + pl;
          sl -= sl >= H2NS ? H2NS : 0;
          const int lds = pl < np ? sl * H2SLOT + (pinfo[i] & 0xFFFF) : H2LDS;   // (H2LDS: the dummy word)
          *reinterpret_cast<u32x4*>(smem + lds) = R[i];
        }
      };
      u32x4 R[H2NI];
      // prologue: tile tz0's 6 planes (two groups of 3) and tile tz0 + 1's 4 (10 slots)
      load(R, 4 * tz0 - 1, 3);
      transform(R);
      store(R, 4 * tz0 - 1, 3);
      load(R, 4 * tz0 + 2, 3);
      transform(R);
      store(R, 4 * tz0 + 2, 3);
      if (tz0 + 1 < tz1) {
        load(R, 4 * tz0 + 5, 4);
        transform(R);
        store(R, 4 * tz0 + 5, 4);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();   // B_tz0
      for (int tz = tz0; tz < tz1; ++tz) {
        [[maybe_unused]] const int ks = tz - tz0;
        // under tile tz's MFMAs: fetch and transform tile tz + 2's planes (issuing
        // them one tile earlier, after the stores, measured slower: 271 vs 227 us
        // in the step -- they queue behind the epilogue's stores)
        const bool more = tz + 2 < tz1;
        if (more) {
          load(R, 4 * tz + 9, 4);
          transform(R);
        }
        H2_STAMP(32 + 3 * ks, tid == 256 && ks < 8 && u == u0);
        __builtin_amdgcn_s_barrier();   // X_tz: tile tz's ring reads are done
        if (more) store(R, 4 * tz + 9, 4);
        H2_STAMP(33 + 3 * ks, tid == 256 && ks < 8 && u == u0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        H2_STAMP(34 + 3 * ks, tid == 256 && ks < 8 && u == u0);
        __builtin_amdgcn_s_barrier();   // B_tz+1
      }
    }
  }
}
}  // namespace

extern std::atomic<int> g_conv_path;

namespace {
bool head2_ok(const cwdm_conv3d_desc* d);
}

bool head_eligible(const cwdm_conv3d_desc* d) {
  if (g_conv_path.load(std::memory_order_relaxed) == 1) return false;
  return dtype_half(d->dtype) && d->a_w && d->cout <= 16 && d->a_c1 == 0 && d->a_c0 % 32 == 0 && d->a_c0 <= 256 &&
         d->a_mode == 0 && !d->b_w && d->res_mode < 0 && !d->stats && !d->out1 && !d->accumulate &&
         (d->W % 32 == 0 || head2_ok(d)) && d->H % 4 == 0 && d->D % 4 == 0 && d->D * d->H * d->W * d->a_c0 < (1LL << 31);
}

extern std::atomic<unsigned long long*> g_stamps;   // conv3d_v4.hip (cwdm_debug_conv_stamps)
// cwdm_debug_head2 (initial value: env CWDM_HEAD2=0 the first head, else the second)
std::atomic<int> g_head2{[] { const char* e = std::getenv("CWDM_HEAD2"); return (e && e[0] == '0') ? -1 : 0; }()};

namespace {
// the second-generation head where its shape holds
bool head2_ok(const cwdm_conv3d_desc* d) {
  return g_head2.load(std::memory_order_relaxed) >= 0 && d->a_c0 == 64 && d->W % 16 == 0 && d->H % 4 == 0 &&
         d->D % 4 == 0;
}

Head2Geo head2_geo(const HeadParams& p, int& grid) {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  Head2Geo g{};
  g.cx = p.W / 16; g.cy = p.H / 4; g.ntz = p.D / 4;
  const long long cols = (long long)p.B * g.cx * g.cy;
  long long zs = std::min<long long>(std::max<long long>(1, ceil_div((long long)ncu, cols)), g.ntz);
  g.per = (int)ceil_div((long long)g.ntz, zs);
  g.zs = (int)ceil_div((long long)g.ntz, (long long)g.per);
  g.units = (int)(cols * g.zs);
  grid = std::min(g.units, ncu);
  const int cap = g_head2.load(std::memory_order_relaxed);
  if (cap > 0) grid = std::min(grid, cap);
  return g;
}

template <typename T, bool GN, bool SAMP, typename MirT>
int head2_launch(HeadParams p, hipStream_t s) {
  p.stamps = g_stamps.load(std::memory_order_relaxed);
  int grid = 0;
  const Head2Geo g = head2_geo(p, grid);
  auto k = head2_kernel<T, GN, SAMP, MirT>;
  CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, H2LDS + 16));
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(512), H2LDS + 16, s, p, g);
  return CWDM_OK;
}
}  // namespace

int head_conv_forward(const cwdm_conv3d_desc* d, hipStream_t s) {
  HeadParams p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W; p.C = d->a_c0; p.cout = d->cout;
  p.tx = p.W / 32; p.ty = p.H / 4; p.tz = p.D / 4;
  p.x = d->a0;
  p.gn = d->a_gn;
  p.w = reinterpret_cast<const unsigned char*>(d->a_w);
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.out = d->out; p.out_f32 = d->out_dtype == CWDM_F32;
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d head: grid too large");
  prof_begin(s);
  const dim3 grid((unsigned)nblk);
  if (head2_ok(d)) {
    int rc;
    if (d->dtype == CWDM_F16) rc = p.gn ? head2_launch<f16_t, true, false, f16_t>(p, s) : head2_launch<f16_t, false, false, f16_t>(p, s);
    else rc = p.gn ? head2_launch<bf16_t, true, false, bf16_t>(p, s) : head2_launch<bf16_t, false, false, bf16_t>(p, s);
    if (rc) return rc;
  } else if (d->dtype == CWDM_F16) {
    if (p.gn) hipLaunchKernelGGL((head_conv_kernel<f16_t, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<f16_t, false>), grid, dim3(256), 0, s, p);
  } else {
    if (p.gn) hipLaunchKernelGGL((head_conv_kernel<bf16_t, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<bf16_t, false>), grid, dim3(256), 0, s, p);
  }
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * p.C);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

bool head_sampler_eligible(const cwdm_conv3d_desc* d, const cwdm_sampler_args* a) {
  // CWDM_HEAD_SAMPLER=0: the unfused forward + cwdm_sampler_step (A/B switch)
  static const bool on = [] { const char* e = std::getenv("CWDM_HEAD_SAMPLER"); return !(e && e[0] == '0'); }();
  return on && head_eligible(d) && d->a_gn && d->cout == 8 && a->levels <= 1 && a->B == d->B && a->d == d->D && a->h == d->H &&
         a->w == d->W && a->x_t && a->x_prev && a->coef && a->t && a->T > 0 &&
         (!a->mirror || a->mirror_dtype == d->dtype || a->mirror_dtype == CWDM_F32);
}

int head_sampler_forward(const cwdm_conv3d_desc* d, const cwdm_sampler_args* a, hipStream_t s) {
  HeadParams p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W; p.C = d->a_c0; p.cout = d->cout;
  p.tx = p.W / 32; p.ty = p.H / 4; p.tz = p.D / 4;
  p.x = d->a0;
  p.gn = d->a_gn;
  p.w = reinterpret_cast<const unsigned char*>(d->a_w);
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.samp = *a;
  const int mesz = a->mirror ? dtype_size(a->mirror_dtype) : 0;
  p.mir_vec = a->mirror && a->mr_s[1] == 1 && ((uintptr_t)a->mirror % 16) == 0 && (a->mr_s[0] * mesz) % 16 == 0 &&
              (a->mr_s[2] * mesz) % 16 == 0;
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d head: grid too large");
  const bool f32m = a->mirror && a->mirror_dtype == CWDM_F32;
  prof_begin(s);
  if (head2_ok(d)) {
    int rc;
    if (d->dtype == CWDM_F16)
      rc = f32m ? head2_launch<f16_t, true, true, float>(p, s) : head2_launch<f16_t, true, true, f16_t>(p, s);
    else
      rc = f32m ? head2_launch<bf16_t, true, true, float>(p, s) : head2_launch<bf16_t, true, true, bf16_t>(p, s);
    if (rc) return rc;
  } else if (d->dtype == CWDM_F16) {
    if (f32m) hipLaunchKernelGGL((head_conv_kernel<f16_t, true, true, float>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<f16_t, true, true, f16_t>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  } else {
    if (f32m) hipLaunchKernelGGL((head_conv_kernel<bf16_t, true, true, float>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<bf16_t, true, true, bf16_t>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  }
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * p.C);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

// ---------------------------------------------------------------------------
// The accurate fast mode's output head (fp32 storage): the head conv as a bf16
// conv over a K-expanded input, x3 = [hi(y) | lo(y) | hi(y)] with y =
// SiLU(GN(x)), lo = bf16(y - hi), against weights [hi(w) | hi(w) | lo(w)]
// (head_split3_pack) -- the three products hi.hi + lo.hi + hi.lo of the split
// conv kernels, summed by ONE bf16 head launch in fp32 accumulators.  The exact-
// fp32 brick kernel it replaces ran the 64 -> 8 head at 128^3 in 2.2 ms.
// ---------------------------------------------------------------------------
namespace {
// one thread per (voxel, 8-channel group) of the C-channel fp32 input
__global__ void __launch_bounds__(256) head_split3_prep_kernel(const float* __restrict__ x, const float* __restrict__ gn,
                                                               long long rows, long long V, int C,
                                                               unsigned short* __restrict__ x3) {
  const int Q = C / 8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * Q) return;
  const long long r = i / Q;
  const int q = (int)(i - r * Q);
  const long long b = r / V;
  const float4 a0 = *reinterpret_cast<const float4*>(x + r * C + q * 8);
  const float4 a1 = *reinterpret_cast<const float4*>(x + r * C + q * 8 + 4);
  float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float* g = gn + (b * C + q * 8) * 2;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float sa, sb;
    silu_aff_coef(g[2 * e], g[2 * e + 1], sa, sb);
    v[e] = silu_aff(v[e], sa, sb);
  }
  u32x4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = pack2<bf16_t>(v[2 * e], v[2 * e + 1]);
    lo[e] = pack2<bf16_t>(v[2 * e] - lo2f<bf16_t>(hi[e]), v[2 * e + 1] - hi2f<bf16_t>(hi[e]));
  }
  unsigned short* o = x3 + r * 3 * C + q * 8;
  *reinterpret_cast<u32x4*>(o) = hi;
  *reinterpret_cast<u32x4*>(o + C) = lo;
  *reinterpret_cast<u32x4*>(o + 2 * C) = hi;
}

// w [cout][cin][27] fp32 -> w3 [cout][3 cin][27] fp32 = [hi(w) | hi(w) | lo(w)] (bf16-exact values)
__global__ void head_split3_w_kernel(const float* __restrict__ w, int cout, int cin, int taps, float* __restrict__ w3) {
  const long long n = (long long)cout * cin * taps;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long co = i / ((long long)cin * taps), rest = i - co * cin * taps;
    const float v = w[i];
    const float hi = lo2f<bf16_t>(pack2<bf16_t>(v, 0.f));
    const float lo = lo2f<bf16_t>(pack2<bf16_t>(v - hi, 0.f));
    float* o = w3 + co * 3 * cin * taps + rest;
    o[0] = hi;
    o[(long long)cin * taps] = hi;
    o[2LL * cin * taps] = lo;
  }
}
// the small grids' version (conv3d_sg over a K-expanded input): two channels-last fp32 sources
// (a concat), SiLU(GN) applied if gn is given, output chunk-major [B][3C / 16][V][16] bf16 (cm: the
// 3x3x3 conv's source -- channel j of [hi | lo | hi] in chunk j / 16) or channels-last [B][V][3C]
// (the 1x1 skip's)
__global__ void __launch_bounds__(256) split3_cm_kernel(const float* __restrict__ x0, int c0,
                                                        const float* __restrict__ x1, int c1,
                                                        const float* __restrict__ gn, long long rows, long long V,
                                                        int cm, unsigned short* __restrict__ x3) {
  const int C = c0 + c1, Q = C / 8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * Q) return;
  const long long r = i / Q;
  const int q = (int)(i - r * Q);
  const long long b = r / V, v = r - b * V;
  const bool first = 8 * q < c0;
  const float* src = first ? x0 + r * c0 + 8 * q : x1 + r * c1 + (8 * q - c0);
  const float4 a0 = *reinterpret_cast<const float4*>(src);
  const float4 a1 = *reinterpret_cast<const float4*>(src + 4);
  float y[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  if (gn) {   // (null: an input activated upstream, e.g. cwdm_gn_silu_pool's)
    const float* g = gn + (b * C + 8 * q) * 2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float sa, sb;
      silu_aff_coef(g[2 * e], g[2 * e + 1], sa, sb);
      y[e] = silu_aff(y[e], sa, sb);
    }
  }
  u32x4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = pack2<bf16_t>(y[2 * e], y[2 * e + 1]);
    lo[e] = pack2<bf16_t>(y[2 * e] - lo2f<bf16_t>(hi[e]), y[2 * e + 1] - hi2f<bf16_t>(hi[e]));
  }
  const long long nk = 3 * C / 16;
  auto at = [&](int j) { return cm ? x3 + ((b * nk + j / 16) * V + v) * 16 + (j % 16) : x3 + r * 3 * C + j; };
  *reinterpret_cast<u32x4*>(at(8 * q)) = hi;
  *reinterpret_cast<u32x4*>(at(C + 8 * q)) = lo;
  *reinterpret_cast<u32x4*>(at(2 * C + 8 * q)) = hi;
}
}  // namespace

int head_split3_prep(const float* x, const float* gn, int64_t B, int64_t V, int C, void* x3, hipStream_t s) {
  CWDM_REQUIRE(x && gn && x3 && C % 8 == 0 && B > 0 && V > 0, CWDM_E_INVALID, "head_split3_prep: bad arguments");
  const long long items = B * V * (C / 8);
  hipLaunchKernelGGL(head_split3_prep_kernel, dim3((unsigned)ceil_div(items, 256)), dim3(256), 0, s, x, gn, (long long)B * V,
                     (long long)V, C, reinterpret_cast<unsigned short*>(x3));
  CWDM_LAUNCHED();
  return CWDM_OK;
}

int split3_prep(const float* x0, int c0, const float* x1, int c1, const float* gn, int64_t B, int64_t V, int cm,
                void* x3, hipStream_t s) {
  CWDM_REQUIRE(x0 && x3 && (c1 == 0 || x1) && c0 % 8 == 0 && c1 % 8 == 0 && (c0 + c1) % 16 == 0 && B > 0 && V > 0,
               CWDM_E_INVALID, "split3_prep: bad arguments");
  const long long items = B * V * ((c0 + c1) / 8);
  hipLaunchKernelGGL(split3_cm_kernel, dim3((unsigned)ceil_div(items, 256)), dim3(256), 0, s, x0, c0, x1, c1, gn,
                     (long long)(B * V), (long long)V, cm, reinterpret_cast<unsigned short*>(x3));
  CWDM_LAUNCHED();
  return CWDM_OK;
}

// the K-expanded split weights of a head conv, packed bf16 at out (cwdm_conv3d_packed_bytes(cout, 3 cin,
// 3, BF16) bytes); tmp: 3 cout cin 27 fp32 scratch
int head_split3_pack(const float* w, int cout, int cin, float* tmp, void* out, hipStream_t s, int k) {
  hipLaunchKernelGGL(head_split3_w_kernel, dim3(256), dim3(256), 0, s, w, cout, cin, k * k * k, tmp);
  CWDM_LAUNCHED();
  return cwdm_conv3d_pack(tmp, cout, 3 * cin, k, CWDM_BF16, out, (cwdm_stream_t)s);
}

}  // namespace cwdm

extern "C" int cwdm_debug_head2(int mode) {
  CWDM_REQUIRE(mode >= -1, CWDM_E_INVALID, "cwdm_debug_head2: mode >= -1");
  return cwdm::g_head2.exchange(mode);
}
