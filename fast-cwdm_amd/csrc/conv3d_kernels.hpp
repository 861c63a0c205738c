// Kernel templates of the conv3d implicit GEMM (included by the explicit
// instantiation units conv3d_inst_*.hip and by conv3d.hip for declarations).
#pragma once
// Conv3d (3x3x3, stride 1, pad 1) + optional 1x1 segment as an implicit GEMM on
// CDNA4 MFMA, with the U-Net ResBlock fusions (see include/cwdm.h).
//
// Work decomposition (one 256-thread workgroup = 4 waves):
//   * output tile = a brick of BX*BY*BZ = 256 voxels (GEMM rows) x NT = 32*NF
//     output channels (GEMM columns); wave w owns rows [64w, 64w+64) = two
//     32-row MFMA fragments, all NT columns.
//   * K is walked in chunks of CK input channels (32 bytes per voxel: 16 bf16
//     or 8 fp32).  Per chunk the workgroup stages into LDS
//       - the halo brick (BX+2)(BY+2)(BZ+2) x CK of the conv INPUT, computed
//         on the fly from the source tensor(s): GroupNorm scale/shift + SiLU,
//         nearest-x2 upsample or 2x2x2 average pool, zero padding, and the
//         two-tensor channel concat;
//       - the chunk's packed weights for all 27 taps [tap][n][CK].
//     then every wave runs 27 taps x (2 x NF) MFMAs reading A rows as shifted
//     halo voxels -- the im2col matrix is never materialised.
//   * LDS rows are 32 B; the 16-B half a lane reads is XOR-swizzled with bit 3
//     of the row index so the 16-lane groups of ds_read_b128 hit 16 distinct
//     bank slots for any 16 rows that are distinct mod 16.
//   * epilogue: accumulators -> LDS (fp32) -> row-major, + per-(b, c) bias,
//     + residual (same / upsampled / pooled), store, and per-tile per-channel
//     (sum, sum^2) partials for the next GroupNorm.
// bf16 uses v_mfma_f32_32x32x16_bf16, fp16 v_mfma_f32_32x32x16_f16 (same rate);
// fp32 (parity mode) uses exact-f32 v_mfma_f32_32x32x2_f32.  Accumulation is
// fp32 in all three.
#include "common.hpp"

namespace cwdm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct ConvParams {
  int B, D, H, W;
  int tx, ty, tz;  // spatial tiles per axis
  int cout, nct;   // output channels, channel tiles
  const void* a0; int ac0; const void* a1; int ac1; int amode; const float* agn; const void* aw;
  const void* b0; int bc0; const void* b1; int bc1; const void* bw;
  const float* bias; long long bias_bs;
  const void* res; int rmode;
  void* out; int out_f32;
  float* stats;
  void* out1; int out_c0;  // dual output: channels >= out_c0 go to out1 (stride cout - out_c0)
  int accumulate;          // out += result (gradient accumulation)
  int ksplit;       // K split factor S (1 = none)
  float* partial;   // [S][B*D*H*W][cout] fp32 partial sums when S > 1
};

template <typename T> struct ConvTr;
template <> struct ConvTr<bf16_t> { static constexpr int CK = 16; static constexpr int EPQ = 8; };
template <> struct ConvTr<f16_t> { static constexpr int CK = 16; static constexpr int EPQ = 8; };
template <> struct ConvTr<float> { static constexpr int CK = 8; static constexpr int EPQ = 4; };

// SiLU with the hardware exp2 / reciprocal (1-2 ulp; the reference's fp32 SiLU is
// itself an approximation of x*sigmoid(x) at that level): 5 VALU ops instead of
// an IEEE division sequence.
__device__ __forceinline__ float silu(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.4426950408889634f));
}

// SiLU(x sc + sh) with the affine folded into exp2's argument: a = -sc log2(e),
// b = -sh log2(e) (silu_aff_coef), t = x a + b = -z log2(e), and
// z / (1 + 2^t) = t / (-log2(e) (1 + 2^t)): fma, exp2, fma, rcp, mul -- 5 VALU
// (2 transcendental) instead of 6.  The GroupNorm pre-pass (cwdm_gn_apply) and
// the warp-specialised conv's in-LDS transform both use it: bit-identical.
__device__ __forceinline__ void silu_aff_coef(float sc, float sh, float& a, float& b) {
  a = sc * -1.4426950408889634f;
  b = sh * -1.4426950408889634f;
}
__device__ __forceinline__ float silu_aff(float x, float a, float b) {
  const float t = __builtin_fmaf(x, a, b);
  return t * __builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(t), -1.4426950408889634f, -1.4426950408889634f));
}

// 16-byte quad <-> floats
template <typename T>
__device__ __forceinline__ void unpack(const u32x4& q, float* f);
template <>
__device__ __forceinline__ void unpack<bf16_t>(const u32x4& q, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(q[i] << 16);
    f[2 * i + 1] = __uint_as_float(q[i] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void unpack<f16_t>(const u32x4& q, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = lo2f<f16_t>(q[i]);
    f[2 * i + 1] = hi2f<f16_t>(q[i]);
  }
}
template <>
__device__ __forceinline__ void unpack<float>(const u32x4& q, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = __uint_as_float(q[i]);
}
template <typename T>
__device__ __forceinline__ u32x4 pack(const float* f);
template <>
__device__ __forceinline__ u32x4 pack<bf16_t>(const float* f) {
  u32x4 q;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = pack2<bf16_t>(f[2 * i], f[2 * i + 1]);  // one v_cvt_pk_bf16_f32 per pair
  return q;
}
template <>
__device__ __forceinline__ u32x4 pack<f16_t>(const float* f) {
  u32x4 q;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = pack2<f16_t>(f[2 * i], f[2 * i + 1]);
  return q;
}
template <>
__device__ __forceinline__ u32x4 pack<float>(const float* f) {
  u32x4 q;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = __float_as_uint(f[i]);
  return q;
}

// one MFMA step of K = 32 bytes per operand lane (16 bf16 / fp16 elements over
// the lane pair, or 4 x the exact-fp32 K = 2 form): acc += A . B
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void mfma_acc(f32x16& acc, const u32x4& a, const u32x4& b, bf16_t*) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                               0, 0);
}
__device__ __forceinline__ void mfma_acc(f32x16& acc, const u32x4& a, const u32x4& b, f16_t*) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0,
                                              0, 0);
}
__device__ __forceinline__ void mfma_acc(f32x16& acc, const u32x4& a, const u32x4& b, float*) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a[s]), __uint_as_float(b[s]), acc, 0, 0, 0);
}

__device__ __forceinline__ u32x4 ldg16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }

template <typename T, int BX, int BY, int BZ, int NF>
struct ConvCfg {
  static constexpr int HX = BX + 2, HY = BY + 2, HZ = BZ + 2, HV = HX * HY * HZ;
  static constexpr int NT = 32 * NF;
  static constexpr int HALO_B = HV * 32;
  static constexpr int WB = 27 * NT * 32;
  static constexpr int EPI_LD = NT + 4;
  static constexpr int EPI_B = 256 * EPI_LD * 4;
  static constexpr int RED_B = 256 * 16 * 4;
  static constexpr int MAIN_B = HALO_B + WB;
  static constexpr int SMEM = MAIN_B > (EPI_B > RED_B ? EPI_B : RED_B) ? MAIN_B : (EPI_B > RED_B ? EPI_B : RED_B);
  static_assert(BX * BY * BZ == 256, "brick must be 256 voxels");
};

// Chunk staging.  Halo (or, for the 1x1 segment, brick-interior) items are
// (voxel, 16-byte quad) pairs, two threads per voxel.  fetch() issues every
// global load of a chunk into registers (nothing waits), store() transforms
// (GroupNorm scale/shift + SiLU, compile-time) and writes the swizzled LDS
// image.  The main loop calls fetch(c+1) before the MFMAs of chunk c, so HBM
// latency hides behind compute.  MODE: 0 same grid, 1 nearest-x2 upsample
// (source at half resolution), 2 AvgPool2 (source at double resolution; no
// prefetch: 8 loads per item are done inside store()).
template <typename T, int BX, int BY, int BZ, int MODE, bool GN>
struct Stager {
  static constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ;
  static constexpr int HX = BX + 2, HY = BY + 2, HV = HX * HY * (BZ + 2);
  static constexpr int NI = (HV + 127) / 128;
  u32x4 r[NI];
  unsigned ok;
  int vox[NI];          // cached source voxel index per halo item (segment A)
  unsigned cache_ok = 0;
  bool cached = false;
  float sc[EPQ], sh[EPQ];
  const T* base;
  int csrc;
  bool seg_a;

  __device__ __forceinline__ void coords(int it, bool interior, int* hv, int* hx, int* hy, int* hz) const {
    if (interior) { *hx = it % BX + 1; *hy = (it / BX) % BY + 1; *hz = it / (BX * BY) + 1; }
    else { *hx = it % HX; *hy = (it / HX) % HY; *hz = it / (HX * HY); }
    *hv = (*hz * HY + *hy) * HX + *hx;
  }

  // GroupNorm scale/shift of this thread's quad (fetch() does it unless told
  // to defer it, so the 2*EPQ registers are not live while the loads fly)
  __device__ __forceinline__ void load_gn(const ConvParams& p, int chunk, int b, int tid) {
    const int q = tid & 1;
    const int cb = chunk * CK + q * EPQ;
    const int ctot = p.ac0 + p.ac1;
#pragma unroll
    for (int e = 0; e < EPQ; ++e) {
      sc[e] = p.agn[((long long)b * ctot + cb + e) * 2 + 0];
      sh[e] = p.agn[((long long)b * ctot + cb + e) * 2 + 1];
    }
  }

  template <bool LOAD_GN = true>
  __device__ __forceinline__ void fetch(const ConvParams& p, bool segA, int chunk, int b, int x0, int y0, int z0,
                                        int tid) {
    seg_a = segA;
    const int q = tid & 1;
    const int c0 = segA ? p.ac0 : p.bc0, c1 = segA ? p.ac1 : p.bc1;
    const int cb = chunk * CK + q * EPQ;
    const void* src;
    int ch;
    if (cb < c0) { src = segA ? p.a0 : p.b0; ch = cb; csrc = c0; }
    else { src = segA ? p.a1 : p.b1; ch = cb - c0; csrc = c1; }
    base = reinterpret_cast<const T*>(src) + ch;
    if (GN && segA && LOAD_GN) {
      const int ctot = c0 + c1;
#pragma unroll
      for (int e = 0; e < EPQ; ++e) {
        sc[e] = p.agn[((long long)b * ctot + cb + e) * 2 + 0];
        sh[e] = p.agn[((long long)b * ctot + cb + e) * 2 + 1];
      }
    }
    ok = 0;
    if (MODE == 2 && segA) return;
    const bool interior = !segA;
    if (segA) {
      // source voxel indices of the halo items are chunk-invariant: computed once
      if (!cached) {
        cache_ok = 0;
        const int SD = MODE == 1 ? p.D >> 1 : p.D, SH = MODE == 1 ? p.H >> 1 : p.H, SW = MODE == 1 ? p.W >> 1 : p.W;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int it = (tid >> 1) + 128 * j;
          vox[j] = 0;
          if (it < HV) {
            int hv, hx, hy, hz;
            coords(it, false, &hv, &hx, &hy, &hz);
            int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
            if (ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) {
              if (MODE == 1) { ox >>= 1; oy >>= 1; oz >>= 1; }
              vox[j] = ((b * SD + oz) * SH + oy) * SW + ox;
              cache_ok |= 1u << j;
            }
          }
        }
        cached = true;
      }
      ok = cache_ok;
      // branch-free: out-of-volume items load voxel 0 and are zeroed later
#pragma unroll
      for (int j = 0; j < NI; ++j) r[j] = ldg16(base + (long long)vox[j] * csrc);
      return;
    }
    const int n = BX * BY * BZ;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int it = (tid >> 1) + 128 * j;
      r[j] = u32x4{0u, 0u, 0u, 0u};
      if (it < n) {
        int hv, hx, hy, hz;
        coords(it, interior, &hv, &hx, &hy, &hz);
        const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
        if (ox < p.W && oy < p.H && oz < p.D) {
          const long long v = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
          r[j] = ldg16(base + v * csrc);
          ok |= 1u << j;
        }
      }
    }
  }

  // in-place GroupNorm+SiLU of fetched item j (MODE 0/1 only)
  template <int J>
  __device__ __forceinline__ void transform_item() {
    if constexpr (J < NI) {
      if (MODE == 2 || !seg_a) return;
      // mask as data, not control flow: keeps the VALU stream branch-free so it
      // can interleave with the MFMAs
      const unsigned keep = 0u - ((ok >> J) & 1u);
      if (GN) {
        const float onf = __uint_as_float(keep & 0x3f800000u);  // 1.0f or 0.0f
        float f[EPQ];
        unpack<T>(r[J], f);
#pragma unroll
        for (int e = 0; e < EPQ; ++e) f[e] = silu(f[e] * sc[e] + sh[e]) * onf;
        r[J] = pack<T>(f);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) r[J][k] &= keep;
      }
    }
  }

  // in-place GroupNorm+SiLU (and zeroing of out-of-volume items) of the
  // fetched registers, segment A, MODE 0/1
  __device__ __forceinline__ void transform() {
    transform_item<0>(); transform_item<1>(); transform_item<2>(); transform_item<3>();
    transform_item<4>(); transform_item<5>(); transform_item<6>(); transform_item<7>();
    transform_item<8>(); transform_item<9>(); transform_item<10>(); transform_item<11>();
    transform_item<12>(); transform_item<13>(); transform_item<14>(); transform_item<15>();
    static_assert(NI <= 16, "transform unroll");
  }

  // write already-transformed registers; SWZ selects the XOR-swizzled image
  template <bool SWZ>
  __device__ __forceinline__ void write(unsigned char* lds, int tid) const {
    const int q = tid & 1;
    const bool interior = !seg_a;
    const int n = interior ? BX * BY * BZ : HV;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int it = (tid >> 1) + 128 * j;
      if (it < n) {
        int hv, hx, hy, hz;
        coords(it, interior, &hv, &hx, &hy, &hz);
        const int off = SWZ ? hv * 32 + ((q ^ ((hv >> 3) & 1)) << 4) : hv * 32 + (q << 4);
        *reinterpret_cast<u32x4*>(lds + off) = r[j];
      }
    }
  }

  template <bool SWZ>
  __device__ __forceinline__ void store(unsigned char* lds, const ConvParams& p, int b, int x0, int y0, int z0,
                                        int tid) const {
    const int q = tid & 1;
    const bool interior = !seg_a;
    const int n = interior ? BX * BY * BZ : HV;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int it = (tid >> 1) + 128 * j;
      if (it < n) {
        int hv, hx, hy, hz;
        coords(it, interior, &hv, &hx, &hy, &hz);
        float f[EPQ];
        if (MODE == 2 && seg_a) {
#pragma unroll
          for (int e = 0; e < EPQ; ++e) f[e] = 0.f;
          const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
          if (ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) {
            const int SD = p.D << 1, SH = p.H << 1, SW = p.W << 1;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const long long vox = (((long long)b * SD + 2 * oz + (k >> 2)) * SH + 2 * oy + ((k >> 1) & 1)) * SW +
                                    2 * ox + (k & 1);
              float g[EPQ];
              unpack<T>(ldg16(base + vox * csrc), g);
#pragma unroll
              for (int e = 0; e < EPQ; ++e) f[e] += GN ? silu(g[e] * sc[e] + sh[e]) : g[e];
            }
#pragma unroll
            for (int e = 0; e < EPQ; ++e) f[e] *= 0.125f;
          }
        } else {
          unpack<T>(r[j], f);
          if (!((ok >> j) & 1)) {
#pragma unroll
            for (int e = 0; e < EPQ; ++e) f[e] = 0.f;  // out-of-volume (zero padding)
          } else if (GN && seg_a) {
#pragma unroll
            for (int e = 0; e < EPQ; ++e) f[e] = silu(f[e] * sc[e] + sh[e]);
          }
        }
        const int off = SWZ ? hv * 32 + ((q ^ ((hv >> 3) & 1)) << 4) : hv * 32 + (q << 4);
        *reinterpret_cast<u32x4*>(lds + off) = pack<T>(f);
      }
    }
  }
};

// weights of one chunk: a contiguous block of the packed layout copied
// global -> LDS with LDS-DMA (no VGPRs; each wave instruction moves 1 KB).
__device__ __forceinline__ void stage_weights(unsigned char* wl, const unsigned char* g, int bytes, int tid) {
  const int wv = tid >> 6, lane = tid & 63;
  for (int off = wv * 1024; off < bytes; off += 4096) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + off + lane * 16),
                                     (__attribute__((address_space(3))) void*)(wl + off), 16, 0, 0);
  }
}

// Epilogue on one output tile held in LDS as fp32 E[ROWS][NT+4]: bias,
// residual, store, GroupNorm partial statistics.
template <typename T, int BX, int BY, int BZ, int NF, int ROWS>
__device__ __forceinline__ void epilogue_rows(const ConvParams& p, float* E, int b, int st, int ct, int x0, int y0,
                                              int z0, int tid) {
  constexpr int NT = 32 * NF, LD = NT + 4;
  static_assert(ROWS == BX * BY * BZ, "rows");
  constexpr int CG = NT / 8;  // 8-channel groups per row
  const int cg = tid % CG;
  const int cbase = ct * NT + cg * 8;
  const int nvalid = min(8, p.cout - cbase);
  float bsum[8], bsq[8], bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bsum[e] = 0.f;
    bsq[e] = 0.f;
    bias[e] = (e < nvalid && p.bias) ? p.bias[(long long)b * p.bias_bs + cbase + e] : 0.f;
  }
  // residuals of every row this thread owns are loaded first, so their HBM
  // latency overlaps (same-grid / upsampled residual, full 8-channel groups)
  constexpr int IT = ROWS * CG / 256;
  constexpr int RQ = sizeof(T) == 2 ? 1 : 2;
  const bool rfast = (p.rmode == 0 || p.rmode == 1) && nvalid == 8;
  u32x4 rr[IT][RQ];
  if (rfast) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int row = (tid + 256 * k) / CG;
      const int rx = row % BX, ry = (row / BX) % BY, rz = row / (BX * BY);
      const int ox = x0 + rx, oy = y0 + ry, oz = z0 + rz;
#pragma unroll
      for (int q = 0; q < RQ; ++q) rr[k][q] = u32x4{0u, 0u, 0u, 0u};
      if (ox < p.W && oy < p.H && oz < p.D) {
        long long rvx = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
        if (p.rmode == 1)
          rvx = (((long long)b * (p.D >> 1) + (oz >> 1)) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1);
        const T* r = reinterpret_cast<const T*>(p.res) + rvx * p.cout + cbase;
#pragma unroll
        for (int q = 0; q < RQ; ++q) rr[k][q] = ldg16(r + q * (16 / sizeof(T)));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int u = tid + 256 * k;
    const int row = u / CG;
    const int rx = row % BX, ry = (row / BX) % BY, rz = row / (BX * BY);
    const int ox = x0 + rx, oy = y0 + ry, oz = z0 + rz;
    if (ox >= p.W || oy >= p.H || oz >= p.D || nvalid <= 0) continue;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = E[row * LD + cg * 8 + e] + bias[e];
    const long long vox = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
    if (rfast) {
      float rv[8];
#pragma unroll
      for (int q = 0; q < RQ; ++q) unpack<T>(rr[k][q], rv + q * (8 / RQ));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rv[e] + v[e];
    } else if (p.rmode >= 0) {
      const T* r = reinterpret_cast<const T*>(p.res);
      float rv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) rv[e] = 0.f;
      if (p.rmode == 2) {
        const int RD = p.D * 2, RH = p.H * 2, RW = p.W * 2;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const long long rvx = (((long long)b * RD + 2 * oz + (kk >> 2)) * RH + 2 * oy + ((kk >> 1) & 1)) * RW +
                                2 * ox + (kk & 1);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e < nvalid) rv[e] += Elem<T>::to_f(r[rvx * p.cout + cbase + e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) rv[e] *= 0.125f;
      } else {
        long long rvx = vox;
        if (p.rmode == 1)
          rvx = (((long long)b * (p.D >> 1) + (oz >> 1)) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nvalid) rv[e] = Elem<T>::to_f(r[rvx * p.cout + cbase + e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rv[e] + v[e];
    }
    // output tensor / channel stride (dual output splits the channels at out_c0)
    void* obase = p.out;
    int ostride = p.cout, oc = cbase;
    if (p.out1 && cbase >= p.out_c0) {
      obase = p.out1;
      ostride = p.cout - p.out_c0;
      oc = cbase - p.out_c0;
    } else if (p.out1) {
      ostride = p.out_c0;
    }
    if (p.out_f32) {
      float* o = reinterpret_cast<float*>(obase) + vox * ostride + oc;
      if (p.accumulate) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nvalid) v[e] += o[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < nvalid) o[e] = v[e];
    } else {
      T* o = reinterpret_cast<T*>(obase) + vox * ostride + oc;
      if (p.accumulate) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nvalid) v[e] += Elem<T>::to_f(o[e]);
      }
      if (nvalid == 8) {
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<u32x4*>(o) = pack<T>(v);
        } else {
          *reinterpret_cast<u32x4*>(o) = pack<float>(v);
          *reinterpret_cast<u32x4*>(o + 4) = pack<float>(v + 4);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nvalid) o[e] = Elem<T>::from_f(v[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsum[e] += v[e];
      bsq[e] += v[e] * v[e];
    }
  }
  if (p.stats) {
    __syncthreads();
    float* R = E;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      R[tid * 16 + e] = bsum[e];
      R[tid * 16 + 8 + e] = bsq[e];
    }
    __syncthreads();
    if (tid < NT) {
      const int g = tid / 8, e = tid % 8;
      const int c = ct * NT + tid;
      float s = 0.f, q = 0.f;
      for (int t = g; t < 256; t += CG) {
        s += R[t * 16 + e];
        q += R[t * 16 + 8 + e];
      }
      if (c < p.cout) {
        const long long parts = (long long)p.tx * p.ty * p.tz;
        const long long pidx = ((long long)b * parts + (st % (p.tx * p.ty * p.tz))) * p.cout + c;
        p.stats[pidx * 2 + 0] = s;
        p.stats[pidx * 2 + 1] = q;
      }
    }
  }
}

// split-K: raw fp32 partial tile -> workspace [ks][vox][cout]
template <typename T, int BX, int BY, int BZ, int NF, int ROWS>
__device__ __forceinline__ void write_partial(const ConvParams& p, const float* E, int ks, int b, int ct, int x0,
                                              int y0, int z0, int tid) {
  constexpr int NT = 32 * NF, LD = NT + 4, CG = NT / 8;
  const long long nvox = (long long)p.B * p.D * p.H * p.W;
  float* part = p.partial + (long long)ks * nvox * p.cout;
  const int cg = tid % CG;
  const int cbase = ct * NT + cg * 8;
  const int nvalid = min(8, p.cout - cbase);
  for (int u = tid; u < ROWS * CG; u += 256) {
    const int row = u / CG;
    const int rx = row % BX, ry = (row / BX) % BY, rz = row / (BX * BY);
    const int ox = x0 + rx, oy = y0 + ry, oz = z0 + rz;
    if (ox >= p.W || oy >= p.H || oz >= p.D || nvalid <= 0) continue;
    const long long vox = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
    float* o = part + vox * p.cout + cbase;
    if (nvalid == 8) {
      *reinterpret_cast<float4*>(o) = *reinterpret_cast<const float4*>(E + row * LD + cg * 8);
      *reinterpret_cast<float4*>(o + 4) = *reinterpret_cast<const float4*>(E + row * LD + cg * 8 + 4);
    } else {
      for (int e = 0; e < nvalid; ++e) o[e] = E[row * LD + cg * 8 + e];
    }
  }
}

// sum the S fp32 slices of one (spatial tile, channel tile) into the epilogue
// staging E[row][LD] in slice order 0..S-1 (deterministic whoever finishes it)
template <int BX, int BY, int BZ, int NF, int ROWS>
__device__ __forceinline__ void sum_slices(const ConvParams& p, float* E, int S, int b, int ct, int x0, int y0, int z0,
                                           int tid) {
  constexpr int NT = 32 * NF, LD = NT + 4, CG = NT / 8;
  const int cg = tid % CG;
  const int cbase = ct * NT + cg * 8;
  const int nvalid = min(8, p.cout - cbase);
  const long long slice = (long long)p.B * p.D * p.H * p.W * p.cout;
  for (int u = tid; u < ROWS * CG; u += 256) {
    const int row = u / CG;
    const int rx = row % BX, ry = (row / BX) % BY, rz = row / (BX * BY);
    const int ox = x0 + rx, oy = y0 + ry, oz = z0 + rz;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    if (!(ox >= p.W || oy >= p.H || oz >= p.D || nvalid <= 0)) {
      const long long vox = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
      for (int k = 0; k < S; ++k) {
        const float* src = p.partial + k * slice + vox * p.cout + cbase;
        if (nvalid == 8) {
          const float4 a = *reinterpret_cast<const float4*>(src), c = *reinterpret_cast<const float4*>(src + 4);
          v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
          v[4] += c.x; v[5] += c.y; v[6] += c.z; v[7] += c.w;
        } else {
          for (int e = 0; e < nvalid; ++e) v[e] += src[e];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) E[row * LD + cg * 8 + e] = v[e];
  }
}

template <typename T, int BX, int BY, int BZ>
__device__ __forceinline__ void tile_origin(const ConvParams& p, int st, int* b, int* x0, int* y0, int* z0) {
  const int ix = st % p.tx, iy = (st / p.tx) % p.ty, iz = (st / (p.tx * p.ty)) % p.tz;
  *b = st / (p.tx * p.ty * p.tz);
  *x0 = ix * BX;
  *y0 = iy * BY;
  *z0 = iz * BZ;
}

template <typename T, int BX, int BY, int BZ, int NF, int MODE, bool GN>
__global__ void __launch_bounds__(256) conv3d_kernel(ConvParams p) {
  using Cfg = ConvCfg<T, BX, BY, BZ, NF>;
  constexpr int CK = ConvTr<T>::CK;
  constexpr int HX = Cfg::HX, HY = Cfg::HY, NT = Cfg::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[Cfg::SMEM];
  unsigned char* halo = smem;
  unsigned char* wl = smem + Cfg::HALO_B;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 31, hh = lane >> 5;
  const int S = p.ksplit;
  const int ks = blockIdx.x % S;
  const int rest = blockIdx.x / S;
  const int ct = rest % p.nct;
  const int st = rest / p.nct;
  int b, x0, y0, z0;
  tile_origin<T, BX, BY, BZ>(p, st, &b, &x0, &y0, &z0);

  int hbase[2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf) {
    const int r = wv * 64 + mf * 32 + lr;
    const int rx = r % BX, ry = (r / BX) % BY, rz = r / (BX * BY);
    hbase[mf] = ((rz + 1) * HY + (ry + 1)) * HX + (rx + 1);
  }

  f32x16 acc[2][NF];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

  const int nA = (p.ac0 + p.ac1) / CK;
  const int nB = p.bw ? (p.bc0 + p.bc1) / CK : 0;
  const int total = nA + nB;
  const int per = (total + S - 1) / S;
  const int g0 = ks * per, g1 = min(total, g0 + per);

  auto wsrc = [&](int gc, int* bytes) {
    const bool segA = gc < nA;
    const int chunk = segA ? gc : gc - nA;
    const int ntaps = segA ? 27 : 1;
    const int nch = segA ? nA : nB;
    *bytes = ntaps * NT * 32;
    return reinterpret_cast<const unsigned char*>(segA ? p.aw : p.bw) +
           ((long long)ct * nch + chunk) * (long long)(ntaps * NT * 32);
  };

  Stager<T, BX, BY, BZ, MODE, GN> sg;
  if (g0 < g1) {
    sg.fetch(p, g0 < nA, g0 < nA ? g0 : g0 - nA, b, x0, y0, z0, tid);
    int wb;
    const unsigned char* wsp = wsrc(g0, &wb);
    stage_weights(wl, wsp, wb, tid);
    sg.template store<true>(halo, p, b, x0, y0, z0, tid);
    __syncthreads();
  }
  for (int gc = g0; gc < g1; ++gc) {
    const bool segA = gc < nA;
    const int ntaps = segA ? 27 : 1;
    const bool has_next = gc + 1 < g1;
    if (has_next) sg.fetch(p, gc + 1 < nA, gc + 1 < nA ? gc + 1 : gc + 1 - nA, b, x0, y0, z0, tid);
    for (int tap = 0; tap < ntaps; ++tap) {
      int toff = 0;
      if (segA) {
        const int dz = tap / 9 - 1, dy = (tap / 3) % 3 - 1, dx = tap % 3 - 1;
        toff = (dz * HY + dy) * HX + dx;
      }
      u32x4 bq[NF], aq[2];
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const int row = n * 32 + lr;
        bq[n] = *reinterpret_cast<const u32x4*>(wl + (tap * NT + row) * 32 + ((hh ^ ((row >> 3) & 1)) << 4));
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int v = hbase[m] + toff;
        aq[m] = *reinterpret_cast<const u32x4*>(halo + v * 32 + ((hh ^ ((v >> 3) & 1)) << 4));
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < NF; ++n) mfma_acc(acc[m][n], aq[m], bq[n], (T*)nullptr);
    }
    if (!has_next) break;
    __syncthreads();  // every wave is done reading this chunk's halo and weights
    int wb;
    const unsigned char* wsp = wsrc(gc + 1, &wb);
    stage_weights(wl, wsp, wb, tid);
    sg.template store<true>(halo, p, b, x0, y0, z0, tid);
    __syncthreads();
  }

  __syncthreads();
  float* E = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = wv * 64 + m * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
        E[row * Cfg::EPI_LD + n * 32 + lr] = acc[m][n][i];
      }
  __syncthreads();
  if (S == 1) {
    epilogue_rows<T, BX, BY, BZ, NF, 256>(p, E, b, st, ct, x0, y0, z0, tid);
    return;
  }
  write_partial<T, BX, BY, BZ, NF, 256>(p, E, ks, b, ct, x0, y0, z0, tid);
}

// split-K, stage 1: partial[0] += partial[1..S-1], elementwise over the whole
// output (bandwidth-bound, every CU busy; the per-tile finish below has only
// one workgroup per tile) ...
template <int Dummy = 0>
__global__ void __launch_bounds__(256) splitk_sum_kernel(float* __restrict__ part, int S, long long n4) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4* p4 = reinterpret_cast<float4*>(part);
  float4 a = p4[i];
  for (int k = 1; k < S; ++k) {
    const float4 b = p4[i + k * n4];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  p4[i] = a;
}

// ... stage 2 (S = 1), or the whole finish for small S: sum the S partial slices of a tile and run the epilogue on it,
// one workgroup per (spatial tile, channel tile)
template <typename T, int BX, int BY, int BZ, int NF>
__global__ void __launch_bounds__(256) conv3d_reduce_kernel(ConvParams p, int S) {
  constexpr int ROWS = BX * BY * BZ, NT = 32 * NF, LD = NT + 4, CG = NT / 8;
  __shared__ __attribute__((aligned(16))) float E[ROWS * LD > 256 * 16 ? ROWS * LD : 256 * 16];
  const int tid = threadIdx.x;
  const int ct = blockIdx.x % p.nct;
  const int st = blockIdx.x / p.nct;
  int b, x0, y0, z0;
  tile_origin<T, BX, BY, BZ>(p, st, &b, &x0, &y0, &z0);
  const int cg = tid % CG;
  const int cbase = ct * NT + cg * 8;
  if (S == 1 && ct * NT + NT <= p.cout) {  // workgroup-uniform: the whole channel tile is valid
    // pre-summed slice: every row's loads in flight at once (fully unrolled)
    constexpr int IT = ROWS * CG / 256;
    static_assert(ROWS * CG % 256 == 0, "rows per thread");
    float4 va[IT], vb[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int row = (tid + 256 * k) / CG;
      const int rx = row % BX, ry = (row / BX) % BY, rz = row / (BX * BY);
      const int ox = min(x0 + rx, p.W - 1), oy = min(y0 + ry, p.H - 1), oz = min(z0 + rz, p.D - 1);
      const float* src = p.partial + ((((long long)b * p.D + oz) * p.H + oy) * p.W + ox) * p.cout + cbase;
      va[k] = *reinterpret_cast<const float4*>(src);
      vb[k] = *reinterpret_cast<const float4*>(src + 4);
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int row = (tid + 256 * k) / CG;
      float* e = E + row * LD + cg * 8;
      *reinterpret_cast<float4*>(e) = va[k];
      *reinterpret_cast<float4*>(e + 4) = vb[k];
    }
    __syncthreads();
    epilogue_rows<T, BX, BY, BZ, NF, ROWS>(p, E, b, st, ct, x0, y0, z0, tid);
    return;
  }
  sum_slices<BX, BY, BZ, NF, ROWS>(p, E, S, b, ct, x0, y0, z0, tid);
  __syncthreads();
  epilogue_rows<T, BX, BY, BZ, NF, ROWS>(p, E, b, st, ct, x0, y0, z0, tid);
}

// ===========================================================================
// Wide-grid kernel (output W >= 32): brick 32(x) x 4(y) x 4(z) = 512 rows,
// wave w owns z-plane w = four 32-voxel x-lines = four 32-row A fragments.
// For a fixed (dz, dx) the three dy taps read input lines y-1 .. y+4, so each
// wave loads 6 A fragments and reuses them across the 3 dy taps (12 MFMA uses):
// half the LDS reads of one-tap-at-a-time.  The halo image is linear (no
// swizzle) so every (dz, line, dx) offset is an immediate; lanes of a read
// group touch 16 consecutive voxels (2-way bank conflict, LDS stays < 40%
// busy).  Weights are double-buffered and filled by LDS-DMA one chunk ahead;
// the next chunk's halo is fetched into registers at the top of the chunk and
// transformed (GN+SiLU) after the first dz slab, so HBM latency and the
// prologue VALU both hide under the MFMAs.  One 4-wave workgroup per CU.
// ===========================================================================
template <typename T, int NF>
struct WideCfg {
  static constexpr int BX = 32, BY = 4, BZ = 4, HX = 34, HY = 6, HZ = 6, HV = HX * HY * HZ;
  static constexpr int NT = 32 * NF;
  static constexpr int HALO_B = HV * 32;
  static constexpr int WB = 27 * NT * 32;
  static constexpr int EPI_LD = NT + 4;
  static constexpr int EPI_B = 512 * EPI_LD * 4;
  static constexpr int MAIN_B = HALO_B + 2 * WB;
  static constexpr int SMEM = MAIN_B > EPI_B ? MAIN_B : EPI_B;
};

template <int G, int NI, typename SG>
__device__ __forceinline__ void transform_group(SG* sg) {
  // items of the next chunk assigned to (dz, dx) groups 3..8 (the dz = 0, +1
  // slabs), spread evenly: the loads issued at the top of the chunk get the
  // whole first slab (~2300 MFMA cycles) to land before the first transform
  constexpr int GG = G < 3 ? -1 : G - 3;
  constexpr int j0 = GG < 0 ? 0 : (GG * NI) / 6, j1 = GG < 0 ? 0 : ((GG + 1) * NI) / 6;
  if constexpr (j0 < j1) sg->template transform_item<j0>();
  if constexpr (j0 + 1 < j1) sg->template transform_item<j0 + 1>();
  if constexpr (j0 + 2 < j1) sg->template transform_item<j0 + 2>();
}

template <typename T, int NF, int DZ, int DX, typename SG>
__device__ __forceinline__ void wide_group(f32x16 (&acc)[4][NF], const unsigned char* halo_lane,
                                           const unsigned char* w_lane, SG* sg, bool xform) {
  using C = WideCfg<T, NF>;
  constexpr int dx = DX;
  {
    u32x4 a[6];
#pragma unroll
    for (int L = 0; L < 6; ++L)
      a[L] = *reinterpret_cast<const u32x4*>(halo_lane + ((DZ * C::HY + (L - 1)) * C::HX + dx) * 32);
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int tap = ((DZ + 1) * 3 + (dy + 1)) * 3 + (dx + 1);
      u32x4 bq[NF];
#pragma unroll
      for (int n = 0; n < NF; ++n)
        bq[n] = *reinterpret_cast<const u32x4*>(w_lane + (tap * C::NT + n * 32) * 32);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < NF; ++n) mfma_acc(acc[m][n], a[m + dy + 1], bq[n], (T*)nullptr);
    }
  }
  if (xform) transform_group<(DZ + 1) * 3 + (DX + 1), SG::NI>(sg);
}

template <typename T, int NF, int DZ, typename SG>
__device__ __forceinline__ void wide_slab_x(f32x16 (&acc)[4][NF], const unsigned char* halo_lane,
                                            const unsigned char* w_lane, SG* sg, bool xform) {
  wide_group<T, NF, DZ, -1>(acc, halo_lane, w_lane, sg, xform);
  wide_group<T, NF, DZ, 0>(acc, halo_lane, w_lane, sg, xform);
  wide_group<T, NF, DZ, 1>(acc, halo_lane, w_lane, sg, xform);
}

template <typename T, int NF, int DZ>
__device__ __forceinline__ void wide_slab(f32x16 (&acc)[4][NF], const unsigned char* halo_lane,
                                          const unsigned char* w_lane) {
  using C = WideCfg<T, NF>;
#pragma unroll
  for (int dx = -1; dx <= 1; ++dx) {
    u32x4 a[6];
#pragma unroll
    for (int L = 0; L < 6; ++L)
      a[L] = *reinterpret_cast<const u32x4*>(halo_lane + ((DZ * C::HY + (L - 1)) * C::HX + dx) * 32);
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      constexpr int dummy = 0;
      (void)dummy;
      const int tap = ((DZ + 1) * 3 + (dy + 1)) * 3 + (dx + 1);
      u32x4 bq[NF];
#pragma unroll
      for (int n = 0; n < NF; ++n)
        bq[n] = *reinterpret_cast<const u32x4*>(w_lane + (tap * C::NT + n * 32) * 32);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < NF; ++n) mfma_acc(acc[m][n], a[m + dy + 1], bq[n], (T*)nullptr);
    }
  }
}

template <typename T, int NF, int MODE, bool GN>
__global__ void __launch_bounds__(256) conv3d_wide_kernel(ConvParams p) {
  using C = WideCfg<T, NF>;
  constexpr int CK = ConvTr<T>::CK, NT = C::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::SMEM];
  unsigned char* halo = smem;
  unsigned char* wbuf0 = smem + C::HALO_B;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 31, hh = lane >> 5;
  const int S = p.ksplit;
  const int ks = blockIdx.x % S;
  const int rest = blockIdx.x / S;
  const int ct = rest % p.nct;
  const int st = rest / p.nct;
  int b, x0, y0, z0;
  tile_origin<T, C::BX, C::BY, C::BZ>(p, st, &b, &x0, &y0, &z0);

  // lane bases: A at (z = wv, line 0, x = lr), centre tap; B at row lr
  const unsigned char* halo_lane = halo + (((wv + 1) * C::HY + 1) * C::HX + lr + 1) * 32 + hh * 16;
  const int w_lane_off = lr * 32 + ((hh ^ ((lr >> 3) & 1)) << 4);

  f32x16 acc[4][NF];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

  const int nA = (p.ac0 + p.ac1) / CK;
  const int nB = p.bw ? (p.bc0 + p.bc1) / CK : 0;
  const int total = nA + nB;
  const int per = (total + S - 1) / S;
  const int g0 = ks * per, g1 = min(total, g0 + per);

  auto wsrc = [&](int gc, int* bytes) {
    const bool segA = gc < nA;
    const int chunk = segA ? gc : gc - nA;
    const int ntaps = segA ? 27 : 1;
    const int nch = segA ? nA : nB;
    *bytes = ntaps * NT * 32;
    return reinterpret_cast<const unsigned char*>(segA ? p.aw : p.bw) +
           ((long long)ct * nch + chunk) * (long long)(ntaps * NT * 32);
  };

  Stager<T, C::BX, C::BY, C::BZ, MODE, GN> sg;
  if (g0 < g1) {
    int wb;
    const unsigned char* wsp = wsrc(g0, &wb);
    stage_weights(wbuf0, wsp, wb, tid);
    sg.fetch(p, g0 < nA, g0 < nA ? g0 : g0 - nA, b, x0, y0, z0, tid);
    if constexpr (MODE == 2) {
      sg.template store<false>(halo, p, b, x0, y0, z0, tid);
    } else {
      sg.transform();
      sg.template write<false>(halo, tid);
    }
    __syncthreads();
  }
  // staging of chunk gc+1 (LDS-DMA weights + halo registers) overlaps chunk gc's MFMAs
  auto prefetch = [&](int gn) {
    int wb;
    const unsigned char* wsp = wsrc(gn, &wb);
    stage_weights(wbuf0 + ((gn - g0) & 1) * C::WB, wsp, wb, tid);
    sg.fetch(p, gn < nA, gn < nA ? gn : gn - nA, b, x0, y0, z0, tid);
  };
  auto commit = [&](bool has_next) {
    __syncthreads();  // all waves done with this chunk's halo and weights
    if (has_next) {
      if constexpr (MODE == 2) sg.template store<false>(halo, p, b, x0, y0, z0, tid);
      else sg.template write<false>(halo, tid);
    }
    __syncthreads();  // (drains the LDS-DMA of the next weights as well)
  };
  // 3x3x3 segment: straight-line body, acc stays in the accumulator registers
  const int gA1 = min(g1, nA);
  for (int gc = g0; gc < gA1; ++gc) {
    const bool has_next = gc + 1 < g1;
    if (has_next) prefetch(gc + 1);
    const unsigned char* w_lane = wbuf0 + ((gc - g0) & 1) * C::WB + w_lane_off;
    // the next chunk's GN+SiLU runs between the MFMA groups (VALU issues in the
    // MFMA gaps of the same wave)
    wide_slab_x<T, NF, -1>(acc, halo_lane, w_lane, &sg, has_next);
    wide_slab_x<T, NF, 0>(acc, halo_lane, w_lane, &sg, has_next);
    wide_slab_x<T, NF, 1>(acc, halo_lane, w_lane, &sg, has_next);
    commit(has_next);
  }
  // 1x1 segment (skip_connection): centre tap only, weights = tap 0 of the chunk
  for (int gc = max(g0, nA); gc < g1; ++gc) {
    const bool has_next = gc + 1 < g1;
    if (has_next) prefetch(gc + 1);
    const unsigned char* w_lane = wbuf0 + ((gc - g0) & 1) * C::WB + w_lane_off;
    u32x4 a[4], bq[NF];
#pragma unroll
    for (int L = 0; L < 4; ++L) a[L] = *reinterpret_cast<const u32x4*>(halo_lane + (L * C::HX) * 32);
#pragma unroll
    for (int n = 0; n < NF; ++n) bq[n] = *reinterpret_cast<const u32x4*>(w_lane + (n * 32) * 32);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n) mfma_acc(acc[m][n], a[m], bq[n], (T*)nullptr);
    commit(has_next);
  }

  __syncthreads();
  float* E = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = wv * 128 + m * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
        E[row * C::EPI_LD + n * 32 + lr] = acc[m][n][i];
      }
  __syncthreads();
  if (S == 1) {
    epilogue_rows<T, C::BX, C::BY, C::BZ, NF, 512>(p, E, b, st, ct, x0, y0, z0, tid);
    return;
  }
  write_partial<T, C::BX, C::BY, C::BZ, NF, 512>(p, E, ks, b, ct, x0, y0, z0, tid);
}

inline int pick_nf(int cout) { return (cout % 64 == 0) ? 2 : 1; }

struct Brick { int bx, by, bz; };
// Grids from kWideMinW up take the 32-wide x tiles of the DMA conv (conv3d_v4.hpp,
// the last x tile masked) and its statistics bricks; below, the small-grid
// kernel's 16x4x4 / 8x8x4 bricks (conv3d_sg.hip).  24: config 5's 28^3 level ran
// on the small-grid kernel at 0.28 PF (per 32-channel chunk ~8.3k cycles of
// LDS-DMA for 1.7k of MFMA, tools/sg_stamps.py); on the DMA kernel with 32-channel
// tiles it computes 12.5 % masked voxels but stays MFMA-bound.
constexpr int kWideMinW = 24;
inline Brick pick_brick(int64_t D, int64_t H, int64_t W) {
  (void)D; (void)H;
  if (W >= kWideMinW) return {32, 4, 4};  // conv3d_wide_kernel / conv3d_v4_kernel
  if (W >= 16) return {16, 4, 4};
  return {8, 8, 4};
}

// algorithmic flops of one conv launch: 2 x output voxels x cout x K
inline double conv_flops(const ConvParams& p) {
  const double K = 27.0 * (p.ac0 + p.ac1) + (p.bw ? (double)(p.bc0 + p.bc1) : 0.0);
  return 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * K;
}

template <typename T, int BX, int BY, int BZ, int NF>
int launch_conv(const ConvParams& p, hipStream_t s) {
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz * p.nct;
  CWDM_REQUIRE(nblk * p.ksplit < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d: grid too large");
  const dim3 grid((unsigned)(nblk * p.ksplit));
  const bool gn = p.agn != nullptr;
  prof_begin(s);
  if (p.amode == 0) {
    if (gn) hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF, 0, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF, 0, false>), grid, dim3(256), 0, s, p);
  } else if (p.amode == 1) {
    if (gn) hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF, 1, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF, 1, false>), grid, dim3(256), 0, s, p);
  } else {
    if (gn) hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF, 2, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF, 2, false>), grid, dim3(256), 0, s, p);
  }
  prof_end(s, conv_flops(p));
  CWDM_LAUNCHED();
  if (p.ksplit > 1) {
    const long long n4 = (long long)p.B * p.D * p.H * p.W * p.cout / 4;
    hipLaunchKernelGGL(splitk_sum_kernel<0>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, s, p.partial, p.ksplit, n4);
    CWDM_LAUNCHED();
    ConvParams q = p;
    q.ksplit = 1;
    hipLaunchKernelGGL((conv3d_reduce_kernel<T, BX, BY, BZ, NF>), dim3((unsigned)nblk), dim3(256), 0, s, q, 1);
    CWDM_LAUNCHED();
  }
  return CWDM_OK;
}

template <typename T, int NF>
int launch_wide(const ConvParams& p, hipStream_t s) {
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz * p.nct;
  CWDM_REQUIRE(nblk * p.ksplit < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d: grid too large");
  const dim3 grid((unsigned)(nblk * p.ksplit));
  const bool gn = p.agn != nullptr;
  prof_begin(s);
  if (p.amode == 0) {
    if (gn) hipLaunchKernelGGL((conv3d_wide_kernel<T, NF, 0, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_wide_kernel<T, NF, 0, false>), grid, dim3(256), 0, s, p);
  } else if (p.amode == 1) {
    if (gn) hipLaunchKernelGGL((conv3d_wide_kernel<T, NF, 1, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_wide_kernel<T, NF, 1, false>), grid, dim3(256), 0, s, p);
  } else {
    if (gn) hipLaunchKernelGGL((conv3d_wide_kernel<T, NF, 2, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_wide_kernel<T, NF, 2, false>), grid, dim3(256), 0, s, p);
  }
  prof_end(s, conv_flops(p));
  CWDM_LAUNCHED();
  if (p.ksplit > 1) {
    const long long n4 = (long long)p.B * p.D * p.H * p.W * p.cout / 4;
    hipLaunchKernelGGL(splitk_sum_kernel<0>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, s, p.partial, p.ksplit, n4);
    CWDM_LAUNCHED();
    ConvParams q = p;
    q.ksplit = 1;
    hipLaunchKernelGGL((conv3d_reduce_kernel<T, 32, 4, 4, NF>), dim3((unsigned)nblk), dim3(256), 0, s, q, 1);
    CWDM_LAUNCHED();
  }
  return CWDM_OK;
}

}  // namespace cwdm
