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
// bf16 uses v_mfma_f32_32x32x16_bf16; fp32 (parity mode) uses exact-f32
// v_mfma_f32_32x32x2_f32.  Accumulation is fp32 in both.
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
};

template <typename T> struct ConvTr;
template <> struct ConvTr<bf16_t> { static constexpr int CK = 16; static constexpr int EPQ = 8; };
template <> struct ConvTr<float> { static constexpr int CK = 8; static constexpr int EPQ = 4; };

__device__ __forceinline__ float silu(float v) { return v / (1.0f + __expf(-v)); }

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
  for (int i = 0; i < 4; ++i) q[i] = (unsigned)f2bf(f[2 * i]) | ((unsigned)f2bf(f[2 * i + 1]) << 16);
  return q;
}
template <>
__device__ __forceinline__ u32x4 pack<float>(const float* f) {
  u32x4 q;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = __float_as_uint(f[i]);
  return q;
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

// Stage one chunk of the halo (conv input) into LDS.
template <typename T, int BX, int BY, int BZ>
__device__ __forceinline__ void stage_halo(unsigned char* lds, const void* s0, int c0, const void* s1, int c1,
                                           int mode, const float* gn, int ctot, int chunk, int b, int x0, int y0,
                                           int z0, int D, int H, int W, int tid) {
  constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ;
  constexpr int HX = BX + 2, HY = BY + 2, HV = HX * HY * (BZ + 2);
  const int q = tid & 1;
  const int cb = chunk * CK + q * EPQ;  // first concat channel of this thread's quad
  const void* src;
  int ch, csrc;
  if (cb < c0) { src = s0; ch = cb; csrc = c0; }
  else { src = s1; ch = cb - c0; csrc = c1; }
  float sc[EPQ], sh[EPQ];
  if (gn) {
#pragma unroll
    for (int e = 0; e < EPQ; ++e) {
      sc[e] = gn[((long long)b * ctot + cb + e) * 2 + 0];
      sh[e] = gn[((long long)b * ctot + cb + e) * 2 + 1];
    }
  }
  // source grid dims
  int SD = D, SH = H, SW = W;
  if (mode == 1) { SD = D >> 1; SH = H >> 1; SW = W >> 1; }
  else if (mode == 2) { SD = D << 1; SH = H << 1; SW = W << 1; }
  const T* base = reinterpret_cast<const T*>(src) + ch;
  for (int hv = tid >> 1; hv < HV; hv += 128) {
    const int hx = hv % HX, hy = (hv / HX) % HY, hz = hv / (HX * HY);
    const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
    float f[EPQ];
    if (ox < 0 || oy < 0 || oz < 0 || ox >= W || oy >= H || oz >= D) {
#pragma unroll
      for (int e = 0; e < EPQ; ++e) f[e] = 0.f;
    } else if (mode == 2) {
#pragma unroll
      for (int e = 0; e < EPQ; ++e) f[e] = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int sz = 2 * oz + (k >> 2), sy = 2 * oy + ((k >> 1) & 1), sx = 2 * ox + (k & 1);
        const long long vox = (((long long)b * SD + sz) * SH + sy) * SW + sx;
        float g[EPQ];
        unpack<T>(ldg16(base + vox * csrc), g);
#pragma unroll
        for (int e = 0; e < EPQ; ++e) {
          float v = g[e];
          if (gn) v = silu(v * sc[e] + sh[e]);
          f[e] += v;
        }
      }
#pragma unroll
      for (int e = 0; e < EPQ; ++e) f[e] *= 0.125f;
    } else {
      int sx = ox, sy = oy, sz = oz;
      if (mode == 1) { sx >>= 1; sy >>= 1; sz >>= 1; }
      const long long vox = (((long long)b * SD + sz) * SH + sy) * SW + sx;
      unpack<T>(ldg16(base + vox * csrc), f);
      if (gn) {
#pragma unroll
        for (int e = 0; e < EPQ; ++e) f[e] = silu(f[e] * sc[e] + sh[e]);
      }
    }
    const int off = hv * 32 + ((q ^ ((hv >> 3) & 1)) << 4);
    *reinterpret_cast<u32x4*>(lds + off) = pack<T>(f);
  }
}

template <typename T, int BX, int BY, int BZ, int NF>
__global__ void __launch_bounds__(256) conv3d_kernel(ConvParams p) {
  using Cfg = ConvCfg<T, BX, BY, BZ, NF>;
  constexpr int CK = ConvTr<T>::CK;
  constexpr int HX = Cfg::HX, HY = Cfg::HY, NT = Cfg::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[Cfg::SMEM];
  unsigned char* halo = smem;
  unsigned char* wl = smem + Cfg::HALO_B;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 31, hh = lane >> 5;
  const int ct = blockIdx.x % p.nct;
  const int st = blockIdx.x / p.nct;
  const int ix = st % p.tx, iy = (st / p.tx) % p.ty, iz = (st / (p.tx * p.ty)) % p.tz;
  const int b = st / (p.tx * p.ty * p.tz);
  const int x0 = ix * BX, y0 = iy * BY, z0 = iz * BZ;

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

  for (int seg = 0; seg < 2; ++seg) {
    const void *s0, *s1, *wp;
    int c0, c1, mode;
    const float* gn;
    int ntaps;
    if (seg == 0) { s0 = p.a0; s1 = p.a1; c0 = p.ac0; c1 = p.ac1; mode = p.amode; gn = p.agn; wp = p.aw; ntaps = 27; }
    else {
      if (!p.bw) break;
      s0 = p.b0; s1 = p.b1; c0 = p.bc0; c1 = p.bc1; mode = 0; gn = nullptr; wp = p.bw; ntaps = 1;
    }
    const int ctot = c0 + c1;
    const int nchunks = ctot / CK;
    for (int chunk = 0; chunk < nchunks; ++chunk) {
      __syncthreads();
      stage_halo<T, BX, BY, BZ>(halo, s0, c0, s1, c1, mode, gn, ctot, chunk, b, x0, y0, z0, p.D, p.H, p.W, tid);
      {
        const int nq = ntaps * NT * 2;
        const unsigned char* g = reinterpret_cast<const unsigned char*>(wp) +
                                 ((long long)ct * nchunks + chunk) * (long long)(ntaps * NT * 32);
        for (int i = tid; i < nq; i += 256)
          *reinterpret_cast<u32x4*>(wl + i * 16) = ldg16(g + (long long)i * 16);
      }
      __syncthreads();
      for (int tap = 0; tap < ntaps; ++tap) {
        int toff = 0;
        if (ntaps == 27) {
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
          for (int n = 0; n < NF; ++n) {
            if constexpr (sizeof(T) == 2) {
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, aq[m]),
                                                                  __builtin_bit_cast(bf16x8, bq[n]), acc[m][n], 0, 0, 0);
            } else {
#pragma unroll
              for (int s = 0; s < 4; ++s)
                acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(aq[m][s]), __uint_as_float(bq[n][s]),
                                                                 acc[m][n], 0, 0, 0);
            }
          }
      }
    }
  }

  // ---------------- epilogue ----------------
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

  constexpr int CG = NT / 8;  // 8-channel groups per row
  const int cg = tid % CG;
  const int cbase = ct * NT + cg * 8;
  const int nvalid = min(8, p.cout - cbase);
  float bsum[8], bsq[8], bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bsum[e] = 0.f;
    bsq[e] = 0.f;
    bias[e] = (e < nvalid) ? p.bias[(long long)b * p.bias_bs + cbase + e] : 0.f;
  }
  for (int u = tid; u < 256 * CG; u += 256) {
    const int row = u / CG;
    const int rx = row % BX, ry = (row / BX) % BY, rz = row / (BX * BY);
    const int ox = x0 + rx, oy = y0 + ry, oz = z0 + rz;
    if (ox >= p.W || oy >= p.H || oz >= p.D || nvalid <= 0) continue;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = E[row * Cfg::EPI_LD + cg * 8 + e] + bias[e];
    const long long vox = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
    if (p.rmode >= 0) {
      const T* r = reinterpret_cast<const T*>(p.res);
      float rv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) rv[e] = 0.f;
      if (p.rmode == 2) {
        const int RD = p.D * 2, RH = p.H * 2, RW = p.W * 2;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const long long rvx = (((long long)b * RD + 2 * oz + (k >> 2)) * RH + 2 * oy + ((k >> 1) & 1)) * RW +
                                2 * ox + (k & 1);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e < nvalid) rv[e] += Elem<T>::to_f(r[rvx * p.cout + cbase + e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) rv[e] *= 0.125f;
      } else {
        long long rvx = vox;
        if (p.rmode == 1) rvx = (((long long)b * (p.D >> 1) + (oz >> 1)) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nvalid) rv[e] = Elem<T>::to_f(r[rvx * p.cout + cbase + e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rv[e] + v[e];
    }
    if (p.out_f32) {
      float* o = reinterpret_cast<float*>(p.out) + vox * p.cout + cbase;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < nvalid) o[e] = v[e];
    } else {
      T* o = reinterpret_cast<T*>(p.out) + vox * p.cout + cbase;
      if (nvalid == 8 && sizeof(T) == 2) {
        *reinterpret_cast<u32x4*>(o) = pack<bf16_t>(v);
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
    float* R = reinterpret_cast<float*>(smem);
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

// ---- weight packing: OIDHW fp32 -> [ct][chunk][tap][n][2 quads, swizzled] ----
template <typename T>
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ w, int cout, int cin, int ntaps, int NT,
                                                   int nct, T* __restrict__ out) {
  constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ;
  const int nch = cin / CK;
  const long long total = (long long)nct * nch * ntaps * NT * CK;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int e = i % EPQ;
  long long r = i / EPQ;
  const int qp = r % 2;
  r /= 2;
  const int n = r % NT;
  r /= NT;
  const int tap = r % ntaps;
  r /= ntaps;
  const int chunk = r % nch;
  const int ct = r / nch;
  const int q = qp ^ ((n >> 3) & 1);
  const int co = ct * NT + n, ci = chunk * CK + q * EPQ + e;
  float v = 0.f;
  if (co < cout) v = w[((long long)co * cin + ci) * ntaps + tap];
  out[i] = Elem<T>::from_f(v);
}

inline int pick_nf(int cout) { return (cout % 64 == 0) ? 2 : 1; }

struct Brick { int bx, by, bz; };
inline Brick pick_brick(int64_t D, int64_t H, int64_t W) {
  (void)D; (void)H;
  if (W >= 32) return {32, 4, 2};
  if (W >= 16) return {16, 4, 4};
  return {8, 8, 4};
}

template <typename T, int BX, int BY, int BZ, int NF>
int launch_conv(const ConvParams& p, hipStream_t s) {
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz * p.nct;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d: grid too large");
  hipLaunchKernelGGL((conv3d_kernel<T, BX, BY, BZ, NF>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

template <typename T, int NF>
int dispatch_brick(const ConvParams& p, const Brick& br, hipStream_t s) {
  if (br.bx == 32) return launch_conv<T, 32, 4, 2, NF>(p, s);
  if (br.bx == 16) return launch_conv<T, 16, 4, 4, NF>(p, s);
  return launch_conv<T, 8, 8, 4, NF>(p, s);
}

int ck_of(int dtype) { return dtype == CWDM_BF16 ? 16 : 8; }

}  // namespace cwdm

using namespace cwdm;

extern "C" int64_t cwdm_conv3d_packed_bytes(int cout, int cin, int ksize, int dtype) {
  if (cout <= 0 || cin <= 0 || (ksize != 1 && ksize != 3)) return -1;
  const int ck = ck_of(dtype);
  if (cin % ck) return -1;
  const int NT = 32 * pick_nf(cout);
  const int nct = (int)ceil_div(cout, NT);
  const int ntaps = ksize * ksize * ksize;
  const int esz = dtype == CWDM_BF16 ? 2 : 4;
  return (int64_t)nct * (cin / ck) * ntaps * NT * ck * esz;
}

extern "C" int cwdm_conv3d_pack(const float* w, int cout, int cin, int ksize, int dtype, void* packed,
                                cwdm_stream_t stream) {
  CWDM_REQUIRE(w && packed, CWDM_E_INVALID, "cwdm_conv3d_pack: null pointer");
  CWDM_REQUIRE(ksize == 1 || ksize == 3, CWDM_E_UNSUPPORTED, "cwdm_conv3d_pack: kernel size must be 1 or 3");
  CWDM_REQUIRE(dtype == CWDM_F32 || dtype == CWDM_BF16, CWDM_E_INVALID, "cwdm_conv3d_pack: bad dtype");
  const int ck = ck_of(dtype);
  CWDM_REQUIRE(cin % ck == 0, CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_pack: input channels must be a multiple of " + std::to_string(ck));
  const int NT = 32 * pick_nf(cout);
  const int nct = (int)ceil_div(cout, NT);
  const int ntaps = ksize * ksize * ksize;
  const long long total = (long long)nct * (cin / ck) * ntaps * NT * ck;
  dim3 grid((unsigned)ceil_div(total, 256));
  if (dtype == CWDM_BF16)
    hipLaunchKernelGGL(pack_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, w, cout, cin, ntaps, NT, nct,
                       reinterpret_cast<bf16_t*>(packed));
  else
    hipLaunchKernelGGL(pack_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, w, cout, cin, ntaps, NT, nct,
                       reinterpret_cast<float*>(packed));
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int64_t cwdm_conv3d_parts(int dtype, int64_t D, int64_t H, int64_t W, int cout) {
  (void)dtype; (void)cout;
  Brick br = pick_brick(D, H, W);
  return ceil_div(D, br.bz) * ceil_div(H, br.by) * ceil_div(W, br.bx);
}

extern "C" int cwdm_conv3d_forward(const cwdm_conv3d_desc* d, cwdm_stream_t stream) {
  CWDM_REQUIRE(d && d->a0 && d->a_w && d->out && d->bias, CWDM_E_INVALID, "cwdm_conv3d_forward: null pointer");
  CWDM_REQUIRE(d->dtype == CWDM_F32 || d->dtype == CWDM_BF16, CWDM_E_INVALID, "cwdm_conv3d_forward: bad dtype");
  CWDM_REQUIRE(d->B > 0 && d->D > 0 && d->H > 0 && d->W > 0 && d->cout > 0, CWDM_E_SHAPE,
               "cwdm_conv3d_forward: empty shape");
  const int ck = ck_of(d->dtype);
  CWDM_REQUIRE(d->a_c0 > 0 && d->a_c0 % ck == 0 && d->a_c1 % ck == 0 && (d->a_c1 == 0 || d->a1), CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_forward: segment A channels must be multiples of " + std::to_string(ck));
  if (d->b_w)
    CWDM_REQUIRE(d->b0 && d->b_c0 > 0 && d->b_c0 % ck == 0 && d->b_c1 % ck == 0 && (d->b_c1 == 0 || d->b1),
                 CWDM_E_UNSUPPORTED, "cwdm_conv3d_forward: segment B channels must be multiples of " + std::to_string(ck));
  CWDM_REQUIRE(d->a_mode >= 0 && d->a_mode <= 2 && d->res_mode >= -1 && d->res_mode <= 2, CWDM_E_INVALID,
               "cwdm_conv3d_forward: bad resample mode");
  if (d->a_mode == 1 || d->res_mode == 1)
    CWDM_REQUIRE(d->D % 2 == 0 && d->H % 2 == 0 && d->W % 2 == 0, CWDM_E_SHAPE,
                 "cwdm_conv3d_forward: upsample needs an even output grid");
  CWDM_REQUIRE(d->res_mode < 0 || d->res, CWDM_E_INVALID, "cwdm_conv3d_forward: residual pointer missing");
  CWDM_REQUIRE(d->out_dtype == CWDM_F32 || d->out_dtype == d->dtype, CWDM_E_INVALID,
               "cwdm_conv3d_forward: output dtype must be fp32 or the compute dtype");
  const int nf = pick_nf(d->cout);
  CWDM_REQUIRE(nf == 2 || d->cout % 32 == 0 || d->cout < 32, CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_forward: cout must be a multiple of 32 or below 32");
  ConvParams p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W;
  Brick br = pick_brick(d->D, d->H, d->W);
  p.tx = (int)ceil_div(d->W, br.bx); p.ty = (int)ceil_div(d->H, br.by); p.tz = (int)ceil_div(d->D, br.bz);
  p.cout = d->cout; p.nct = (int)ceil_div(d->cout, 32 * nf);
  p.a0 = d->a0; p.ac0 = d->a_c0; p.a1 = d->a1; p.ac1 = d->a_c1; p.amode = d->a_mode; p.agn = d->a_gn; p.aw = d->a_w;
  p.b0 = d->b0; p.bc0 = d->b_c0; p.b1 = d->b1; p.bc1 = d->b_c1; p.bw = d->b_w;
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.res = d->res; p.rmode = d->res_mode;
  p.out = d->out; p.out_f32 = (d->out_dtype == CWDM_F32 && d->dtype != CWDM_F32) ? 1 : (d->dtype == CWDM_F32);
  p.stats = d->stats;
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == CWDM_BF16)
    return nf == 2 ? dispatch_brick<bf16_t, 2>(p, br, s) : dispatch_brick<bf16_t, 1>(p, br, s);
  return nf == 2 ? dispatch_brick<float, 2>(p, br, s) : dispatch_brick<float, 1>(p, br, s);
}
