// Pure 1x1x1 conv on the wide levels (segment B alone: the ResBlock
// skip_connection conv of unet.py:264-271 where the forward does not fuse it,
// and its input gradient in the backward -- the dual-output, accumulating
// "skip dgrad" of the plan): a channels-last GEMM over voxels,
//
//   out[b, v, n] (+)= bias[n] + sum_k in[b, v, k] W[n][k],   in = concat(b0, b1)
//
// memory-bound (K, N <= a few hundred), so the design is about streaming: one
// workgroup = 256 voxels x 128 output channels; wave w = 64 voxels (two 32-voxel
// blocks) x 4 blocks of 32 channels = 8 accumulators of v_mfma_f32_32x32x16
// (A = 32 output channels x 16 K of the packed weights, B = 16 K x 32 voxels
// straight from the channels-last rows, 16 B per lane); the next K step's
// fragments are loaded while this step's MFMAs run.  An accumulator lane holds
// 4 runs of 4 consecutive channels of one voxel; lane pairs (l, l + 32) swap
// halves so the epilogue stores (and, accumulating, loads) 16 bytes = 8
// channels per lane.  The brick kernels this replaces ran the R0 skip dgrads
// at ~0.06 PF (690-910 us each, ~3 ms per training step).
#include <atomic>
#include "conv3d_kernels.hpp"

namespace cwdm {

struct PwParams {
  long long V;            // voxels per batch entry (all of them: B * V rows)
  long long rows;         // B * V
  int K, K0;              // input channels (b0: K0, b1: K - K0)
  const void* b0;
  const void* b1;
  const unsigned char* w; // cwdm_conv3d_pack layout, ksize 1 (NT rows per channel tile, 16-channel chunks)
  int N, NT;
  const float* bias; long long bias_bs;
  void* out; void* out1; int out_c0; int accumulate;
  int nnb;                // 128-channel blocks of N
  // fused GroupNorm-backward apply (GapplyFuse): gx0 / gx1 split as out / out1
  const void* gx0; const void* gx1; const void* gdu; const float* gss; const float* gcoef;
};

thread_local GapplyFuse* g_gapply = nullptr;
// the fused-apply skip dgrad's row-major epilogue on / off (cwdm_debug_pw_lt), and its launches
std::atomic<int> g_pw_lt{[] { const char* e = std::getenv("CWDM_PW_LT"); return (e && e[0] == '0') ? 0 : 1; }()};
std::atomic<int> g_pw_lt_launches{0};

namespace {

// element (co, ci) of the packed weights (pack_elem's layout, one tap)
template <typename T>
__device__ __forceinline__ long long pw_widx(int co, int ci, int K, int NT) {
  constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ;
  const int ct = co / NT, n = co % NT, chunk = ci / CK, q = (ci % CK) / EPQ, e = ci % EPQ;
  const int qp = q ^ ((n >> 3) & 1);
  return ((((long long)ct * (K / CK) + chunk) * NT + n) * 2 + qp) * EPQ + e;
}

// d/dz SiLU(z) * du as gn_bwd_apply_kernel computes it (grad.hip dsilu)
__device__ __forceinline__ float pw_dsilu(float z, float du) {
  const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -1.4426950408889634f));
  return du * (s * (1.0f + z * (1.0f - s)));
}

// NM: 32-channel output blocks per workgroup (4: 128 channels, 2 waves / SIMD;
// 2: 64 channels, the fused-apply instance -- 3 waves / SIMD to keep more of
// its three input streams in flight)
// LT: the row-major epilogue (accumulators transposed through LDS, every load / store a
// run of whole rows) and the XCD-grouped block order (the nnb channel blocks of a voxel
// tile on one XCD, so its dout rows come from that XCD's L2 after the first)
template <typename T, bool GA, int NM, bool LT = false>
__global__ void __launch_bounds__(256, NM == 2 ? 3 : 2) pw_kernel(PwParams p) {
  constexpr int NC = 32 * NM;                      // output channels per workgroup
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  long long wid = blockIdx.x;
  if constexpr (LT) {
    const unsigned G = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
    wid = (long long)(xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  }
  const long long vt = wid / p.nnb;
  const int nb = (int)(wid % p.nnb);
  const long long row0 = vt * 256 + wv * 64;       // this wave's first voxel row (over B * V)
  const int n0 = nb * NC;
  // fused GroupNorm-backward apply (GA): the block's NC channels' (sc, sh, k0,
  // k1, k2) for the (at most two) batch entries its 256 rows touch, in LDS
  __shared__ float gk[2][5][NC];
  const long long b_lo = (vt * 256) / p.V;
  if (GA) {
    for (int i = tid; i < 2 * NC; i += 256) {
      const int bl = i / NC, cl = i % NC, c = n0 + cl;
      const long long b = b_lo + bl;
      if (c < p.N && b * p.V < p.rows) {
        const float2 ss = *reinterpret_cast<const float2*>(p.gss + (b * p.N + c) * 2);
        const float4 k = *reinterpret_cast<const float4*>(p.gcoef + (b * p.N + c) * 4);
        gk[bl][0][cl] = ss.x; gk[bl][1][cl] = ss.y;
        gk[bl][2][cl] = k.x; gk[bl][3][cl] = k.y; gk[bl][4][cl] = k.z;
      }
    }
    __syncthreads();
  }
  const int col = lane & 31, kg = lane >> 5;       // MFMA operand lane: column / row 0..31, K half
  const T* w = reinterpret_cast<const T*>(p.w);
  f32x16 acc[2][NM];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[j][m][i] = 0.f;

  // operand sources of K step s (16 channels): B = voxel row (row0 + 32 j + col),
  // channels 16 s + 8 kg .. +8; A = output channel n0 + 32 m + col, same channels
  auto ldB = [&](int s, int j) -> u32x4 {
    const long long r = row0 + 32 * j + col;
    const int k = 16 * s + 8 * kg;
    if (r >= p.rows) return u32x4{0u, 0u, 0u, 0u};
    const T* src = k < p.K0 ? reinterpret_cast<const T*>(p.b0) + r * p.K0 + k
                            : reinterpret_cast<const T*>(p.b1) + r * (p.K - p.K0) + (k - p.K0);
    return *reinterpret_cast<const u32x4*>(src);
  };
  auto ldA = [&](int s, int m) -> u32x4 {
    const int co = n0 + 32 * m + col;
    if (co >= p.N) return u32x4{0u, 0u, 0u, 0u};
    return *reinterpret_cast<const u32x4*>(w + pw_widx<T>(co, 16 * s + 8 * kg, p.K, p.NT));
  };
  const int ns = p.K / 16;
  u32x4 a[NM], b[2], an[NM], bn[2];
#pragma unroll
  for (int m = 0; m < NM; ++m) a[m] = ldA(0, m);
#pragma unroll
  for (int j = 0; j < 2; ++j) b[j] = ldB(0, j);
  for (int s = 0; s < ns; ++s) {
    if (s + 1 < ns) {
#pragma unroll
      for (int m = 0; m < NM; ++m) an[m] = ldA(s + 1, m);
#pragma unroll
      for (int j = 0; j < 2; ++j) bn[j] = ldB(s + 1, j);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < NM; ++m) mfma_acc(acc[j][m], a[m], b[j], (T*)nullptr);
    if (s + 1 < ns) {
#pragma unroll
      for (int m = 0; m < NM; ++m) a[m] = an[m];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = bn[j];
    }
  }
  // epilogue: acc[j][m][i] = channel n0 + 32 m + 8 (i >> 2) + 4 kg + (i & 3) of voxel row row0 + 32 j + col.
  // Lanes l and l + 32 hold the two 4-channel halves of each 8-channel group:
  // v_permlane32_swap over the group pairs (2 gg, 2 gg + 1) gives every lane 8
  // consecutive channels, channel base n0 + 32 m + 16 gg + 8 kg -> 16-byte stores
  // (the 8-byte stores scattered every instruction over 32 rows: the R0 skip
  // dgrads ran at 1.5-2.2 TB/s).  The swaps run on every lane (no divergence
  // around a cross-lane op); only the loads / stores are predicated.
  const bool f8 = p.N % 8 == 0 && (!p.out1 || p.out_c0 % 8 == 0);
  if constexpr (LT) {
    // (the host takes LT only with f8)  Wave wv's 32 x NC accumulator block j goes to its
    // LDS slice as fp32 (row = voxel, 4 pad words: the 16-byte writes of lanes col and
    // col + 1 land 4 banks apart); then lane (rl, cg) owns channels n0 + 8 cg .. + 8 of rows
    // RPI it + rl: every load / store instruction covers RPI whole NC-channel row segments.
    // Same arithmetic, same order as the swapped-lane epilogue below (bitwise equal).
    constexpr int LPR = NC / 8, RPI = 64 / LPR, NIT = 32 / RPI, SROW = NC + 4;
    constexpr int NIH = NM == 4 ? NIT / 2 : NIT;   // row groups whose loads are in flight together (registers)
    __shared__ __attribute__((aligned(16))) float stg[4 * 32 * SROW];
    float* const ws = stg + wv * 32 * SROW;
    const int rl = lane / LPR, cg = lane % LPR, cl = 8 * cg, c = n0 + cl;
    const bool cok = c < p.N;
    const bool second = p.out1 && c >= p.out_c0;
    const long long ost = second ? p.N - p.out_c0 : (p.out1 ? p.out_c0 : p.N);
    T* const ob = second ? reinterpret_cast<T*>(p.out1) + (c - p.out_c0) : reinterpret_cast<T*>(p.out) + c;
    const T* const xb = !GA ? nullptr
                            : second ? reinterpret_cast<const T*>(p.gx1) + (c - p.out_c0)
                                     : reinterpret_cast<const T*>(p.gx0) + c;
    const T* const db = GA ? reinterpret_cast<const T*>(p.gdu) + c : nullptr;
    // 16-lane groups read rows' 8-word runs: lanes cg and cg + 8 start in opposite halves
    const int hs = (cg >> 3) & 1;
    int kb = -1;
    float kc[5][8];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(ws + col * SROW + 32 * m + 8 * g + 4 * kg) =
              float4{acc[j][m][4 * g], acc[j][m][4 * g + 1], acc[j][m][4 * g + 2], acc[j][m][4 * g + 3]};
      __syncthreads();
#pragma unroll
      for (int i0 = 0; i0 < NIT; i0 += NIH) {
      u32x4 qo[NIT], qx[NIT], qd[NIT];
#pragma unroll
      for (int it = i0; it < i0 + NIH; ++it) {
        const long long r = row0 + 32 * j + RPI * it + rl;
        const bool ok = cok && r < p.rows;
        qo[it] = qx[it] = qd[it] = u32x4{0u, 0u, 0u, 0u};
        if (ok && p.accumulate) qo[it] = *reinterpret_cast<const u32x4*>(ob + r * ost);
        if (GA && ok) {
          qx[it] = *reinterpret_cast<const u32x4*>(xb + r * ost);
          qd[it] = *reinterpret_cast<const u32x4*>(db + r * p.N);
        }
      }
#pragma unroll
      for (int it = i0; it < i0 + NIH; ++it) {
        const long long r = row0 + 32 * j + RPI * it + rl;
        const bool rin = r < p.rows, ok = cok && rin;
        const float* sp = ws + (RPI * it + rl) * SROW + cl;
        const float4 h0 = *reinterpret_cast<const float4*>(sp + 4 * hs);
        const float4 h1 = *reinterpret_cast<const float4*>(sp + 4 - 4 * hs);
        float v[8] = {hs ? h1.x : h0.x, hs ? h1.y : h0.y, hs ? h1.z : h0.z, hs ? h1.w : h0.w,
                      hs ? h0.x : h1.x, hs ? h0.y : h1.y, hs ? h0.z : h1.z, hs ? h0.w : h1.w};
        const int bb = rin ? (int)(r / p.V) : 0;
        if (p.bias && ok) {
          const float* bs = p.bias + (long long)bb * p.bias_bs + c;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bs[e];
        }
        auto unpack = [&](const u32x4& q, float (&f)[8]) {
#pragma unroll
          for (int i = 0; i < 4; ++i) { f[2 * i] = lo2f<T>(q[i]); f[2 * i + 1] = hi2f<T>(q[i]); }
        };
        if (p.accumulate) {
          float f[8];
          unpack(qo[it], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += f[e];
        }
        if (GA) {
          const int bl = rin ? (int)(bb - b_lo) : 0;
          if (bl != kb) {
#pragma unroll
            for (int t = 0; t < 5; ++t) {
              const float4 k0 = *reinterpret_cast<const float4*>(&gk[bl][t][cl]);
              const float4 k1 = *reinterpret_cast<const float4*>(&gk[bl][t][cl + 4]);
              kc[t][0] = k0.x; kc[t][1] = k0.y; kc[t][2] = k0.z; kc[t][3] = k0.w;
              kc[t][4] = k1.x; kc[t][5] = k1.y; kc[t][6] = k1.z; kc[t][7] = k1.w;
            }
            kb = bl;
          }
          float xv[8], dv[8];
          unpack(qx[it], xv);
          unpack(qd[it], dv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = pw_dsilu(xv[e] * kc[0][e] + kc[1][e], dv[e]);
            v[e] += kc[2][e] * dz + kc[3][e] * xv[e] + kc[4][e];
          }
        }
        u32x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = pack2<T>(v[2 * i], v[2 * i + 1]);
        if (ok) *reinterpret_cast<u32x4*>(ob + r * ost) = w;
      }
      }
      __syncthreads();   // (block j + 1 reuses the slice)
    }
    return;
  }
  if (f8) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long long r = row0 + 32 * j + col;
      const bool rin = r < p.rows;
      const int bb = rin ? (int)(r / p.V) : 0;
      const int bl = GA && rin ? (int)(bb - b_lo) : 0;
      // groups ga = 2 gg, gb = 2 gg + 1 of acc[j][m]: in the accumulator layout
      // this lane holds channels 8 g + 4 kg + e of both; after the swap, the 8
      // channels from c.  All of the row's loads first (one memory latency per
      // row instead of one per 8 channels: the epilogue runs at 1 wave / SIMD)
      auto chan = [&](int m, int gg) { return n0 + 32 * m + 16 * gg + 8 * kg; };
      auto optr = [&](int c) -> T* {
        if (p.out1 && c >= p.out_c0) return reinterpret_cast<T*>(p.out1) + r * (p.N - p.out_c0) + (c - p.out_c0);
        return reinterpret_cast<T*>(p.out) + r * (p.out1 ? p.out_c0 : p.N) + c;
      };
      // (GA: half a row's loads at a time -- the fused apply's registers fit 2 waves / SIMD)
      constexpr int MB = GA ? (NM == 2 ? 1 : 2) : NM;
#pragma unroll
      for (int m0 = 0; m0 < NM; m0 += MB) {
      u32x4 qo[NM][2], qx[NM][2], qd[NM][2];
#pragma unroll
      for (int m = m0; m < m0 + MB; ++m)
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int c = chan(m, gg);
          const bool ok = rin && c < p.N;
          qo[m][gg] = qx[m][gg] = qd[m][gg] = u32x4{0u, 0u, 0u, 0u};
          if (ok && p.accumulate) qo[m][gg] = *reinterpret_cast<const u32x4*>(optr(c));
          if (GA && ok) {
            const T* xs = (p.out1 && c >= p.out_c0)
                              ? reinterpret_cast<const T*>(p.gx1) + r * (p.N - p.out_c0) + (c - p.out_c0)
                              : reinterpret_cast<const T*>(p.gx0) + r * (p.out1 ? p.out_c0 : p.N) + c;
            qx[m][gg] = *reinterpret_cast<const u32x4*>(xs);
            qd[m][gg] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(p.gdu) + r * p.N + c);
          }
        }
#pragma unroll
      for (int m = m0; m < m0 + MB; ++m) {
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int ga = 2 * gg, gb = 2 * gg + 1;
          const int c = chan(m, gg);
          const bool ok = rin && c < p.N;
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[j][m][4 * ga + e];
            v[4 + e] = acc[j][m][4 * gb + e];
          }
          if (p.bias && rin) {
            const float* bs = p.bias + (long long)bb * p.bias_bs + n0 + 32 * m + 4 * kg;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (8 * ga + 4 * kg + e + n0 + 32 * m < p.N) v[e] += bs[8 * ga + e];
              if (8 * gb + 4 * kg + e + n0 + 32 * m < p.N) v[4 + e] += bs[8 * gb + e];
            }
          }
          // 8 channels at c (post-swap layout) -> the accumulator layout (as the
          // residual of conv3d_v4.hpp's fast epilogue); the swaps run on every lane
          auto to_acc = [&](const u32x4& q, float (&f)[8]) {
            const auto s0 = __builtin_amdgcn_permlane32_swap(q[0], q[2], false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(q[1], q[3], false, false);
            const unsigned g0 = s0[0], g1 = s1[0], h0 = s0[1], h1 = s1[1];
            f[0] = lo2f<T>(g0); f[1] = hi2f<T>(g0); f[2] = lo2f<T>(g1); f[3] = hi2f<T>(g1);
            f[4] = lo2f<T>(h0); f[5] = hi2f<T>(h0); f[6] = lo2f<T>(h1); f[7] = hi2f<T>(h1);
          };
          if (p.accumulate) {
            float f[8];
            to_acc(qo[m][gg], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += f[e];
          }
          if (GA) {
            // + the GroupNorm-backward apply of the same (voxel, channel)
            float xv[8], dv[8];
            to_acc(qx[m][gg], xv);
            to_acc(qd[m][gg], dv);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int lc = 32 * m + 8 * (h ? gb : ga) + 4 * kg;   // channel - n0 of v[4 h .. 4 h + 3]
              float4 k[5];
#pragma unroll
              for (int t = 0; t < 5; ++t) k[t] = *reinterpret_cast<const float4*>(&gk[bl][t][lc]);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float x = xv[4 * h + e];
                const float dz = pw_dsilu(x * k[0][e] + k[1][e], dv[4 * h + e]);
                v[4 * h + e] += k[2][e] * dz + k[3][e] * x + k[4][e];
              }
            }
          }
          const unsigned p0 = pack2<T>(v[0], v[1]), p1 = pack2<T>(v[2], v[3]);
          const unsigned p2 = pack2<T>(v[4], v[5]), p3 = pack2<T>(v[6], v[7]);
          const auto t0 = __builtin_amdgcn_permlane32_swap(p0, p2, false, false);
          const auto t1 = __builtin_amdgcn_permlane32_swap(p1, p3, false, false);
          u32x4 w;
          w[0] = t0[0]; w[1] = t1[0]; w[2] = t0[1]; w[3] = t1[1];
          if (ok) *reinterpret_cast<u32x4*>(optr(c)) = w;
        }
      }
      }
    }
    return;
  }
  if (GA) return;   // (the host takes the fused apply only with f8)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const long long r = row0 + 32 * j + col;
    if (r >= p.rows) continue;
    const int bb = (int)(r / p.V);
#pragma unroll
    for (int m = 0; m < NM; ++m) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = n0 + 32 * m + 8 * g + 4 * kg;   // 4 consecutive channels c .. c+3
        if (c >= p.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = acc[j][m][4 * g + e] + (p.bias ? p.bias[(long long)bb * p.bias_bs + c + e] : 0.f);
        T* o;
        if (p.out1 && c >= p.out_c0) o = reinterpret_cast<T*>(p.out1) + r * (p.N - p.out_c0) + (c - p.out_c0);
        else o = reinterpret_cast<T*>(p.out) + r * (p.out1 ? p.out_c0 : p.N) + c;
        uint2 q;
        if (p.accumulate) {
          q = *reinterpret_cast<const uint2*>(o);
          v[0] += lo2f<T>(q.x); v[1] += hi2f<T>(q.x);
          v[2] += lo2f<T>(q.y); v[3] += hi2f<T>(q.y);
        }
        q.x = pack2<T>(v[0], v[1]);
        q.y = pack2<T>(v[2], v[3]);
        *reinterpret_cast<uint2*>(o) = q;
      }
    }
  }
}

// The accurate fast mode's 1x1 skip (fp32 in / out, the conv3d_v5s split):
// three bf16 MFMA passes per 16 K -- hi(x) hi(w) + lo(x) hi(w) + hi(x) lo(w),
// lo = bf16(v - hi) -- with both operands split in registers (the weights from
// their fp32 packing), 2^-16 relative per product.  The exact-fp32 brick kernel
// it replaces ran the 128^3 skips at ~40 TF/s (1.0-1.3 ms each, 5 ms per
// accurate-mode step).  Same tiling as pw_kernel: workgroup = 256 voxels x 32 NM
// output channels, wave = 2 x 32 voxels; fp32 epilogue straight from the
// accumulators (4 consecutive channels = 16 bytes per lane and row).
template <int NM>
__global__ void __launch_bounds__(256, 2) pw_split_kernel(PwParams p) {
  constexpr int NC = 32 * NM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long long vt = blockIdx.x / p.nnb;
  const int nb = blockIdx.x % p.nnb;
  const long long row0 = vt * 256 + wv * 64;
  const int n0 = nb * NC;
  const int col = lane & 31, kg = lane >> 5;
  const float* w = reinterpret_cast<const float*>(p.w);
  f32x16 acc[2][NM];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[j][m][i] = 0.f;
  // 8 consecutive K values of K step s: B = voxel row (row0 + 32 j + col), A = output channel
  // n0 + 32 m + col (its two 4-channel quads of the fp32 packing)
  auto ldB = [&](int s, int j, float4 (&f)[2]) {
    const long long r = row0 + 32 * j + col;
    const int k = 16 * s + 8 * kg;
    if (r >= p.rows) { f[0] = f[1] = make_float4(0.f, 0.f, 0.f, 0.f); return; }
    const float* src = k < p.K0 ? reinterpret_cast<const float*>(p.b0) + r * p.K0 + k
                                : reinterpret_cast<const float*>(p.b1) + r * (p.K - p.K0) + (k - p.K0);
    f[0] = *reinterpret_cast<const float4*>(src);
    f[1] = *reinterpret_cast<const float4*>(src + 4);
  };
  auto ldA = [&](int s, int m, float4 (&f)[2]) {
    const int co = n0 + 32 * m + col;
    if (co >= p.N) { f[0] = f[1] = make_float4(0.f, 0.f, 0.f, 0.f); return; }
    const int k = 16 * s + 8 * kg;
    f[0] = *reinterpret_cast<const float4*>(w + pw_widx<float>(co, k, p.K, p.NT));
    f[1] = *reinterpret_cast<const float4*>(w + pw_widx<float>(co, k + 4, p.K, p.NT));
  };
  auto split = [](const float4 (&f)[2], u32x4& hi, u32x4& lo) {
    const float v[8] = {f[0].x, f[0].y, f[0].z, f[0].w, f[1].x, f[1].y, f[1].z, f[1].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      hi[e] = pack2<bf16_t>(v[2 * e], v[2 * e + 1]);
      lo[e] = pack2<bf16_t>(v[2 * e] - lo2f<bf16_t>(hi[e]), v[2 * e + 1] - hi2f<bf16_t>(hi[e]));
    }
  };
  const int ns = p.K / 16;
  float4 fa[NM][2], fb[2][2];
#pragma unroll
  for (int m = 0; m < NM; ++m) ldA(0, m, fa[m]);
#pragma unroll
  for (int j = 0; j < 2; ++j) ldB(0, j, fb[j]);
  for (int s = 0; s < ns; ++s) {
    u32x4 ah[NM], al[NM], bh[2], bl[2];
#pragma unroll
    for (int m = 0; m < NM; ++m) split(fa[m], ah[m], al[m]);
#pragma unroll
    for (int j = 0; j < 2; ++j) split(fb[j], bh[j], bl[j]);
    if (s + 1 < ns) {
#pragma unroll
      for (int m = 0; m < NM; ++m) ldA(s + 1, m, fa[m]);
#pragma unroll
      for (int j = 0; j < 2; ++j) ldB(s + 1, j, fb[j]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        mfma_acc(acc[j][m], ah[m], bh[j], (bf16_t*)nullptr);
        mfma_acc(acc[j][m], ah[m], bl[j], (bf16_t*)nullptr);
        mfma_acc(acc[j][m], al[m], bh[j], (bf16_t*)nullptr);
      }
  }
  // acc[j][m][4 g + e] = channel n0 + 32 m + 8 g + 4 kg + e of voxel row row0 + 32 j + col
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const long long r = row0 + 32 * j + col;
    if (r >= p.rows) continue;
    const long long bb = r / p.V;
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = n0 + 32 * m + 8 * g + 4 * kg;
        if (c >= p.N) continue;
        float4 v = make_float4(acc[j][m][4 * g], acc[j][m][4 * g + 1], acc[j][m][4 * g + 2], acc[j][m][4 * g + 3]);
        if (p.bias) {
          const float* bs = p.bias + bb * p.bias_bs + c;
          v.x += bs[0]; v.y += bs[1]; v.z += bs[2]; v.w += bs[3];
        }
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + r * p.N + c) = v;
      }
  }
}

}  // namespace

// shapes the pointwise kernel takes: a pure 1x1 (segment B only), 16-bit, no
// residual / statistics, output in the compute dtype, channels in 16s
bool pw_eligible(const cwdm_conv3d_desc* d) {
  if (!dtype_half(d->dtype) || d->a_w || !d->b_w || d->res_mode >= 0 || d->stats || d->out_dtype != d->dtype)
    return false;
  const int K = d->b_c0 + d->b_c1;
  if (K % 16 || d->b_c0 % 16 || d->cout % 8 || (d->out1 && d->out_c0 % 4)) return false;
  return d->B * d->D * d->H * d->W < (1LL << 40);
}

bool head_eligible(const cwdm_conv3d_desc* d);
// the skip dgrad d runs pw_kernel and can take a GapplyFuse (the conditions pw_forward checks)
bool pw_gapply_ok(const cwdm_conv3d_desc* d) {
  return !head_eligible(d) && pw_eligible(d) && d->cout % 8 == 0 && (!d->out1 || d->out_c0 % 8 == 0) &&
         d->D * d->H * d->W >= 256 && !d->bias;
}

int pw_forward(const cwdm_conv3d_desc* d, hipStream_t s) {
  PwParams p{};
  p.V = d->D * d->H * d->W;
  p.rows = d->B * p.V;
  p.K = d->b_c0 + d->b_c1; p.K0 = d->b_c0;
  p.b0 = d->b0; p.b1 = d->b1;
  p.w = reinterpret_cast<const unsigned char*>(d->b_w);
  p.N = d->cout;
  p.NT = 32 * pick_nf(d->cout);   // the packed layout's rows per channel tile (cwdm_conv3d_pack)
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.out = d->out; p.out1 = d->out1; p.out_c0 = d->out_c0; p.accumulate = d->accumulate;
  if (g_gapply && !g_gapply->used && p.N % 8 == 0 && (!d->out1 || d->out_c0 % 8 == 0) && p.V >= 256 &&
      !d->bias) {
    p.gx0 = g_gapply->x0; p.gx1 = g_gapply->x1; p.gdu = g_gapply->du;
    p.gss = g_gapply->ss; p.gcoef = g_gapply->coef;
    g_gapply->used = true;
  }
  const bool ga = p.gdu != nullptr;
  // row-major LDS epilogue (pw_kernel LT): cwdm_debug_pw_lt / env CWDM_PW_LT = 0 restores the swapped-lane one
  const bool lt = g_pw_lt.load(std::memory_order_relaxed) && ga;
  if (lt) g_pw_lt_launches.fetch_add(1, std::memory_order_relaxed);
  // the fused apply on 64-channel blocks where 128-channel ones would leave a
  // half-empty block (N = 192: 916 -> 770 us at 128^3; N = 128 stays on 128:
  // 491 vs 526 us); env CWDM_PW_GA_NM = 2 / 4 forces one (A/B knob)
  static const int ga_nm = [] { const char* e = std::getenv("CWDM_PW_GA_NM"); return e ? std::atoi(e) : 0; }();
  const int nm = !ga ? 4 : (ga_nm == 2 || ga_nm == 4) ? ga_nm : (d->cout % 128 ? 2 : 4);
  p.nnb = (int)ceil_div(d->cout, 32 * nm);
  const long long nblk = ceil_div(p.rows, 256) * p.nnb;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d (pointwise): grid too large");
  prof_begin(s);
  if (d->dtype == CWDM_F16) {
    if (lt && nm == 2) hipLaunchKernelGGL((pw_kernel<f16_t, true, 2, true>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else if (lt) hipLaunchKernelGGL((pw_kernel<f16_t, true, 4, true>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else if (ga && nm == 2) hipLaunchKernelGGL((pw_kernel<f16_t, true, 2>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else if (ga) hipLaunchKernelGGL((pw_kernel<f16_t, true, 4>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((pw_kernel<f16_t, false, 4>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  } else {
    if (lt && nm == 2) hipLaunchKernelGGL((pw_kernel<bf16_t, true, 2, true>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else if (lt) hipLaunchKernelGGL((pw_kernel<bf16_t, true, 4, true>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else if (ga && nm == 2) hipLaunchKernelGGL((pw_kernel<bf16_t, true, 2>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else if (ga) hipLaunchKernelGGL((pw_kernel<bf16_t, true, 4>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((pw_kernel<bf16_t, false, 4>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  }
  prof_end(s, 2.0 * p.rows * (double)p.N * p.K);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

// the accurate fast mode's pure 1x1 (a_w_split marks it: the split weights of
// the conv this skip belongs to): fp32, no residual / statistics / second output
bool pw_split_eligible(const cwdm_conv3d_desc* d) {
  if (d->dtype != CWDM_F32 || !d->a_w_split || d->a_w || !d->b_w || d->res_mode >= 0 || d->stats ||
      d->out_dtype != CWDM_F32 || d->out1 || d->accumulate)
    return false;
  const int K = d->b_c0 + d->b_c1;
  return K % 16 == 0 && d->b_c0 % 16 == 0 && d->cout % 32 == 0 && d->B * d->D * d->H * d->W < (1LL << 40);
}

int pw_split_forward(const cwdm_conv3d_desc* d, hipStream_t s) {
  PwParams p{};
  p.V = d->D * d->H * d->W;
  p.rows = d->B * p.V;
  p.K = d->b_c0 + d->b_c1; p.K0 = d->b_c0;
  p.b0 = d->b0; p.b1 = d->b1;
  p.w = reinterpret_cast<const unsigned char*>(d->b_w);
  p.N = d->cout;
  p.NT = 32 * pick_nf(d->cout);   // the fp32 packing's rows per channel tile
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.out = d->out;
  const int nm = d->cout % 128 ? 2 : 4;
  p.nnb = (int)ceil_div(d->cout, 32 * nm);
  const long long nblk = ceil_div(p.rows, 256) * p.nnb;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d (pointwise split): grid too large");
  prof_begin(s);
  if (nm == 2) hipLaunchKernelGGL((pw_split_kernel<2>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((pw_split_kernel<4>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  prof_end(s, 2.0 * p.rows * (double)p.N * p.K);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace cwdm

extern "C" int cwdm_debug_pw_lt(int on) {
  if (on < 0) return cwdm::g_pw_lt_launches.load(std::memory_order_relaxed);
  return cwdm::g_pw_lt.exchange(on ? 1 : 0);
}
