// Conv3d 3x3x3 (stride 1, pad 1) implicit GEMM, DMA-staged variant for the
// wide U-Net levels (W >= 32, H % 4 == 0, D % 4 == 0, cout % 64 == 0; a last
// x tile past W computes zero-padded voxels and masks them at the epilogue).
//
// Design (MI355X / gfx950):
//   * The input is already activated (GroupNorm+SiLU applied by
//     cwdm_gn_apply, or a raw tensor), so staging is a pure copy: every byte
//     of the halo and of the weights reaches LDS through LDS-DMA
//     (buffer_load/global_load ... lds): no VGPRs, no VALU, no ds_write.
//     Zero padding comes for free from the buffer range check (out-of-volume
//     lanes get an out-of-range offset and the DMA writes zeros).
//   * Tile = a 32(x) x 4(y) x 4(z) brick (512 voxels) x 64 output channels.
//     4 waves; wave w owns output channels [32 (w & 1), +32) and the two
//     z-planes 2 (w >> 1) .. +1 of the brick: 8 accumulators of 32 ch x 32 vox.
//   * Operands are transposed w.r.t. the plain conv (A = weights, B =
//     activations), so an accumulator lane holds 16 channels of ONE voxel and
//     the epilogue stores straight from registers (no LDS transpose).
//   * Halo image in LDS: quad-major [2 quads][1280 voxel slots][16 B]; the 16
//     lanes of a ds_read_b128 group read 16 consecutive voxels of one quad
//     plane: conflict-free, and every (dz, line, dx) offset is an immediate.
//   * K loop: chunks of 16 (bf16) / 8 (fp32) input channels; per chunk 9
//     groups (dz, dx), each = 3 dy taps x 2 planes x 4 lines = 24 MFMAs that
//     reuse 6 input lines per plane.  Weights: every lane loads its own A
//     fragments (16 B of one output channel) straight into VGPRs, one group
//     ahead, through a 3-slot register ring with counted vmcnt waits.
//   * The halo is double-buffered (the next chunk's DMA is issued at the top
//     of the current chunk): one raw s_barrier per chunk, no exposed DMA
//     latency.  Two workgroups share a CU (80 KB LDS each, <= 256 registers
//     per lane), so one workgroup's barrier and epilogue hide under the
//     other's MFMAs.
//   * Epilogue from registers: + bias, + residual (same / upsampled grid),
//     store (or accumulate), per-channel (sum, sum^2) partials for the next
//     GroupNorm, reduced across lanes with DPP and across waves in LDS.
#pragma once
#include <type_traits>

#include "conv3d_kernels.hpp"

namespace cwdm {

struct V4Params {
  int B, D, H, W;
  int tx, ty, tz;      // tiles per axis
  int nct, cout;       // channel tiles (of 64), output channels
  int nch, nch0;       // K chunks in total / from source 0
  const void* a0; int ac0; const void* a1; int ac1;
  unsigned a0_bytes, a1_bytes;        // per-batch bytes of each source (DMA range check)
  long long a0_bstride, a1_bstride;   // per-batch bytes of each source (batch offset)
  int amode;                          // 0 same grid, 1 nearest x2 upsample (source at half resolution)
  int a0_cm;                          // source 0 is chunk-major [B][C / CK][V][CK] (cwdm_gn_apply output)
  int a0_cvox;                        // voxels per batch of source 0 (chunk stride of the chunk-major layout)
  const unsigned char* aw;            // packed weights, NT = 64
  const float* bias; long long bias_bs;
  const void* res; int rmode;         // -1 none, 0 same grid, 1 upsampled
  void* out; int out_f32;
  float* stats;
  void* out1; int out_c0;
  int accumulate;
  int stagger_cycles;  // delay of the second workgroup on each CU (0: off)
  int nblk;  // work items in total (B * tx * ty * tz * nct * ksplit); gridDim.x <= nblk
  // split-K (small grids): work item = (tile, K slice ks); slice ks runs chunks
  // [ks kper, min(nch, (ks + 1) kper)) and stores its fp32 partial tile at
  // out + ks * ks_stride (the launcher points out at the fp32 slices, [V][cout]
  // each, with no bias / residual / statistics); splitk_sum_kernel +
  // conv3d_reduce_kernel finish the output.
  int ksplit, kper;
  long long ks_stride;
  unsigned long long* stamps;  // diagnostics: per-workgroup s_memtime stamps (cwdm_debug_conv_stamps), else null
  // Fused reduce pass of the SiLU(GroupNorm) backward (training: the dgrad conv
  // whose output du feeds gn_silu_bwd at the same grid; cwdm::GbwdFuse).  With
  // gx0 set the 16-bit fast epilogue stores du as usual and, instead of the
  // forward statistics, writes per-(tile, channel) partials (sum dz, sum dz xhat)
  // to stats (the [B][tiles][C][2] layout gn_bwd_finalize reads):
  // dz = du SiLU'(x sc + sh), xhat = (x - mu) rs, du as stored (rounded).  x =
  // the GroupNorm input (gx0: channels [0, gc0), gx1: the rest; channels-last);
  // gss = its [B][C][2] scale / shift, gmr = [B][G][2] mean / rstd, gdiv = C / G.
  const void* gx0; const void* gx1; int gc0;
  const float* gss; const float* gmr; int ggroups;
  FastDiv gdiv;
  // conv3d_v5: GroupNorm scale / shift [B][ac0 + ac1][2] of the raw sources, applied in LDS (null: none)
  const float* agn;
  int diag;   // timing-only diagnostics build (-DCWDM_V5_DIAG, env CWDM_V5_DIAGMASK): parts of v5 switched off
  // conv3d_v5 apply-ahead (conv3d_v5_kernel<..., AA > 0>): the kernel writes SiLU(x sc + sh) of the raw
  // channels-last sources ax0 (axc0 channels) / ax1 (axc1), sc / sh = agn, chunk-major into a0 itself,
  // aa_lead sweep iterations ahead of the tiles that read it (batch 1)
  const void* ax0; const void* ax1; int axc0, axc1; int aa_lead;
  int aa_units;   // steps of the share per chunk (<= the instance's AA loads)
  int aa_prio;    // helpers at s_setprio 1 for the share's transform (env CWDM_V5_AA_PRIO, A/B knob)
  unsigned* aa_cnt;   // this launch's sweep counters (kV5AaCnt words, zero at launch; the last workgroup out re-zeroes them)
  int aa_spin;        // bound of a counter wait (s_sleep rounds); a wait that runs out sets CWDM_DEV_E_AA_TIMEOUT
  int aa_extra;       // debug (cwdm_debug_v5_aa_timeout): arrivals a wait needs beyond the grid (forces the timeout path)
  // warp-specialised conv, batch 1, <= 2 channel tiles: GroupNorm partials per WORKGROUP instead of per
  // tile -- row blockIdx.x of stats holds the sums over the workgroup's tiles (in its tile order), every
  // channel of the row written (zeros for a channel tile it never ran): gridDim.x rows for the finalize
  int stats_wg;
};


__device__ unsigned g_v4_cu_arrivals[8 * 256];

// conv3d_v5 apply-ahead arguments (conv3d_v5.hip): the raw sources of a GroupNorm'd input, their
// scale / shift, the sweep lead and the per-chunk share of the kernel instance (v5_aa_units)
constexpr int kV5AaWords = 4096;   // apply-ahead sweep counters of one launch (conv3d_v5.hip kV5AaCnt)
struct V5Aa { const void* x0; int c0; const void* x1; int c1; const float* gn; int lead, units; unsigned* cnt; };

struct V4Cfg {
  static constexpr int HX = 34, HY = 6, HZ = 6, HV = HX * HY * HZ;  // 1224 halo voxels
  static constexpr int HVP = 1280;                                   // slots per quad plane (20 pieces)
  static constexpr int PIECES = 2 * HVP / 64;                        // 40 DMA pieces per chunk
  static constexpr int HALO_B = 2 * HVP * 16;                        // 40960 per buffer
  static constexpr int SMEM = 2 * HALO_B;                            // double-buffered halo: 80 KB
  // unused padding slots 1224..1279 of quad plane k & 1 of halo buffer k >> 1
  // (896 B each; the halo DMA never writes them): statistics scratch of wave k
  // and, in region 0 at +256, the bias of the next tile; fused GroupNorm
  // backward (gx0): the tile's scale / shift rows (64 channels x 8 B) in region
  // 1 + 2 s at +256 and its groups' mean / rstd in region 2 at +256 + 256 s,
  // double-buffered by tile parity s (the next tile's land before this epilogue)
  static constexpr int pad(int k) { return (k >> 1) * HALO_B + (k & 1) * HVP * 16 + HV * 16; }
  static constexpr int gss_off(int s) { return pad(1 + 2 * s) + 256; }
  static constexpr int gmr_off(int s) { return pad(2) + 256 + 256 * s; }
};

template <typename T>
__device__ __forceinline__ void v4_mfma(f32x16& acc, const u32x4& a, const u32x4& b) {
  mfma_acc(acc, a, b, (T*)nullptr);
}

// Weight fragments are loaded with compiler-invisible global loads: the
// compiler's own wait insertion would otherwise drain every in-flight halo
// DMA (vmcnt(0)) at the first use of an ordinary load.  Every use of a
// fragment sits behind v4_wait_w, whose "+v" operands pin the registers until
// the counted wait retires the load.
__device__ __forceinline__ void v4_gload(u32x4& dst, const unsigned char* src) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(src) : "memory");
}
#ifdef CWDM_CONV_STAMPS  // diagnostics build (tools/conv_stamps.py): per-workgroup s_memtime stamps
#define V4_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 24 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define V4_STAMP(k) do { } while (0)
#endif
// the (dz, dx) weight group of a chunk after whose weight loads the next chunk's halo DMA goes out
// (1..7; a build knob: the fills and the MFMA phase's LDS operand reads serialize on the CU's LDS)
#ifndef V4_HALO_GI
#define V4_HALO_GI 1
#endif
#define V4_WAIT_W(n, w) \
  asm volatile("s_waitcnt vmcnt(" #n ")" : "+v"((w)[0]), "+v"((w)[1]), "+v"((w)[2]) :: "memory")

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}

// sum of v over the 16 lanes of each DPP row, result in every lane of the row
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));  // quad_perm 1,0,3,2
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));  // quad_perm 2,3,0,1
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true)); // row_half_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true)); // row_mirror
  return v;
}

// the 6 input lines (y0 - 1 .. y0 + 4) of plane K % 2 for group K / 2 = (dz, dx)
template <int K>
__device__ __forceinline__ void v4_read_step(u32x4 (&av)[6], const unsigned char* hb) {
  constexpr int G = K / 2, PL = K % 2, DZ = G / 3 - 1, DX = G % 3 - 1;
#pragma unroll
  for (int L = 0; L < 6; ++L)
    av[L] = *reinterpret_cast<const u32x4*>(hb + (((PL + 1 + DZ) * V4Cfg::HY + L) * V4Cfg::HX + (DX + 1)) * 16);
}

// Epilogue of one output tile from the accumulator registers: + residual,
// store (or accumulate), per-channel (sum, sum^2) partials for the next
// GroupNorm.  R: 4 x 256 B of LDS (one slice per wave) for the cross-wave
// statistics; every wave of the workgroup calls this.
// CT32: 32-channel tiles (ct counts 32-channel tiles; wave wv = z-plane wv, one
// plane per wave); else 64-channel tiles, wave = (32-channel half wv & 1, plane
// pair wv >> 1)
template <typename T, bool FAST, bool CT32 = false, bool GB = false>
__device__ __forceinline__ void v4_epilogue(const V4Params& p, f32x16 (&acc)[2][4], int b, int sl, int ct, int x0,
                                            int y0, int z0, int ks, int tid, int wv, unsigned char* smem,
                                            int gslot = 0) {
  constexpr int NPL = CT32 ? 1 : 2;
  using T16 = std::conditional_t<sizeof(T) == 2, T, bf16_t>;   // the 16-bit storage type (bf16 / fp16)
  const int lane = tid & 63, lr = lane & 31, hh = lane >> 5;
  const int zb = CT32 ? wv : 2 * (wv >> 1);                    // the wave's first z-plane in the tile
  const int c0w = CT32 ? ct * 32 : ct * 64 + (wv & 1) * 32;    // the wave's first output channel
  const int cbase = c0w + 4 * hh;
  float ssum[16], ssq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { ssum[i] = 0.f; ssq[i] = 0.f; }
  const int ox = x0 + lr;
  const bool xin = ox < p.W;          // lanes of a partial last x tile store nothing
  const float xm = xin ? 1.f : 0.f;   // and add nothing to the statistics
  const long long HW = (long long)p.H * p.W;
  // voxel of (plane pl, line m) = vox0 + pl * HW + m * W
  const long long vox0 = (((long long)b * p.D + z0 + zb) * p.H + y0) * p.W + ox;
  if constexpr (FAST) {
    // 16-bit fast path (bf16 / fp16): 16-byte residual loads and stores.  A lane pair (l, l+32)
    // holds channels 8j..8j+7 of one voxel split 4 / 4; v_permlane32_swap turns
    // two such groups (j, j+1) into 8 consecutive channels per lane.
    // Buffer loads / stores on per-batch resources: lanes past W get an
    // out-of-range offset (loads return 0, stores are dropped), so no lane
    // branches around a memory instruction, and the residual / no-residual
    // variants are separate straight-line code: with branches inside, the
    // waitcnt pass fell back to vmcnt(0) after every store (measured: the
    // residual epilogue serialised its 16 stores).
    const int cl = c0w + 8 * hh;   // this lane's first channel (jj = 0)
    const long long V = (long long)p.D * HW;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<T16*>(p.out) + (long long)b * V * p.cout, (short)0, (int)(V * p.cout * 2), 0x00020000);
    const unsigned vb0 = (unsigned)((((z0 + zb) * p.H) + y0) * p.W + ox);  // (plane 0, line 0) in the batch
    const unsigned rowb = (unsigned)p.W * (unsigned)p.cout * 2u, planeb = (unsigned)HW * (unsigned)p.cout * 2u;
    const unsigned obase = vb0 * (unsigned)p.cout * 2u + (unsigned)cl * 2u;
    auto run = [&](auto res_c) {
      constexpr bool RES = decltype(res_c)::value;
      u32x4 rq[2][4][2];  // residual rows of both planes, all loads in flight at once
      if constexpr (RES) {
        const long long rV = p.rmode == 1 ? V / 8 : V;
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(reinterpret_cast<const T16*>(p.res) + (long long)b * rV * p.cout), (short)0,
            (int)(rV * p.cout * 2), 0x00020000);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            unsigned r0 = obase + (unsigned)pl * planeb + (unsigned)m * rowb;
            if (p.rmode == 1) {
              const int oy = y0 + m, oz = z0 + zb + pl;
              const unsigned rvb = (unsigned)(((oz >> 1) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1));
              r0 = rvb * (unsigned)p.cout * 2u + (unsigned)cl * 2u;
            }
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              rq[pl][m][jj] = __builtin_amdgcn_raw_buffer_load_b128(rr, xin ? r0 + 32u * jj : 0xFFFFFFF0u, 0, 0);
          }
        // all 16 loads ahead of every store: a load issued after a store would
        // make its wait drain that store too (vmcnt counts in issue order)
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const unsigned oo = obase + (unsigned)pl * planeb + (unsigned)m * rowb;
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            float v[8];  // groups j = 2 jj (v[0..3]) and 2 jj + 1 (v[4..7]) in accumulator layout
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = acc[pl][m][8 * jj + k];
            if constexpr (RES) {
              const u32x4 q = rq[pl][m][jj];
              const auto s0 = __builtin_amdgcn_permlane32_swap(q[0], q[2], false, false);
              const auto s1 = __builtin_amdgcn_permlane32_swap(q[1], q[3], false, false);
              const unsigned g0 = s0[0], g1 = s1[0], h0 = s0[1], h1 = s1[1];
              v[0] += lo2f<T16>(g0); v[1] += hi2f<T16>(g0);
              v[2] += lo2f<T16>(g1); v[3] += hi2f<T16>(g1);
              v[4] += lo2f<T16>(h0); v[5] += hi2f<T16>(h0);
              v[6] += lo2f<T16>(h1); v[7] += hi2f<T16>(h1);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float vv = v[k] * xm;
              ssum[8 * jj + k] += vv;
              ssq[8 * jj + k] += vv * vv;
            }
            const unsigned p0 = pack2<T16>(v[0], v[1]), p1 = pack2<T16>(v[2], v[3]);
            const unsigned p2 = pack2<T16>(v[4], v[5]), p3 = pack2<T16>(v[6], v[7]);
            const auto t0 = __builtin_amdgcn_permlane32_swap(p0, p2, false, false);
            const auto t1 = __builtin_amdgcn_permlane32_swap(p1, p3, false, false);
            u32x4 w;
            w[0] = t0[0]; w[1] = t1[0]; w[2] = t0[1]; w[3] = t1[1];
            __builtin_amdgcn_raw_buffer_store_b128(w, ro, xin ? oo + 32u * jj : 0xFFFFFFF0u, 0, 0);
          }
        }
      }
    };
    // fused GroupNorm backward reduce (no residual: a dgrad conv).  Phase 1 stores
    // du and keeps it, packed and swapped (8 consecutive channels per lane, 64
    // registers), while the 128 accumulators die; phase 2 walks the same rows of
    // x with the same layout -- so the sums need no swaps and the kernel stays
    // inside its 256 registers (taking the sums from the accumulators spilled).
    // GB sums: ssum / ssq [8 jj + k] = channel c0w + 16 jj + 8 hh + k.
    auto run_gb = [&]() {
      u32x4 du16[NPL][4][2];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const unsigned oo = obase + (unsigned)pl * planeb + (unsigned)m * rowb;
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = acc[pl][m][8 * jj + k];
            const unsigned p0 = pack2<T16>(v[0], v[1]), p1 = pack2<T16>(v[2], v[3]);
            const unsigned p2 = pack2<T16>(v[4], v[5]), p3 = pack2<T16>(v[6], v[7]);
            const auto t0 = __builtin_amdgcn_permlane32_swap(p0, p2, false, false);
            const auto t1 = __builtin_amdgcn_permlane32_swap(p1, p3, false, false);
            u32x4 w;
            w[0] = t0[0]; w[1] = t1[0]; w[2] = t0[1]; w[3] = t1[1];
            __builtin_amdgcn_raw_buffer_store_b128(w, ro, xin ? oo + 32u * jj : 0xFFFFFFF0u, 0, 0);
            du16[pl][m][jj] = w;
          }
        }
      const int tb = CT32 ? ct * 32 : ct * 64;                 // the tile's first channel
      const float* cf = reinterpret_cast<const float*>(smem + V4Cfg::gss_off(gslot));   // [c - tb][sc, sh]
      const bool first = tb < p.gc0;                           // one source per tile (host-checked)
      const int xc = first ? p.gc0 : p.cout - p.gc0, xco = first ? 0 : p.gc0;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(reinterpret_cast<const T16*>(first ? p.gx0 : p.gx1) + (long long)b * V * xc), (short)0,
          (int)(V * xc * 2), 0x00020000);
      const unsigned xrowb = (unsigned)p.W * (unsigned)xc * 2u, xplaneb = (unsigned)HW * (unsigned)xc * 2u;
      const unsigned xbase = vb0 * (unsigned)xc * 2u + (unsigned)(cl - xco) * 2u;
      const int lc0 = cl - tb;   // the lane's first channel within the tile
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        u32x4 xq[4][2];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            xq[m][jj] = __builtin_amdgcn_raw_buffer_load_b128(
                rx, xin ? xbase + (unsigned)pl * xplaneb + (unsigned)m * xrowb + 32u * jj : 0xFFFFFFF0u, 0, 0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const u32x4 dq = du16[pl][m][jj], xqq = xq[m][jj];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const unsigned dw = dq[k >> 1], xw = xqq[k >> 1];
              const float du = (k & 1) ? hi2f<T16>(dw) : lo2f<T16>(dw);
              const float xv = (k & 1) ? hi2f<T16>(xw) : lo2f<T16>(xw);
              const float2 scsh = *reinterpret_cast<const float2*>(cf + 2 * (lc0 + 16 * jj + k));
              const float z = xv * scsh.x + scsh.y;
              const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -1.4426950408889634f));
              const float dz = du * (s * (1.0f + z * (1.0f - s))) * xm;
              ssum[8 * jj + k] += dz;
              ssq[8 * jj + k] += dz * xv;   // sum dz x; the tile's sum dz xhat = rs (sum dz x - mu sum dz), below
            }
          }
      }
    };
    if constexpr (GB) run_gb();
    else if (p.rmode >= 0) run(std::true_type{});
    else run(std::false_type{});
  } else {
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (!xin) continue;
        const int oy = y0 + m, oz = z0 + zb + pl;
        const long long vox = vox0 + pl * HW + (long long)m * p.W;
        long long rvox = vox;
        if (p.rmode == 1)
          rvox = (((long long)b * (p.D >> 1) + (oz >> 1)) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = cbase + 8 * j;
          float v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = acc[pl][m][4 * j + k];
          if (p.rmode >= 0) {
            const T* r = reinterpret_cast<const T*>(p.res) + rvox * p.cout + co;
            if constexpr (sizeof(T) == 2) {
              const uint2 rq = *reinterpret_cast<const uint2*>(r);
              v[0] += lo2f<T16>(rq.x); v[1] += hi2f<T16>(rq.x);
              v[2] += lo2f<T16>(rq.y); v[3] += hi2f<T16>(rq.y);
            } else {
              const float4 rq = *reinterpret_cast<const float4*>(r);
              v[0] += rq.x; v[1] += rq.y; v[2] += rq.z; v[3] += rq.w;
            }
          }
          void* obase = p.out;
          int ostride = p.cout, oc = co;
          if (p.out1) {
            if (co >= p.out_c0) { obase = p.out1; ostride = p.cout - p.out_c0; oc = co - p.out_c0; }
            else ostride = p.out_c0;
          }
          if (p.out_f32 || sizeof(T) == 4) {
            float* o = reinterpret_cast<float*>(obase) + ks * p.ks_stride + vox * ostride + oc;
            if (p.accumulate) {
              const float4 oq = *reinterpret_cast<const float4*>(o);
              v[0] += oq.x; v[1] += oq.y; v[2] += oq.z; v[3] += oq.w;
            }
            *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            T16* o = reinterpret_cast<T16*>(obase) + vox * ostride + oc;
            if (p.accumulate) {
              const uint2 oq = *reinterpret_cast<const uint2*>(o);
              v[0] += lo2f<T16>(oq.x); v[1] += hi2f<T16>(oq.x);
              v[2] += lo2f<T16>(oq.y); v[3] += hi2f<T16>(oq.y);
            }
            uint2 sq;
            sq.x = pack2<T16>(v[0], v[1]);
            sq.y = pack2<T16>(v[2], v[3]);
            *reinterpret_cast<uint2*>(o) = sq;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            ssum[4 * j + k] += v[k];
            ssq[4 * j + k] += v[k] * v[k];
          }
        }
      }
    }
  }
  if (p.stats) {
    // the 16 lanes of a row hold the same 16 channels for 16 voxels: reduce
    // within rows by DPP, the two rows of a half-wave by a swap, then across
    // the two voxel-group waves in LDS
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ssum[i] = row16_sum(ssum[i]);
      ssq[i] = row16_sum(ssq[i]);
      ssum[i] += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, ssum[i]), 0x401F));
      ssq[i] += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, ssq[i]), 0x401F));
    }
    float* R = reinterpret_cast<float*>(smem + V4Cfg::pad(wv));  // this wave's [hh][16 sums | 16 squares]
    if (lr == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        R[hh * 32 + i] = ssum[i];
        R[hh * 32 + 16 + i] = ssq[i];
      }
    }
    // LDS-only exchange: wait for the LDS writes, not for the output stores
    // (__syncthreads' fence would drain them: vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (CT32 ? tid < 32 : tid < 64) {
      const int ff = tid >> 5, c32 = tid & 31;
      // channel c32 of the wave's slice: accumulator layout (i = 4 j + k, half h2 ->
      // 8 j + 4 h2 + k), or GB's swapped layout (i = 8 jj + k -> 16 jj + 8 h2 + k)
      const int h2 = GB ? (c32 >> 3) & 1 : (c32 >> 2) & 1;
      const int i = GB ? 8 * (c32 >> 4) + (c32 & 7) : 4 * (c32 >> 3) + (c32 & 3);
      const int tiles = p.tx * p.ty * p.tz;
      float su, sq;
      if constexpr (CT32) {  // the 4 plane waves hold the same 32 channels
        su = 0.f; sq = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float* Rw = reinterpret_cast<const float*>(smem + V4Cfg::pad(w)) + h2 * 32;
          su += Rw[i];
          sq += Rw[16 + i];
        }
      } else {
        const float* R0 = reinterpret_cast<const float*>(smem + V4Cfg::pad(ff)) + h2 * 32;       // vg 0
        const float* R1 = reinterpret_cast<const float*>(smem + V4Cfg::pad(ff + 2)) + h2 * 32;   // vg 1
        su = R0[i] + R1[i];
        sq = R0[16 + i] + R1[16 + i];
      }
      const int c = (CT32 ? ct * 32 : ct * 64) + tid;
      if constexpr (GB) {
        // (sum dz, sum dz x) -> (sum dz, sum dz xhat) with xhat = (x - mu) rs of c's group
        const float* gm = reinterpret_cast<const float*>(smem + V4Cfg::gmr_off(gslot));   // [g - glo][mu, rs]
        const unsigned gi = fdiv((unsigned)c, p.gdiv) - fdiv((unsigned)(c - tid), p.gdiv);
        sq = gm[2 * gi + 1] * (sq - gm[2 * gi] * su);
      }
      const long long pidx = ((long long)b * tiles + sl) * p.cout + c;
      p.stats[pidx * 2 + 0] = su;
      p.stats[pidx * 2 + 1] = sq;
    }
  }
}

// Work item of a persistent workgroup: iteration it of workgroup blockIdx.x ->
// (batch b, spatial tile sl, channel tile ct, origin, K slice ks = chunks
// [c0, c1)) through the XCD-aware bijective map: the tiles an XCD runs are one
// contiguous run (x fastest; K slice slowest, so the tiles an XCD runs share
// their weight chunks).
struct V4Tile { int b, sl, ct, x0, y0, z0, ks, c0, c1; };
__device__ __forceinline__ V4Tile v4_tile_of(const V4Params& p, int it) {
  const int tiles = p.tx * p.ty * p.tz;
  const int nbase = p.nblk / p.ksplit;
  const int t = blockIdx.x + it * gridDim.x;
  const int xcd = t & 7, q8 = p.nblk >> 3, r8 = p.nblk & 7;
  int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (t >> 3);
  V4Tile r;
  r.ks = wg / nbase;
  wg -= r.ks * nbase;
  r.c0 = r.ks * p.kper;
  r.c1 = min(p.nch, r.c0 + p.kper);
  r.ct = wg % p.nct;
  const int st = wg / p.nct;
  r.b = st / tiles;
  r.sl = st - r.b * tiles;
  r.x0 = (r.sl % p.tx) * 32; r.y0 = ((r.sl / p.tx) % p.ty) * 4; r.z0 = (r.sl / (p.tx * p.ty)) * 4;
  // wave-uniform by construction; say so, or every buffer op gets a waterfall loop
  r.ct = __builtin_amdgcn_readfirstlane(r.ct); r.b = __builtin_amdgcn_readfirstlane(r.b);
  r.sl = __builtin_amdgcn_readfirstlane(r.sl); r.x0 = __builtin_amdgcn_readfirstlane(r.x0);
  r.y0 = __builtin_amdgcn_readfirstlane(r.y0); r.z0 = __builtin_amdgcn_readfirstlane(r.z0);
  r.ks = __builtin_amdgcn_readfirstlane(r.ks); r.c0 = __builtin_amdgcn_readfirstlane(r.c0);
  r.c1 = __builtin_amdgcn_readfirstlane(r.c1);
  return r;
}

// Halo pieces of chunk c of tile tt into the halo buffer at hb (LDS-DMA; wave wv
// issues pieces wv + 4 j).  Pieces wv + 4 j and wv + 4 (j + 5) cover the same
// voxel slots of the two quad planes, so 5 voxel indices serve all 10; -2 marks
// the padding slots (never written: bias / statistics scratch).  Recomputed per
// chunk (a few VALU per piece) rather than held in registers.
// PB: byte stride of the two quad planes (v4 / v5: the padded 1280 slots; the
// split-bf16 kernel packs them at 1224 slots -- the padding lanes never write)
// ALL: every lane issues its pieces, the slots past the halo (helper 3's last piece) from an
// out-of-range offset (zeros into the padding): a fixed count of vector-memory ops per chunk
template <typename T, int MODE, int PB = V4Cfg::HVP * 16, bool ALL = false>
__device__ __forceinline__ void v4_issue_halo(const V4Params& p, const V4Tile& tt, int c, unsigned char* hb, int wv,
                                              int lane) {
  using C = V4Cfg;
  constexpr int CK = ConvTr<T>::CK;
  constexpr int ESZ = sizeof(T);
  const int SH = MODE == 1 ? p.H >> 1 : p.H, SW = MODE == 1 ? p.W >> 1 : p.W;
  int svox[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int hv = (wv + 4 * j) * 64 + lane;
    int sv = -2;
    if (hv < C::HV) {
      sv = -1;
      const int hx = hv % C::HX, hy = (hv / C::HX) % C::HY, hz = hv / (C::HX * C::HY);
      int ox = tt.x0 + hx - 1, oy = tt.y0 + hy - 1, oz = tt.z0 + hz - 1;
      if (ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) {
        if (MODE == 1) { ox >>= 1; oy >>= 1; oz >>= 1; }
        sv = (oz * SH + oy) * SW + ox;
      }
    }
    svox[j] = sv;
  }
  const bool s0 = c < p.nch0;
  const unsigned char* base = s0 ? reinterpret_cast<const unsigned char*>(p.a0) + (long long)tt.b * p.a0_bstride
                                 : reinterpret_cast<const unsigned char*>(p.a1) + (long long)tt.b * p.a1_bstride;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(s0 ? p.a0_bytes : p.a1_bytes), 0x00020000);
  const int cs = s0 ? p.ac0 : p.ac1;
  const int cb = (s0 ? c : c - p.nch0) * CK;
  // byte offset of (voxel sv, quad qd) = sv * rowb + cofs + 16 qd
  const bool cm = s0 && p.a0_cm;
  const unsigned rowb = cm ? 32u : (unsigned)cs * ESZ;
  const unsigned cofs = cm ? (unsigned)c * (unsigned)p.a0_cvox * 32u : (unsigned)(cb * ESZ);
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const int pc = wv + 4 * j;
    const int sv = svox[j % 5];
    const unsigned voff = sv >= 0 ? (unsigned)sv * rowb + cofs + (unsigned)((j / 5) * 16) : 0xFFFFFFF0u;
    if (ALL || sv != -2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(hb + (PB == 20 * 1024 ? pc * 1024 : (pc / 20) * PB + (pc % 20) * 1024)),
          16, voff, 0, 0, 0);
  }
}

// Persistent: gridDim.x <= the number of tiles; workgroup k runs tiles
// k, k + gridDim.x, ... as one continuous chunk stream, so the next tile's halo,
// weights and bias are prefetched under the current tile's last chunk.
// GB: the dgrad instance with the fused GroupNorm-backward reduce (V4Params::gx0)
template <typename T, int MODE, bool FAST, bool CT32 = false, bool GB = false>
__global__ void __launch_bounds__(256, 2) conv3d_v4_kernel(V4Params p) {
  static_assert(!FAST || sizeof(T) == 2, "the fast epilogue is 16-bit (bf16 / fp16) only");
  using C = V4Cfg;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[C::SMEM];

  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, hh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int f = wv & 1, vg = wv >> 1;
  // CT32: one z-plane per wave, the tile's 32 channels (the 64-row weight tile
  // ct >> 1, rows 32 (ct & 1) + lr); else planes 2 vg, 2 vg + 1 and channels f 32 + lr
  constexpr int NPL = CT32 ? 1 : 2;
  const int zb = CT32 ? wv : 2 * vg;
  V4_STAMP(0);
#ifdef CWDM_CONV_STAMPS
  if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 24 + 20] = __builtin_amdgcn_s_memrealtime();
  if (p.stamps && tid == 0) {
    p.stamps[(long long)blockIdx.x * 24 + 22] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
    p.stamps[(long long)blockIdx.x * 24 + 23] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
  }
#endif

  // The two workgroups that share a CU would run in lockstep and hit their
  // epilogues (VALU + stores, no MFMA) together.  The second one to arrive on
  // a CU starts half a tile late, so each epilogue runs beside the partner's
  // MFMAs.  (Arrival order per CU from a monotonic counter: every launch adds
  // two arrivals per CU, so the parity needs no reset.)
  if (p.stagger_cycles > 0) {
    unsigned* slot = reinterpret_cast<unsigned*>(smem + V4Cfg::pad(0) + 512);
    if (tid == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
      *slot = atomicAdd(&g_v4_cu_arrivals[((xcc & 7) << 8) | ((hw >> 8) & 0xFF)], 1u) & 1u;
    }
    __syncthreads();
    if (*slot) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      while (__builtin_amdgcn_s_memtime() - t0 < (unsigned long long)p.stagger_cycles) __builtin_amdgcn_s_sleep(32);
    }
    __syncthreads();
  }
  const int nblk = p.nblk;
  using Tile = V4Tile;
  auto tile_of = [&](int it) { return v4_tile_of(p, it); };
  const int ntile = (nblk - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;

  auto issue_halo = [&](const Tile& tt, int c, int hbuf) {
    v4_issue_halo<T, MODE>(p, tt, c, smem + hbuf * C::HALO_B, wv, lane);
  };
  // weight fragments of group g of chunk c, channel tile ct: the 3 dy taps, this
  // lane's row (output channel) lr of the wave's 32-channel slice, quad hh
  const unsigned char* wlane = p.aw + (CT32 ? 0 : f * 1024) + lr * 32 + ((hh ^ ((lr >> 3) & 1)) << 4);
  auto wtile = [&](int ct, int c) {  // this lane's weights of chunk c, channel tile ct
    return CT32 ? wlane + (ct & 1) * 1024 + ((long long)(ct >> 1) * p.nch + c) * 27 * 2048
                : wlane + ((long long)ct * p.nch + c) * 27 * 2048;
  };
  auto load_w = [&](u32x4 (&w)[3], int ct, int c, int g) {
    const unsigned char* src = wtile(ct, c) + ((g / 3) * 9 + (g % 3)) * 2048;
    v4_gload(w[0], src);
    v4_gload(w[1], src + 3 * 2048);
    v4_gload(w[2], src + 6 * 2048);
  };
  // the 64 bias values of a tile into this wave's LDS padding slice (one 4-byte DMA per lane)
  auto issue_bias = [&](const Tile& tt) {
    if (p.bias && wv == 0 && (!CT32 || lane < 32))
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(
                                           p.bias + (long long)tt.b * p.bias_bs + tt.ct * (CT32 ? 32 : 64) + lane),
                                       (__attribute__((address_space(3))) void*)(smem + C::pad(0) + 256), 4, 0, 0);
  };
  // fused GroupNorm backward: the tile's scale / shift and its groups' mean /
  // rstd into slot s of the LDS padding (wave 1, 4-byte DMA per lane)
  auto issue_gcoef = [&](const Tile& tt, int s) {
    if (!GB || wv != 1) return;
    const int nc = CT32 ? 32 : 64, tb = tt.ct * nc;
    const float* gsrc = p.gss + ((long long)tt.b * p.cout + tb) * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (64 * j + lane < 2 * nc)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(gsrc + 64 * j + lane),
                                         (__attribute__((address_space(3))) void*)(smem + C::gss_off(s) + 256 * j), 4,
                                         0, 0);
    const unsigned glo = fdiv((unsigned)tb, p.gdiv), ghi = fdiv((unsigned)(tb + nc - 1), p.gdiv);
    const int nf = 2 * (int)(ghi - glo + 1);   // <= 64 floats (the host requires C / G >= 2)
    const float* msrc = p.gmr + ((long long)tt.b * p.ggroups + glo) * 2;
    if (lane < nf)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(msrc + lane),
                                       (__attribute__((address_space(3))) void*)(smem + C::gmr_off(s)), 4, 0, 0);
  };
  // accumulators start at the bias of their output channel (i = 4 j + k -> channel 8 j + 4 hh + k)
  f32x16 acc[2][4];
  auto init_acc = [&](int ks) {
    float bia[16];
    const float* bl = reinterpret_cast<const float*>(smem + C::pad(0) + 256) + (CT32 ? 0 : f * 32) + 4 * hh;
#pragma unroll
    for (int i = 0; i < 16; ++i) bia[i] = (p.bias && ks == 0) ? bl[8 * (i >> 2) + (i & 3)] : 0.f;
#pragma unroll
    for (int a = 0; a < NPL; ++a)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][m][i] = bia[i];
  };

  // lane read base: halo voxel (z = 2 vg, line 0, x = lr) of quad plane hh
  const int hlane = hh * (C::HVP * 16) + (zb * (C::HX * C::HY) + lr) * 16;

  // a tile's first weight group: ordinary (compiler-tracked) loads, issued
  // before the previous tile's epilogue so their latency hides under it
  auto load_w0 = [&](u32x4 (&w)[3], int ct, int c) {
    const unsigned char* src = wtile(ct, c);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) w[dy] = *reinterpret_cast<const u32x4*>(src + dy * 3 * 2048);
  };
  Tile cur = tile_of(0);
  u32x4 wr[3][3];
  issue_bias(cur);
  issue_gcoef(cur, 0);
  issue_halo(cur, cur.c0, 0);
  load_w0(wr[0], cur.ct, cur.c0);
  int gch = 0;  // chunk counter of the stream (selects the halo buffer)
  for (int it = 0; it < ntile; ++it) {
    const bool more = it + 1 < ntile;
    // the tile's halo, bias and first weight group were issued under the previous tile (or above)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[0][2])::"memory");
    __builtin_amdgcn_s_barrier();
    if (it == 0) V4_STAMP(1);
    init_acc(cur.ks);
    // one chunk: 18 steps, step K = (group K / 2, plane K % 2).  The 6 halo
    // lines of step K + 1 are read before the 12 MFMAs of step K (software
    // pipeline, pinned by sched_barrier), so every MFMA block finds its
    // operands already in registers.  LAST: the tile's last chunk; the next
    // tile's chunk 0 (halo, bias) is issued after its MFMAs and lands under the
    // epilogue.
    auto chunk = [&](auto lastc, int c) {
      constexpr bool LAST = decltype(lastc)::value;
      const unsigned char* hb = smem + (gch & 1) * C::HALO_B + hlane;
      constexpr bool has_next = !LAST;
      u32x4 av[2][6];
      v4_read_step<0>(av[0], hb);
#define V4_STEP(K)                                                                                            \
      if constexpr (!CT32 || (K) % 2 == 0) {                                                                  \
        constexpr int GI = (K) / 2, PL = (K) % 2;                                                             \
        constexpr int KN = CT32 ? (K) + 2 : (K) + 1;       /* next step */                                    \
        constexpr int BC = CT32 ? ((K) / 2) & 1 : (K) & 1; /* its operand buffer; next: BC ^ 1 */             \
        if (PL == 0) {                                                                                        \
          /* weights of group GI + 1: this chunk or the next.  Nothing past the tile's last */                \
          /* group: a load nobody waits for would land in registers the epilogue reuses */                    \
          if (GI + 1 < 9) load_w(wr[(GI + 1) % 3], cur.ct, c, GI + 1);                                        \
          else if (!LAST) load_w(wr[(GI + 1) % 3], cur.ct, c + 1, 0);                                         \
          if (GI == V4_HALO_GI && has_next) issue_halo(cur, c + 1, (gch + 1) & 1);                            \
        }                                                                                                     \
        if (KN < 18) v4_read_step<KN % 18>(av[BC ^ 1], hb);                                                   \
        /* W(G) is retired with the younger weight group (and at group 2 the next */                          \
        /* chunk's halo pieces) still in flight; W(0) landed before the chunk */                              \
        /* (the halo's 10 pieces are younger than W(GI) at groups V4_HALO_GI and V4_HALO_GI + 1) */           \
        if (PL == 0 && GI >= 1 && (GI < 8 || !LAST)) {                                                        \
          if (has_next && (GI == V4_HALO_GI || GI == V4_HALO_GI + 1)) V4_WAIT_W(13, wr[GI % 3]);              \
          else V4_WAIT_W(3, wr[GI % 3]);                                                                      \
        }                                                                                                     \
        if (PL == 0 && GI == 8 && LAST) V4_WAIT_W(0, wr[2]);  /* nothing younger in flight */                 \
        __builtin_amdgcn_sched_barrier(0);                                                                    \
        _Pragma("unroll") for (int dy = 0; dy < 3; ++dy)                                                      \
        _Pragma("unroll") for (int m = 0; m < 4; ++m)                                                         \
          v4_mfma<T>(acc[PL][m], wr[GI % 3][dy], av[BC][m + dy]);                                             \
        __builtin_amdgcn_sched_barrier(0);                                                                    \
      }
      V4_STEP(0) V4_STEP(1) V4_STEP(2) V4_STEP(3) V4_STEP(4) V4_STEP(5)
      V4_STEP(6) V4_STEP(7) V4_STEP(8) V4_STEP(9) V4_STEP(10) V4_STEP(11)
      V4_STEP(12) V4_STEP(13) V4_STEP(14) V4_STEP(15) V4_STEP(16) V4_STEP(17)
#undef V4_STEP
      if constexpr (!LAST) {
        // the next chunk's halo and its first weight group (issued at group 8)
        // must have landed; then every wave is past this chunk's reads of the
        // buffer the following chunk's halo will overwrite
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[0][2])::"memory");
        __builtin_amdgcn_s_barrier();
      } else if (more) {
        // next tile's chunk 0 into the other buffer (last read by chunk gch - 1,
        // which every wave finished before the previous barrier)
        const Tile nxt = tile_of(it + 1);
        issue_bias(nxt);
        issue_gcoef(nxt, (it + 1) & 1);
        issue_halo(nxt, nxt.c0, (gch + 1) & 1);
      }
      if (it == 0 && c - cur.c0 < 8) V4_STAMP(4 + c - cur.c0);
      ++gch;
    };
    for (int c = cur.c0; c + 1 < cur.c1; ++c) chunk(std::false_type{}, c);
    chunk(std::true_type{}, cur.c1 - 1);
    if (it == 0) V4_STAMP(12);
    Tile nxt = cur;
    if (more) {
      nxt = tile_of(it + 1);
      // (GB: after the epilogue -- its x rows and GroupNorm sums need the registers)
      if constexpr (!GB) load_w0(wr[0], nxt.ct, nxt.c0);
    }
    // (K split: out is this slice's fp32 partial, see V4Params)
    v4_epilogue<T, FAST, CT32, GB>(p, acc, cur.b, cur.sl, cur.ct, cur.x0, cur.y0, cur.z0, cur.ks, tid, wv, smem, it & 1);
    if constexpr (GB) if (more) load_w0(wr[0], nxt.ct, nxt.c0);
    if (it == 0) V4_STAMP(13);
    cur = nxt;
  }
  V4_STAMP(15);
#ifdef CWDM_CONV_STAMPS
  if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 24 + 21] = __builtin_amdgcn_s_memrealtime();
#endif
}

}  // namespace cwdm
