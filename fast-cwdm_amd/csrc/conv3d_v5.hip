// Conv3d 3x3x3 (stride 1, pad 1) implicit GEMM with the consumer's GroupNorm +
// SiLU applied in LDS: the warp-specialised DMA conv for the wide U-Net levels
// (16-bit, W >= 24, H % 4 == 0, D % 4 == 0, cout % 64 == 0, no K split).
//
// Why: the DMA conv of conv3d_v4.hpp stages an ALREADY activated input, so
// every GroupNorm+SiLU'd conv input was written once and read back once by a
// streaming pre-pass (cwdm_gn_apply: ~12 GB and 2.5 ms of a 128^3 bf16 step);
// and its epilogue (residual loads, 64 KB of stores per tile) runs on the MFMA
// waves.  Doing the transform on the MFMA waves instead cost more than the pass
// (r02, DESIGN.md §3: the halo is 2.4x the tile and the SIMDs are MFMA-bound).
//
// Design (MI355X / gfx950), one 512-thread workgroup per CU, persistent:
//   * waves 0-3 ("MFMA waves", s_setprio 2) run exactly v4's MFMA schedule on
//     a 32(x) x 4(y) x 4(z) x 64-channel tile: 8 accumulators of 32 ch x 32 vox
//     per wave, 216 v_mfma_f32_32x32x16 per 16-channel chunk, weights straight
//     to VGPRs two groups ahead.  They issue no halo DMA, no VALU epilogue and
//     no global store;
//   * waves 4-7 ("helper waves", one per SIMD beside an MFMA wave) own the
//     data movement: per chunk k they issue the halo DMA of chunk k + 2 (and
//     the chunk's 16 GroupNorm (scale, shift) pairs), wait for their OWN pieces
//     of chunk k + 1, and apply SiLU(x sc + sh) to them in place (zero padding
//     stays zero); the VALU issue slots an MFMA leaves free (24 of 32 cycles)
//     absorb it.  Three 40 KB halo buffers rotate: read (k), transform (k + 1),
//     DMA (k + 2).  One s_barrier per chunk for all 8 waves.
//   * tile hand-off: after a tile's last chunk the MFMA waves write their
//     accumulators as 16-bit values into LDS (rows = voxels, 128 B, 16-B column
//     XOR row & 7: conflict-free) -- z-planes 0-1 into the halo buffer they just
//     finished, planes 2-3 into a spare 32 KB -- and go straight on with the
//     next tile.  During the next tile's first chunk the helpers drain it:
//     + residual (prefetched a tile earlier into registers), per-channel
//     (sum, sum^2) GroupNorm partials, 16-byte stores of whole 128-B rows.
//     Helper h drains exactly the 1 KB blocks of the staging buffer that its
//     own halo DMA of chunk k + 2 overwrites next, so no helper waits on
//     another.  Partials reduce across the 4 helpers in a fixed order through
//     LDS (deterministic).
// The output is rounded to 16 bits before the residual add (v4 adds in fp32
// and rounds once); without a residual the output is bit-identical to v4 on a
// cwdm_gn_apply'd input.
#include <atomic>
#include <cstdlib>

#include "conv3d_v4.hpp"

namespace cwdm {

struct V5Cfg {
  static constexpr int HALO_B = V4Cfg::HALO_B;          // 40960: one halo buffer (2 quad planes x 1280 slots x 16 B)
  static constexpr int STG1 = 3 * HALO_B;               // staging rows 256..511 (z-planes 2, 3): 32 KB
  static constexpr int BIAS = STG1 + 32768;             // bias of tile parity s at + 256 s (64 fp32)
  static constexpr int SCR = BIAS + 512;                // statistics partials [4 helper][64 ch][2] fp32
  static constexpr int GSS = SCR + 2048;                // GroupNorm (sc, sh) [3 buffers][4 helpers][16 ch][2] fp32
  static constexpr int CNT = GSS + 1536;                // statistics arrival counters
  static constexpr int RUN = CNT + 256;                 // per-workgroup statistics (stats_wg): [2 ch tiles][64][2] fp32
  static constexpr int SMEM = RUN + 1024;               // 163072 of the CU's 163840
};
static_assert(V5Cfg::SMEM <= 163840, "v5 LDS");

// diagnostics build (make STAMPS=1, tools/v5_stamps.py): per workgroup 64 u64 s_memtime stamps --
// [0] start, [1] MFMA waves past B0, [2 + k] MFMA wave 0 at chunk k's barrier, [18 + k] released from it,
// [34 + k] helper 0 at chunk k's barrier (k < 16), [50] / [51] s_memrealtime at start / end of MFMA wave 0,
// [52] end of helper 0, [53] HW_ID, [54] XCC_ID
// timing-only diagnostics build (make V5DIAG=1; the results are garbage): env CWDM_V5_DIAGMASK bits
// 1 helpers issue no halo DMA, 2 MFMA waves read no LDS operands, 4 MFMA waves load no weights,
// 8 the in-LDS GroupNorm transform without its SiLU math (load + store only), 16 no transform at all,
// 32 helpers drain nothing (no stores / statistics)
#ifdef CWDM_V5_DIAG
#define V5_DIAG(bit) ((p.diag & (bit)) != 0)
#else
#define V5_DIAG(bit) false
#endif
// bit 64: each tile runs its K chunks rotated by its spatial index (the same sum in another order), so
// neighbouring CUs ask for different weight chunks at the same time
#define V5_PHYS(t, c) (V5_DIAG(64) ? (t).c0 + ((c) - (t).c0 + (t).sl) % ((t).c1 - (t).c0) : (c))

#ifdef CWDM_CONV_STAMPS
#define V5_STAMP(k, cond)                                                                        \
  do {                                                                                           \
    if (p.stamps && (cond)) p.stamps[(long long)blockIdx.x * 64 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define V5_STAMP(k, cond) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// Apply-ahead (AA > 0): the GroupNorm + SiLU of the input without a pre-pass
// over HBM and without transforming every halo voxel 2.4x in LDS.  The
// persistent grid sweeps the work items in order -- iteration it runs items
// [it G, (it + 1) G), G = gridDim.x (XCD x the contiguous eighth x of each
// block) -- so the voxels iteration it reads are a prefix [0, need(it)) of the
// source: through the top halo plane of its last tile.  Each workgroup's
// helper waves transform 1/G of range R(r) = [need(r - 1), need(r)) during
// iteration r - L (L = aa_lead), once per voxel, from the raw channels-last
// source into the chunk-major copy the halo DMA reads (written through to
// memory: sc1); a counter per range collects the G workgroups' completions,
// and a helper waits on R(it)'s counter before it issues tile it's first
// DMA.  R(0 .. L - 1) is transformed by all eight waves before the first tile
// (the one grid-wide wait).  Batch 1, same-grid sources.
// Counters: per launch (p.aa_cnt: the U-Net plan's sync block, zeroed once per
// forward, or a lone launch's workspace tail, zeroed by a memset node before
// it), so launches on other streams never share them; the workgroup that exits
// last re-zeroes them for the plan's next AA launch.
// Visibility (MI355X_MICROARCH.md, inter-workgroup visibility, Valid forms):
// the transformed bytes are stored write-through (sc1: they leave the writer's
// L2), every storing wave drains them (s_waitcnt vmcnt(0)) before the
// workgroup barrier behind which ONE lane adds to the range counter (agent
// scope); the reader polls that counter with agent-scope (sc1) loads.  The
// reader's halo LDS-DMA is not an sc1 load, and no acquire fence follows the
// poll (an agent acquire only invalidates this CU's L1: ~1.7 us per tile; an
// agent release on the writer would write back the XCD's dirty L2 per range):
// what makes a plain load safe here is that no CU reads a byte of range r + 1
// before r + 1 is published -- the sweep reads prefixes of the source, range
// boundaries fall on whole z planes (H W voxels x 32 B: 128-B aligned), and L1 /
// L2 hold nothing of the copy from earlier launches (kernel boundaries write
// back and invalidate) -- so neither cache can hold a stale line of it.
// Residency: every wait needs all G workgroups resident at once; G <= the CUs
// x the instance's occupancy (v5_aa_grid).  A wait that still runs out (CUs
// held by another process, CU masking) sets CWDM_DEV_E_AA_TIMEOUT in the
// device error word (cwdm_device_status) instead of failing silently.
// ---------------------------------------------------------------------------
constexpr int kV5AaCnt = kV5AaWords;           // [0] the prologue ranges, [r] range r, [kV5AaCnt - 1] exits
__device__ unsigned g_cwdm_dev_err;            // sticky CWDM_DEV_E_* bits (cwdm_device_status)

// bounded wait for `need` arrivals on counter c (agent-scope sc1 polls); false (and the
// device error word set) when the bound runs out
__device__ __forceinline__ bool v5aa_wait(unsigned* c, unsigned need, int spin, int sleep2) {
  for (int n = 0; __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need; ++n) {
    if (n >= spin) {
      __hip_atomic_fetch_or(&g_cwdm_dev_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if (sleep2) __builtin_amdgcn_s_sleep(2);
    else __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");   // nothing that reads the range is hoisted above the poll
  return true;
}

__device__ __forceinline__ int v5aa_pos() {
  const int G = gridDim.x;
  const int b = blockIdx.x;
  return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
}
__device__ __forceinline__ V4Tile v5aa_tile_of(const V4Params& p, int it) {
  const int wg = it * (int)gridDim.x + v5aa_pos();
  V4Tile r;
  r.ks = 0; r.c0 = 0; r.c1 = p.nch; r.b = 0;
  r.ct = wg % p.nct;
  r.sl = wg / p.nct;
  r.x0 = (r.sl % p.tx) * 32; r.y0 = ((r.sl / p.tx) % p.ty) * 4; r.z0 = (r.sl / (p.tx * p.ty)) * 4;
  r.ct = __builtin_amdgcn_readfirstlane(r.ct); r.sl = __builtin_amdgcn_readfirstlane(r.sl);
  r.x0 = __builtin_amdgcn_readfirstlane(r.x0); r.y0 = __builtin_amdgcn_readfirstlane(r.y0);
  r.z0 = __builtin_amdgcn_readfirstlane(r.z0);
  return r;
}
// need(j): source voxels the tiles of sweep iterations <= j read (0 for j < 0)
__host__ __device__ __forceinline__ unsigned v5aa_need(int j, int G, int nblk, int nct, int tx, int ty, int D, int H,
                                                       int W) {
  if (j < 0) return 0u;
  long long w = (long long)(j + 1) * G;
  if (w > nblk) w = nblk;
  const int st = (int)(w - 1) / nct;
  const int z1 = (st / (tx * ty)) * 4 + 5;
  return (unsigned)(z1 < D ? z1 : D) * (unsigned)H * (unsigned)W;
}

template <typename T, int MODE, bool GN, int AA = 0>
__global__ void __launch_bounds__(512) conv3d_v5_kernel(V4Params p) {
  using C = V4Cfg;
  using T16 = T;
  constexpr int NI = 10 + (GN ? 1 : 0);   // VMEM instructions per chunk of one helper wave
  __shared__ __attribute__((aligned(1024))) unsigned char smem[V5Cfg::SMEM];

  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, hh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = p.nblk;
  const int ntile = (nblk - (AA ? v5aa_pos() : (int)blockIdx.x) + (int)gridDim.x - 1) / (int)gridDim.x;
  if (ntile <= 0) return;
  auto tile_of = [&](int it) { return AA ? v5aa_tile_of(p, it) : v4_tile_of(p, it); };
  const int tiles = p.tx * p.ty * p.tz;

  // apply-ahead: this thread's lane slot among nslot cooperating lanes -- quad q (8 channels) of
  // voxel offset vo within each step of vps voxels; the 8 channels' SiLU coefficients
  const int G = (int)gridDim.x;
  const unsigned V = (unsigned)p.D * (unsigned)p.H * (unsigned)p.W;
  struct AaLane { const unsigned char* src; unsigned rowb, oq; int vo, vps; bool on; float a[8], b[8]; };
  auto aa_lane = [&](int slot, int nslot) {
    AaLane l{};
    if constexpr (AA > 0) {
      const int Q = (p.axc0 + p.axc1) >> 3, q0 = p.axc0 >> 3;
      l.vps = nslot / Q;
      l.on = slot < l.vps * Q;
      const int q = l.on ? slot % Q : 0;
      l.vo = l.on ? slot / Q : 0;
      l.src = q < q0 ? reinterpret_cast<const unsigned char*>(p.ax0) + q * 16
                     : reinterpret_cast<const unsigned char*>(p.ax1) + (q - q0) * 16;
      l.rowb = (unsigned)(q < q0 ? p.axc0 : p.axc1) * 2u;
      l.oq = (unsigned)(q >> 1) * V * 32u + (unsigned)(q & 1) * 16u;
#pragma unroll
      for (int e = 0; e < 8; ++e) silu_aff_coef(p.agn[(q * 8 + e) * 2], p.agn[(q * 8 + e) * 2 + 1], l.a[e], l.b[e]);
    } else {
      (void)slot; (void)nslot;
    }
    return l;
  };
  const __amdgpu_buffer_rsrc_t ract = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.a0), (short)0, (int)(AA ? V * (unsigned)(p.axc0 + p.axc1) * 2u : 0u), 0x00020000);
  auto aa_load = [&](const AaLane& l, unsigned v, bool ok) -> u32x4 {
    // a global (not flat) load: flat ops count in lgkmcnt too, which the barrier waits drain
    return *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(
        (const __attribute__((address_space(1))) unsigned char*)(l.src) + (size_t)(ok ? v : 0u) * l.rowb);
  };
  auto aa_store = [&](const AaLane& l, const u32x4& x, unsigned v, bool ok) {
    float xv[8], y[8];
    unpack<T>(x, xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = silu_aff(xv[e], l.a[e], l.b[e]);
    // written through to memory (sc1): read by other XCDs' halo DMA after the range counter
    __builtin_amdgcn_raw_buffer_store_b128(pack<T>(y), ract, ok ? l.oq + v * 32u : 0xFFFFFFF0u, 0, 16);
  };
  // piece [lo, hi) of this workgroup in range [r0, r1)
  auto aa_piece = [&](unsigned r0, unsigned r1, unsigned& lo, unsigned& hi) {
    const int pos = v5aa_pos();
    lo = r0 + (unsigned)((unsigned long long)(r1 - r0) * (unsigned)pos / (unsigned)G);
    hi = r0 + (unsigned)((unsigned long long)(r1 - r0) * (unsigned)(pos + 1) / (unsigned)G);
  };
  auto aa_need = [&](int j) { return v5aa_need(j, G, nblk, p.nct, p.tx, p.ty, p.D, p.H, p.W); };
  const int aa_nit = (nblk + G - 1) / G;
  if constexpr (AA > 0) {
    V5_STAMP(55, tid == 0);
    // ranges 0 .. L - 1 by all eight waves, then the grid-wide wait for them
    const AaLane l = aa_lane(tid, 512);
    unsigned lo, hi;
    aa_piece(0u, aa_need(p.aa_lead - 1), lo, hi);
    const int nst = l.vps > 0 ? (int)((hi - lo + (unsigned)l.vps - 1) / (unsigned)l.vps) : 0;
    for (int s0 = 0; s0 < nst; s0 += 4) {
      u32x4 x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned v = lo + (unsigned)((s0 + k) * l.vps + l.vo);
        x[k] = aa_load(l, v, l.on && v < hi);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned v = lo + (unsigned)((s0 + k) * l.vps + l.vo);
        aa_store(l, x[k], v, l.on && v < hi);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(&p.aa_cnt[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v5aa_wait(&p.aa_cnt[0], (unsigned)(G + p.aa_extra), p.aa_spin, 1);
    }
    __syncthreads();
  }

  V5_STAMP(0, tid == 0);
#ifdef CWDM_CONV_STAMPS
  if (p.stamps && tid == 0) {
    p.stamps[(long long)blockIdx.x * 64 + 50] = __builtin_amdgcn_s_memrealtime();
    p.stamps[(long long)blockIdx.x * 64 + 53] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    p.stamps[(long long)blockIdx.x * 64 + 54] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
  }
#endif
  if (wv < 4) {
    // ------------------------------------------------------------ MFMA waves
    __builtin_amdgcn_s_setprio(2);
    const int f = wv & 1, vg = wv >> 1, zb = 2 * vg;
    const unsigned char* wlane = p.aw + f * 1024 + lr * 32 + ((hh ^ ((lr >> 3) & 1)) << 4);
    auto load_w = [&](u32x4 (&w)[3], int ct, int c, int g) {
      if (V5_DIAG(4)) return;
      const unsigned char* src = wlane + ((long long)ct * p.nch + c) * 27 * 2048 + ((g / 3) * 9 + (g % 3)) * 2048;
      v4_gload(w[0], src);
      v4_gload(w[1], src + 3 * 2048);
      v4_gload(w[2], src + 6 * 2048);
    };
    const int hlane = hh * (C::HVP * 16) + (zb * (C::HX * C::HY) + lr) * 16;
    f32x16 acc[2][4];
    u32x4 wr[3][3];
    V4Tile cur = tile_of(0);
    load_w(wr[0], cur.ct, V5_PHYS(cur, cur.c0), 0);
    load_w(wr[1], cur.ct, V5_PHYS(cur, cur.c0), 1);
    __builtin_amdgcn_s_barrier();   // B0: chunk 0 transformed, bias 0 landed
    V5_STAMP(1, tid == 0);
    int gch = 0;
    for (int it = 0; it < ntile; ++it) {
      const bool more = it + 1 < ntile;
      const V4Tile nxt = more ? tile_of(it + 1) : cur;
      {
        float bia[16];
        const float* bl = reinterpret_cast<const float*>(smem + V5Cfg::BIAS + (it & 1) * 256) + f * 32 + 4 * hh;
#pragma unroll
        for (int i = 0; i < 16; ++i) bia[i] = p.bias ? bl[8 * (i >> 2) + (i & 3)] : 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][m][i] = bia[i];
      }
      auto chunk = [&](auto lastc, int c) {
        constexpr bool LAST = decltype(lastc)::value;
        const unsigned char* hb = smem + (gch % 3) * C::HALO_B + hlane;
        u32x4 av[2][6];
        if (!V5_DIAG(2)) v4_read_step<0>(av[0], hb);
#define V5_STEP(K)                                                                                           \
        {                                                                                                    \
          constexpr int GI = (K) / 2, PL = (K) % 2, KN = (K) + 1, BC = (K) & 1;                              \
          /* straight-line loads and counted waits only: a runtime branch between an asm load and its  */ \
          /* wait lets the register allocator copy the destination before the data lands (the last tile */ \
          /* reloads its own first group instead of skipping the load: nxt == cur there)               */ \
          /* weights two groups ahead (one MFMA wave per SIMD: nothing else hides an L2 round trip) */   \
          if (PL == 0) {                                                                                     \
            if (GI + 2 < 9) load_w(wr[(GI + 2) % 3], cur.ct, V5_PHYS(cur, c), GI + 2);                       \
            else if (!LAST) load_w(wr[(GI + 2) % 3], cur.ct, V5_PHYS(cur, c + 1), GI - 7);                   \
            else load_w(wr[(GI + 2) % 3], nxt.ct, V5_PHYS(nxt, nxt.c0), GI - 7);                             \
          }                                                                                                  \
          if (KN < 18 && !V5_DIAG(2)) v4_read_step<KN % 18>(av[BC ^ 1], hb);                                 \
          if (PL == 0) V4_WAIT_W(6, wr[GI % 3]);                                                             \
          __builtin_amdgcn_sched_barrier(0);                                                                 \
          _Pragma("unroll") for (int dy = 0; dy < 3; ++dy)                                                   \
          _Pragma("unroll") for (int m = 0; m < 4; ++m)                                                      \
            v4_mfma<T>(acc[PL][m], wr[GI % 3][dy], av[BC][m + dy]);                                          \
          __builtin_amdgcn_sched_barrier(0);                                                                 \
        }
        V5_STEP(0) V5_STEP(1) V5_STEP(2) V5_STEP(3) V5_STEP(4) V5_STEP(5)
        V5_STEP(6) V5_STEP(7) V5_STEP(8) V5_STEP(9) V5_STEP(10) V5_STEP(11)
        V5_STEP(12) V5_STEP(13) V5_STEP(14) V5_STEP(15) V5_STEP(16) V5_STEP(17)
#undef V5_STEP
        V5_STAMP(2 + gch, tid == 0 && gch < 16);
        __builtin_amdgcn_s_barrier();   // chunk k read; chunk k + 1 transformed
        V5_STAMP(18 + gch, tid == 0 && gch < 16);
        ++gch;
      };
      for (int c = cur.c0; c + 1 < cur.c1; ++c) chunk(std::false_type{}, c);
      chunk(std::true_type{}, cur.c1 - 1);
      // hand the tile to the helpers: 16-bit rows, planes 2 vg, 2 vg + 1 -> staging half vg
      unsigned char* st = smem + (vg == 0 ? ((gch + 2) % 3) * C::HALO_B : V5Cfg::STG1);
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int m = 0; m < 4; ++m)
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
            const int row = pl * 128 + m * 32 + lr;
            const int q = 4 * f + 2 * jj + hh;
            *reinterpret_cast<u32x4*>(st + row * 128 + ((q ^ (lr & 7)) << 4)) = w;
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // B2: tile staged
      cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[0][2]), "+v"(wr[1][0]), "+v"(wr[1][1]),
                 "+v"(wr[1][2])::"memory");   // the dummy reloads of the last tile
#ifdef CWDM_CONV_STAMPS
    if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 64 + 51] = __builtin_amdgcn_s_memrealtime();
#endif
    return;
  }

  // -------------------------------------------------------------- helper waves
  const int h = wv - 4;
  const int r8 = lane >> 3, q = lane & 7;
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + V5Cfg::CNT);   // statistics arrivals (monotonic)
  // chunk prefetch cursor (the next chunk to DMA)
  int pit = 0;
  V4Tile pt = tile_of(0);
  int pc = pt.c0;
  auto issue_next = [&](int buf) -> bool {
    if (pit >= ntile) return false;
    if (!V5_DIAG(1)) v4_issue_halo<T, MODE>(p, pt, V5_PHYS(pt, pc), smem + buf * C::HALO_B, h, lane);
    if constexpr (GN) {
      if (lane < 32)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(p.agn + ((long long)pt.b * (p.ac0 + p.ac1) +
                                                                      V5_PHYS(pt, pc) * 16) * 2 + lane),
            (__attribute__((address_space(3))) void*)(smem + V5Cfg::GSS + (buf * 4 + h) * 128), 4, 0, 0);
    }
    if (pc + 1 < pt.c1) ++pc;
    else if (++pit < ntile) { pt = tile_of(pit); pc = pt.c0; }
    return true;
  };
  // SiLU(x sc + sh) in place over this wave's pieces (voxel slots (h + 4 j) * 64 + lane, both
  // quad planes) of the chunk in buffer buf; slots outside the volume stay zero
  auto transform = [&](int x0, int y0, int z0, int buf) {
    if constexpr (GN) {
      if (V5_DIAG(16)) return;
      unsigned char* hb = smem + buf * C::HALO_B;
      const float* gs = reinterpret_cast<const float*>(smem + V5Cfg::GSS + (buf * 4 + h) * 128);
      u32x4 x[2][5];
#pragma unroll
      for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int qd = 0; qd < 2; ++qd)
          x[qd][j] = *reinterpret_cast<const u32x4*>(hb + qd * (C::HVP * 16) + ((h + 4 * j) * 64 + lane) * 16);
      float mk[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int hv = (h + 4 * j) * 64 + lane;
        const int hx = hv % C::HX, hy = (hv / C::HX) % C::HY, hz = hv / (C::HX * C::HY);
        const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
        mk[j] = (hv < C::HV && ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) ? 1.f : 0.f;
      }
      // interior tiles (the halo inside the volume: most of them) skip the masks
      const bool inner = x0 >= 1 && y0 >= 1 && z0 >= 1 && x0 + C::HX - 1 <= p.W && y0 + C::HY - 1 <= p.H &&
                         z0 + C::HZ - 1 <= p.D;
#pragma unroll
      for (int qd = 0; qd < 2; ++qd) {
        float sa[8], sb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) silu_aff_coef(gs[2 * (8 * qd + e)], gs[2 * (8 * qd + e) + 1], sa[e], sb[e]);
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          float xv[8], y[8];
          unpack<T>(x[qd][j], xv);
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = V5_DIAG(8) ? xv[e] : silu_aff(xv[e], sa[e], sb[e]);
          if (!inner) {
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] *= mk[j];
          }
          *reinterpret_cast<u32x4*>(hb + qd * (C::HVP * 16) + ((h + 4 * j) * 64 + lane) * 16) = pack<T>(y);
        }
      }
    } else {
      (void)x0; (void)y0; (void)z0; (void)buf;
    }
  };
  const long long HW = (long long)p.H * p.W, VV = (long long)p.D * HW;
  const unsigned rowb = (unsigned)p.W * (unsigned)p.cout * 2u, planeb = (unsigned)HW * (unsigned)p.cout * 2u;
  float s1[8], s2[8];   // this lane's statistics over both drain parts of a tile
  bool wg_final = false;   // stats_wg: the drain of this workgroup's last tile (writes the row)
  u32x4 dq[8];          // a drain slice's output rows and their byte offsets (drain -> drain_put)
  unsigned doff[8];
  // the residual rows of drain part `part` of tile tt (this lane's rows i = 8 part .. + 7): loaded
  // one chunk ahead of their drain (part 0 under the tile's last chunk, part 1 under part 0's
  // chunk), so their latency is not on the helper's path at the tile seam
  u32x4 rq[8];
  auto drain_load = [&](const V4Tile& tt, int part) {
    if (p.rmode < 0) return;
    const int ox = tt.x0 + 8 * h + r8;
    const bool xin = ox < p.W;
    const long long rV = p.rmode == 1 ? VV / 8 : VV;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const T16*>(p.res) + (long long)tt.b * rV * p.cout), (short)0,
        (int)(rV * p.cout * 2), 0x00020000);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = 8 * part + k;
      const int oy = tt.y0 + (i & 3), oz = tt.z0 + (i >> 2);
      unsigned rv = p.rmode == 1 ? (unsigned)(((oz >> 1) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1))
                                 : (unsigned)((oz * p.H + oy) * p.W + ox);
      rq[k] = __builtin_amdgcn_raw_buffer_load_b128(
          rr, xin ? rv * (unsigned)p.cout * 2u + (unsigned)(tt.ct * 64 + 8 * q) * 2u : 0xFFFFFFF0u, 0, 0);
    }
  };
  // drain rows k0 .. k1 - 1 of part `part` of staged tile tt: row k = voxel (x0 + 8 h + r8, y0 + (i & 3),
  // z0 + (i >> 2)), i = 8 part + k, channels tile + 8 q .. + 7; part 0 from halo buffer sb (all its rows
  // at once: the next DMA overwrites it), part 1 from the spare (spread over the next tile's chunks); the
  // residual rows are in rq (drain_load); the statistics leave with the last row of part 1
  auto drain = [&](const V4Tile& tt, int part, int sb, int k0, int k1) {
    if (V5_DIAG(32)) return;
    const int ox = tt.x0 + 8 * h + r8;
    const bool xin = ox < p.W;
    const float xm = xin ? 1.f : 0.f;
    u32x4 sv[8];
    const unsigned char* base = smem + (part ? V5Cfg::STG1 : sb * C::HALO_B);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < k0 || k >= k1) continue;
      const int row = 8 * (h + 4 * k) + r8;
      sv[k] = *reinterpret_cast<const u32x4*>(base + row * 128 + ((q ^ r8) << 4));
    }
    if (part == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
    }
    const unsigned obase =
        ((unsigned)((tt.z0 * p.H + tt.y0) * p.W) + (unsigned)ox) * (unsigned)p.cout * 2u + (unsigned)(tt.ct * 64 + 8 * q) * 2u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < k0 || k >= k1) continue;
      const int i = 8 * part + k;
      float v[8];
      unpack<T>(sv[k], v);
      if (p.rmode >= 0) {
        float r[8];
        unpack<T>(rq[k], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float vv = v[e] * xm;
        s1[e] += vv;
        s2[e] += vv * vv;
      }
      const unsigned oo = obase + (unsigned)(i >> 2) * planeb + (unsigned)(i & 3) * rowb;
      dq[k] = pack<T>(v);
      doff[k] = xin ? oo : 0xFFFFFFF0u;
    }
    if (part == 1 && k1 == 8 && p.stats) {
      // sum over the 8 lanes of each channel block q (lanes q + 8 r8): xor 8 (DPP), 16 (swizzle), 32 (permlane)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float& sx = e < 8 ? s1[e] : s2[e - 8];
        sx += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sx), 0x128, 0xF, 0xF, true));
        sx += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, sx), 0x401F));
        const unsigned u = __builtin_bit_cast(unsigned, sx);
        const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        sx += __builtin_bit_cast(float, lane < 32 ? (unsigned)sw[1] : (unsigned)sw[0]);
      }
      // this helper's partial -> scratch [h][c][2]; the helper that arrives last sums the
      // four in helper order (deterministic) and writes the tile's partial
      // (one slot: consecutive part-1 drains are two barriers apart)
      float* sc = reinterpret_cast<float*>(smem + V5Cfg::SCR) + (h * 64 + 8 * q) * 2;
      if (lane < 8) {
#pragma unroll
        for (int e = 0; e < 8; e += 2)
          *reinterpret_cast<float4*>(sc + 2 * e) = make_float4(s1[e], s2[e], s1[e + 1], s2[e + 1]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      unsigned old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      old = __builtin_amdgcn_readfirstlane(old);
      if ((old & 3u) == 3u) {
        const float* s0 = reinterpret_cast<const float*>(smem + V5Cfg::SCR) + lane * 2;
        float su = 0.f, sq = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) { su += s0[k * 128]; sq += s0[k * 128 + 1]; }
        if (p.stats_wg) {
          // this workgroup's running sums (its tiles in order: deterministic); the last tile's
          // last arriver writes the row -- both channel tiles, zeros where it ran none
          float2* run = reinterpret_cast<float2*>(smem + V5Cfg::RUN);
          float2 r = run[tt.ct * 64 + lane];
          r.x += su; r.y += sq;
          run[tt.ct * 64 + lane] = r;
          if (wg_final) {
            for (int ct = 0; ct < p.nct; ++ct)
              *reinterpret_cast<float2*>(p.stats + ((long long)blockIdx.x * p.cout + ct * 64 + lane) * 2) =
                  run[ct * 64 + lane];
          }
        } else {
          const long long pidx = ((long long)tt.b * tiles + tt.sl) * p.cout + tt.ct * 64 + lane;
          *reinterpret_cast<float2*>(p.stats + pidx * 2) = make_float2(su, sq);
        }
      }
    }
  };
  // the stores of drain slice k0 .. k1 - 1 (tile tt)
  auto drain_put = [&](const V4Tile& tt, int k0, int k1) {
    if (V5_DIAG(32)) return;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<T16*>(p.out) + (long long)tt.b * VV * p.cout, (short)0, (int)(VV * p.cout * 2), 0x00020000);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < k0 || k >= k1) continue;
      __builtin_amdgcn_raw_buffer_store_b128(dq[k], ro, doff[k], 0, 0);
    }
  };
  auto issue_bias = [&](const V4Tile& tt, int slot) {
    if (p.bias && h == 0)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(p.bias + (long long)tt.b * p.bias_bs + tt.ct * 64 + lane),
          (__attribute__((address_space(3))) void*)(smem + V5Cfg::BIAS + slot * 256), 4, 0, 0);
  };

  if constexpr (AA > 0) {
    // ------------------------------------------------- helper waves, apply-ahead sweep
    // Per chunk, in this order (every chunk issues the same vector-memory ops, so the counted
    // waits need no branches): the drain slice's LDS reads and math (outputs held in registers;
    // the compiler's wait for its residual retires chunk k + 1's pieces), AA = A raw loads of this
    // tile's share of range R(it + L), the halo DMA of chunk k + 2, a counted wait that retires
    // everything older than the AA loads, the AA transform + write-through stores, part 1's
    // residual loads, the drain stores.
    constexpr int NA = 10;   // halo pieces per chunk and helper (every lane issues: v4_issue_halo<.., true>)
    const AaLane al = aa_lane(h * 64 + lane, 256);
    const int L = p.aa_lead;
    int pit = 0;
    V4Tile pt = tile_of(0);
    int pc = pt.c0;
    bool chk = false;   // the cursor's tile reads a range some other workgroup may still write
    auto issue_aa = [&](int buf) {
      v4_issue_halo<T, MODE, C::HVP * 16, true>(p, pt, pc, smem + buf * C::HALO_B, h, lane);
      if (pc + 1 < pt.c1) {
        ++pc;
      } else if (pit + 1 < ntile) {
        ++pit; pt = tile_of(pit); pc = pt.c0;
        chk = pit >= L && pit < aa_nit;
      }   // past the last tile: the last chunk again, into a buffer nobody reads
    };
    V4Tile cur = tile_of(0);
    if (h == 0 && lane == 0) *cnt = 0u;
    if (p.stats_wg && h == 0) {
      reinterpret_cast<float4*>(smem + V5Cfg::RUN)[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    issue_aa(0);
    issue_bias(cur, 0);
    issue_aa(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // B0
    int gch = 0;
    int pend = 0, pr = 0;
    const int nch = cur.c1 - cur.c0;
    const int nslice = (nch - 1) < 3 ? (nch - 1) : 3;
    const int srows = (8 + nslice - 1) / nslice;
    const int cs = nch >= 3 ? 1 : 0;   // the AA share skips the part-0 drain chunk where it can
    V4Tile dt = cur;
    for (int it = 0; it < ntile; ++it) {
      const bool more = it + 1 < ntile;
      const V4Tile nxt = more ? tile_of(it + 1) : cur;
      unsigned plo = 0u, phi = 0u;   // this tile's share of R(it + L)
      if (it + L < aa_nit) aa_piece(aa_need(it + L - 1), aa_need(it + L), plo, phi);
      for (int c = cur.c0; c < cur.c1; ++c) {
        const bool first = c == cur.c0, lastc = c + 1 == cur.c1;
        const int cc = c - cur.c0;
        // the range tile it + 1's halo reads: every workgroup's share written? (the DMA of its
        // first chunk goes out in this chunk; the wait's vmcnt(0) retires only what is due anyway)
        if (chk && pc == pt.c0) {
#ifdef CWDM_CONV_STAMPS
          const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
          v5aa_wait(&p.aa_cnt[pit], (unsigned)(G + p.aa_extra), p.aa_spin, 0);
          chk = false;
#ifdef CWDM_CONV_STAMPS
          if (p.stamps && tid == 256) p.stamps[(long long)blockIdx.x * 64 + 56] += __builtin_amdgcn_s_memtime() - t0;
#endif
        }
        // the previous tile's AA share is retired in every helper (chunk 0's wait + barrier): publish it
        if (cc == 1 && it > 0 && it - 1 + L < aa_nit && tid == 256)
          __hip_atomic_fetch_add(&p.aa_cnt[it - 1 + L], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int d0 = 0, k0 = 0, k1 = 0;
        if (pend == 2) {
          drain(dt, 0, (gch + 2) % 3, 0, 8);
          d0 = 1; k0 = 0; k1 = 8;
          pend = 1; pr = 0;
        } else if (pend == 1) {
          k0 = pr; k1 = pr + srows < 8 ? pr + srows : 8;
          drain(dt, 1, 0, k0, k1);
          pr = k1;
          if (pr == 8) pend = 0;
        }
        if (k1 > k0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // this chunk's AA loads (steps n0 .. n0 + AA - 1 of the share; none in the skipped chunk)
        const int n0 = cc >= cs ? (cc - cs) * p.aa_units : -1;
        // (compiler-invisible loads, as the MFMA waves' weights: an ordinary load's own wait would
        // retire the halo DMA issued behind it -- LDS-DMA and loads mixed in vmcnt make the compiler
        // wait for zero)
        u32x4 ax[AA];
        unsigned av[AA];
        bool aok[AA];
#pragma unroll
        for (int a = 0; a < AA; ++a) {
          av[a] = plo + (unsigned)((n0 + a) * al.vps + al.vo);
          aok[a] = n0 >= 0 && a < p.aa_units && al.on && av[a] < phi;
          v4_gload(ax[a], al.src + (size_t)(aok[a] ? av[a] : 0u) * al.rowb);
        }
        issue_aa((gch + 2) % 3);
        // chunk k + 1's pieces and the AA loads (everything older than this chunk's DMA) retired
        if constexpr (AA == 1) {
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ax[0]) : "n"(NA) : "memory");
        } else if constexpr (AA == 2) {
          asm volatile("s_waitcnt vmcnt(%2)" : "+v"(ax[0]), "+v"(ax[1]) : "n"(NA) : "memory");
        } else if constexpr (AA == 4) {
          asm volatile("s_waitcnt vmcnt(%4)" : "+v"(ax[0]), "+v"(ax[1]), "+v"(ax[2]), "+v"(ax[3]) : "n"(NA) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(%8)"
                       : "+v"(ax[0]), "+v"(ax[1]), "+v"(ax[2]), "+v"(ax[3]), "+v"(ax[4]), "+v"(ax[5]), "+v"(ax[6]),
                         "+v"(ax[7])
                       : "n"(NA)
                       : "memory");
        }
        if (p.aa_prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int a = 0; a < AA; ++a)
          if (a < p.aa_units) aa_store(al, ax[a], av[a], aok[a]);
        if (p.aa_prio) __builtin_amdgcn_s_setprio(0);
        if (d0) drain_load(dt, 1);
        if (k1 > k0) drain_put(dt, k0, k1);
        // the finishing tile's part-0 residual rows, under its last chunk
        if (lastc) drain_load(cur, 0);
        if (first && more) issue_bias(nxt, (it + 1) & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        V5_STAMP(34 + gch, tid == 256 && gch < 16);
        __builtin_amdgcn_s_barrier();
        if (lastc) {
          __builtin_amdgcn_s_barrier();   // B2: the MFMA waves staged tile it
          dt = cur;
          pend = 2;
        }
        ++gch;
      }
      cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    drain(dt, 0, (gch + 2) % 3, 0, 8);
    drain_put(dt, 0, 8);
    drain_load(dt, 1);
    wg_final = true;
    drain(dt, 1, 0, 0, 8);
    drain_put(dt, 0, 8);
    V5_STAMP(52, tid == 256);
    // the last workgroup out re-zeroes the sweep counters for the next launch
    if (h == 0) {
      unsigned old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(&p.aa_cnt[kV5AaCnt - 1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = __builtin_amdgcn_readfirstlane(old);
      if (old == (unsigned)G - 1u) {
        for (int r = lane; r < aa_nit; r += 64)
          __hip_atomic_store(&p.aa_cnt[r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) __hip_atomic_store(&p.aa_cnt[kV5AaCnt - 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }

  // prologue: chunk 0 and tile 0's bias, chunk 1; transform chunk 0
  V4Tile cur = tile_of(0);
  if (h == 0 && lane == 0) *cnt = 0u;
  if (p.stats_wg && h == 0) {
    reinterpret_cast<float4*>(smem + V5Cfg::RUN)[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  issue_next(0);
  issue_bias(cur, 0);
  issue_next(1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
  transform(cur.x0, cur.y0, cur.z0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // B0
  int gch = 0;
  int pend = 0;                   // drain parts of dt still to run (2: both, 1: part 1 from row pr)
  int pr = 0;
  // part 1 (the spare staging half, free until this tile's own hand-off) drains in S slices over the
  // next tile's chunks 1 .. S: one whole part per chunk left the helpers behind the MFMA waves at
  // every tile seam of the 4-chunk (64-input-channel) convs (r05 stamps: ~2k cycles per tile)
  const int nslice = (cur.c1 - cur.c0 - 1) < 3 ? (cur.c1 - cur.c0 - 1) : 3;
  const int srows = (8 + nslice - 1) / nslice;
  V4Tile dt = cur;
  for (int it = 0; it < ntile; ++it) {
    const bool more = it + 1 < ntile;
    const V4Tile nxt = more ? tile_of(it + 1) : cur;
    for (int c = cur.c0; c < cur.c1; ++c) {
      const bool first = c == cur.c0, lastc = c + 1 == cur.c1;
      // the drain slice runs first: its residual wait (the compiler's) then also retires chunk
      // k + 1's pieces, and part 0 frees this wave's blocks of the buffer chunk k + 2 goes to
      // (part 0 is followed by part 1's residual loads: 8 stores + 8 loads in flight before the DMA)
      const bool d0 = pend == 2 && p.rmode >= 0;
      int nst = 0;   // stores of this chunk's drain slice
      if (pend == 2) {
        drain(dt, 0, (gch + 2) % 3, 0, 8);
        drain_put(dt, 0, 8);
        drain_load(dt, 1);
        pend = 1; pr = 0; nst = 8;
      } else if (pend == 1) {
        const int k1 = pr + srows < 8 ? pr + srows : 8;
        drain(dt, 1, 0, pr, k1);
        drain_put(dt, pr, k1);
        nst = k1 - pr; pr = k1;
        if (pr == 8) pend = 0;
      }
      if (nst) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const bool iss = issue_next((gch + 2) % 3);
      if (!(lastc && !more)) {
        // chunk k + 1 (the rest of this tile, or the next tile's first chunk): own pieces landed?
        // (everything issued after them: this slice's stores, part 1's residual loads, this DMA)
        if (d0) {
          if (iss) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + 16) : "memory");
          else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        } else if (nst >= 8) {
          if (iss) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + 8) : "memory");
          else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if (nst >= 4) {
          if (iss) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + 4) : "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else if (nst >= 2) {
          if (iss) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + 2) : "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
          if (iss) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const V4Tile& t1 = lastc ? nxt : cur;
        transform(t1.x0, t1.y0, t1.z0, (gch + 1) % 3);
      }
      // the finishing tile's part-0 residual rows, under its last chunk
      if (lastc) drain_load(cur, 0);
      if (first && more) issue_bias(nxt, (it + 1) & 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      V5_STAMP(34 + gch, tid == 256 && gch < 16);
      __builtin_amdgcn_s_barrier();
      if (lastc) {
        __builtin_amdgcn_s_barrier();   // B2: the MFMA waves staged tile it
        dt = cur;
        pend = 2;
      }
      ++gch;
    }
    cur = nxt;
  }
  // the last tile (the MFMA waves have left; its part-0 residual rows were loaded under its last chunk)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  drain(dt, 0, (gch + 2) % 3, 0, 8);
  drain_put(dt, 0, 8);
  drain_load(dt, 1);
  wg_final = true;
  drain(dt, 1, 0, 0, 8);
  drain_put(dt, 0, 8);
  V5_STAMP(52, tid == 256);
}


// ---------------------------------------------------------------------------
// The accurate fast mode: fp32 activations, conv MFMAs on bf16 hi/lo splits,
// three bf16 products per fp32 product: hi(x) hi(w) + lo(x) hi(w) + hi(x) lo(w)
// (lo(x) lo(w), ~2^-18 of the product -- about 64x fp32 epsilon -- is dropped).  Same warp-specialised
// pipeline as conv3d_v5_kernel, but per PAIR of fp32 chunks (16 channels):
//   * helpers DMA both chunks (8 fp32 channels = 32 B per voxel slot each) and
//     convert each in place (the GroupNorm+SiLU applied first when agn is set)
//     into two bf16 planes: plane 0 = hi(x), plane 1 = lo(x) = bf16(x - hi(x));
//     the planes are packed at 1224 slots (no padding), so four chunk buffers --
//     two pairs, double-buffered -- fit the CU's LDS;
//   * the MFMA waves run three bf16 passes per pair (cwdm_conv3d_pack_split):
//     A = [hi(x_a) | lo(x_a)] . [hi(w_a) | hi(w_a)], B = the same for chunk b,
//     C = [hi(x_a) | hi(x_b)] . [lo(w_a) | lo(w_b)] -- pass C's second K half is
//     read from the other chunk's buffer (only the lane base differs), so
//     3 MFMA passes per 16 fp32 channels instead of 4 (2^-16 relative per
//     product instead of bf16's 2^-8; the exact-fp32 MFMA runs at 1/16 rate);
//   * fp32 outputs leave from the accumulators (no 16-bit staging), with the
//     (sum, sum^2) partials reduced across the two plane waves of a channel
//     half through LDS (the second to arrive writes them: deterministic).
// Channels: c0 and c1 multiples of 16 (a pair never straddles the sources).
// ---------------------------------------------------------------------------
struct V5sCfg {
  static constexpr int PLANE = V4Cfg::HV * 16;   // 19584: one quad plane of a chunk (1224 slots)
  static constexpr int BUF = 2 * PLANE;          // one fp32 chunk as its (hi, lo) planes
  static constexpr int PAIR = 2 * BUF;           // two chunks: one pipeline stage
  static constexpr int BIAS = 2 * PAIR;          // 156672: bias of tile parity s at + 256 s
  static constexpr int SCR = BIAS + 512;         // statistics partials
  static constexpr int GSS = SCR + 2048;         // GroupNorm (sc, sh) [4 buffers][4 helpers][8 ch][2] fp32 (128 B rows)
  static constexpr int CNT = GSS + 2048;         // statistics arrival counters
  static constexpr int RUN = CNT + 256;          // per-workgroup statistics (stats_wg): [2 ch tiles][64][2] fp32
  static constexpr int SMEM = RUN + 1024;        // 162560 of the CU's 163840
};
static_assert(V5sCfg::SMEM <= 163840, "v5s LDS");

template <int MODE, bool GN>
__global__ void __launch_bounds__(512) conv3d_v5s_kernel(V4Params p) {
  using C = V4Cfg;
  using S = V5sCfg;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[S::SMEM];

  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, hh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = p.nblk;
  const int ntile = (nblk - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  if (ntile <= 0) return;
  auto tile_of = [&](int it) { return v4_tile_of(p, it); };
  const int tiles = p.tx * p.ty * p.tz;
  const int nvc = 3 * (p.nch / 2);   // bf16 weight chunks: three passes per pair of fp32 chunks
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + S::CNT);

  if (wv < 4) {
    // ------------------------------------------------------------ MFMA waves
    __builtin_amdgcn_s_setprio(2);
    const int f = wv & 1, vg = wv >> 1, zb = 2 * vg;
    const unsigned char* wlane = p.aw + f * 1024 + lr * 32 + ((hh ^ ((lr >> 3) & 1)) << 4);
    auto load_w = [&](u32x4 (&w)[3], int ct, int cv, int g) {
      const unsigned char* src = wlane + ((long long)ct * nvc + cv) * 27 * 2048 + ((g / 3) * 9 + (g % 3)) * 2048;
      v4_gload(w[0], src);
      v4_gload(w[1], src + 3 * 2048);
      v4_gload(w[2], src + 6 * 2048);
    };
    const int rows = (zb * (C::HX * C::HY) + lr) * 16;
    const int hl_ab = hh * S::PLANE + rows;   // passes A / B: (hi, lo) planes of one chunk
    const int hl_c = hh * S::BUF + rows;      // pass C: the hi planes of chunk a (K 0-7) and chunk b (K 8-15)
    f32x16 acc[2][4];
    u32x4 wr[3][3];
    V4Tile cur = tile_of(0);
    load_w(wr[0], cur.ct, 3 * (cur.c0 / 2), 0);
    load_w(wr[1], cur.ct, 3 * (cur.c0 / 2), 1);
    __builtin_amdgcn_s_barrier();   // B0
    int gp = 0;
    const long long HW = (long long)p.H * p.W, V = (long long)p.D * HW;
    for (int it = 0; it < ntile; ++it) {
      const bool more = it + 1 < ntile;
      const V4Tile nxt = more ? tile_of(it + 1) : cur;
      {
        float bia[16];
        const float* bl = reinterpret_cast<const float*>(smem + S::BIAS + (it & 1) * 256) + f * 32 + 4 * hh;
#pragma unroll
        for (int i = 0; i < 16; ++i) bia[i] = bl[8 * (i >> 2) + (i & 3)];
        const float bm = p.bias ? 1.f : 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][m][i] = bia[i] * bm;
      }
      // one bf16 weight pass (virtual chunk cv) over the planes at hb; LASTV: the tile's last pass
      auto vpass = [&](auto lastc, int cv, const unsigned char* hb) {
        constexpr bool LASTV = decltype(lastc)::value;
        u32x4 av[2][6];
        v4_read_step<0>(av[0], hb);
#define V5S_STEP(K)                                                                                          \
        {                                                                                                    \
          constexpr int GI = (K) / 2, PL = (K) % 2, KN = (K) + 1, BC = (K) & 1;                              \
          if (PL == 0) {                                                                                     \
            if (GI + 2 < 9) load_w(wr[(GI + 2) % 3], cur.ct, cv, GI + 2);                                    \
            else if (!LASTV) load_w(wr[(GI + 2) % 3], cur.ct, cv + 1, GI - 7);                               \
            else load_w(wr[(GI + 2) % 3], nxt.ct, 3 * (nxt.c0 / 2), GI - 7);                                 \
          }                                                                                                  \
          if (KN < 18) v4_read_step<KN % 18>(av[BC ^ 1], hb);                                                \
          if (PL == 0) V4_WAIT_W(6, wr[GI % 3]);                                                             \
          __builtin_amdgcn_sched_barrier(0);                                                                 \
          _Pragma("unroll") for (int dy = 0; dy < 3; ++dy)                                                   \
          _Pragma("unroll") for (int m = 0; m < 4; ++m)                                                      \
            v4_mfma<bf16_t>(acc[PL][m], wr[GI % 3][dy], av[BC][m + dy]);                                     \
          __builtin_amdgcn_sched_barrier(0);                                                                 \
        }
        V5S_STEP(0) V5S_STEP(1) V5S_STEP(2) V5S_STEP(3) V5S_STEP(4) V5S_STEP(5)
        V5S_STEP(6) V5S_STEP(7) V5S_STEP(8) V5S_STEP(9) V5S_STEP(10) V5S_STEP(11)
        V5S_STEP(12) V5S_STEP(13) V5S_STEP(14) V5S_STEP(15) V5S_STEP(16) V5S_STEP(17)
#undef V5S_STEP
      };
      const int p1 = cur.c1 / 2;
      for (int pp = cur.c0 / 2; pp + 1 < p1; ++pp) {
        const unsigned char* base = smem + (gp & 1) * S::PAIR;
        vpass(std::false_type{}, 3 * pp, base + hl_ab);
        vpass(std::false_type{}, 3 * pp + 1, base + S::BUF + hl_ab);
        vpass(std::false_type{}, 3 * pp + 2, base + hl_c);
        __builtin_amdgcn_s_barrier();   // pair k read; pair k + 1 split
        ++gp;
      }
      {
        const int pp = p1 - 1;
        const unsigned char* base = smem + (gp & 1) * S::PAIR;
        vpass(std::false_type{}, 3 * pp, base + hl_ab);
        vpass(std::false_type{}, 3 * pp + 1, base + S::BUF + hl_ab);
        vpass(std::true_type{}, 3 * pp + 2, base + hl_c);
        __builtin_amdgcn_s_barrier();
        ++gp;
      }
      // fp32 epilogue from the accumulators: + residual, store, (sum, sum^2) partials
      {
        const int c0w = cur.ct * 64 + f * 32, cl = c0w + 4 * hh;
        const int ox = cur.x0 + lr;
        const bool xin = ox < p.W;
        const float xm = xin ? 1.f : 0.f;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<float*>(p.out) + (long long)cur.b * V * p.cout, (short)0, (int)(V * p.cout * 4), 0x00020000);
        const long long rV = p.rmode == 1 ? V / 8 : V;
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(reinterpret_cast<const float*>(p.res) + (long long)cur.b * rV * p.cout), (short)0,
            (int)(rV * p.cout * 4), 0x00020000);
        float ssum[16], ssq[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) { ssum[i] = 0.f; ssq[i] = 0.f; }
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int oy = cur.y0 + m, oz = cur.z0 + zb + pl;
            const unsigned vo = (unsigned)((oz * p.H + oy) * p.W + ox);
            const unsigned rvo = p.rmode == 1 ? (unsigned)(((oz >> 1) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1)) : vo;
            float4 rq[4];
            if (p.rmode >= 0) {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(
                    rr, xin ? (rvo * (unsigned)p.cout + (unsigned)(cl + 8 * j)) * 4u : 0xFFFFFFF0u, 0, 0);
                rq[j] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                                    __uint_as_float(q[3]));
              }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float v[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) v[k] = acc[pl][m][4 * j + k];
              if (p.rmode >= 0) { v[0] += rq[j].x; v[1] += rq[j].y; v[2] += rq[j].z; v[3] += rq[j].w; }
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                ssum[4 * j + k] += v[k] * xm;
                ssq[4 * j + k] += v[k] * v[k] * xm;
              }
              u32x4 w;
#pragma unroll
              for (int k = 0; k < 4; ++k) w[k] = __float_as_uint(v[k]);
              __builtin_amdgcn_raw_buffer_store_b128(w, ro, xin ? (vo * (unsigned)p.cout + (unsigned)(cl + 8 * j)) * 4u
                                                               : 0xFFFFFFF0u, 0, 0);
            }
          }
        if (p.stats) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            ssum[i] = row16_sum(ssum[i]);
            ssq[i] = row16_sum(ssq[i]);
            ssum[i] += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, ssum[i]), 0x401F));
            ssq[i] += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, ssq[i]), 0x401F));
          }
          // this wave's partial: scratch [f][vg][2 halves][16] sums, then squares at + 256
          float* sc = reinterpret_cast<float*>(smem + S::SCR) + (f * 2 + vg) * 32 + hh * 16;
          if (lr == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) { sc[i] = ssum[i]; sc[256 + i] = ssq[i]; }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          unsigned old = 0;
          if (lane == 0) old = __hip_atomic_fetch_add(cnt + f, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
          old = __builtin_amdgcn_readfirstlane(old);
          if (old & 1u) {   // the second of the channel half's two plane waves
            if (lane < 32) {
              const int h2 = (lane >> 2) & 1, i = 4 * (lane >> 3) + (lane & 3);
              const float* s0 = reinterpret_cast<const float*>(smem + S::SCR) + f * 64 + h2 * 16 + i;
              const float su = s0[0] + s0[32], sq = s0[256] + s0[256 + 32];
              if (p.stats_wg) {
                // per-workgroup running sums (tile order: deterministic); the last tile writes the row,
                // both channel tiles (zeros where this workgroup ran none)
                float2* run = reinterpret_cast<float2*>(smem + S::RUN);
                float2 r = run[cur.ct * 64 + f * 32 + lane];
                r.x += su; r.y += sq;
                run[cur.ct * 64 + f * 32 + lane] = r;
                if (it + 1 == ntile)
                  for (int ct = 0; ct < p.nct; ++ct)
                    *reinterpret_cast<float2*>(p.stats + ((long long)blockIdx.x * p.cout + ct * 64 + f * 32 + lane) * 2) =
                        run[ct * 64 + f * 32 + lane];
              } else {
                const long long pidx = ((long long)cur.b * tiles + cur.sl) * p.cout + c0w + lane;
                *reinterpret_cast<float2*>(p.stats + pidx * 2) = make_float2(su, sq);
              }
            }
          }
        }
      }
      cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[0][2]), "+v"(wr[1][0]), "+v"(wr[1][1]),
                 "+v"(wr[1][2])::"memory");
    return;
  }

  // -------------------------------------------------------------- helper waves
  const int h = wv - 4;
  int pit = 0;
  V4Tile pt = tile_of(0);
  int pc = pt.c0;   // the next pair's first fp32 chunk
  // the next pair (two chunks) into pipeline stage st: buffers 2 st, 2 st + 1
  auto issue_pair = [&](int st) -> bool {
    if (pit >= ntile) return false;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      v4_issue_halo<float, MODE, S::PLANE>(p, pt, pc + k, smem + st * S::PAIR + k * S::BUF, h, lane);
      if constexpr (GN) {
        if (lane < 16)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(p.agn + ((long long)pt.b * (p.ac0 + p.ac1) + (pc + k) * 8) * 2 +
                                                              lane),
              (__attribute__((address_space(3))) void*)(smem + S::GSS + ((2 * st + k) * 4 + h) * 128), 4, 0, 0);
      }
    }
    if (pc + 2 < pt.c1) pc += 2;
    else if (++pit < ntile) { pt = tile_of(pit); pc = pt.c0; }
    return true;
  };
  // fp32 chunk in buffer bi, this wave's voxel slots (h + 4 j) * 64 + lane (< HV: the planes
  // are packed, a padding slot would be the next plane's): (GroupNorm + SiLU,) then
  // plane 0 <- hi, plane 1 <- lo of the 8 channels
  auto split = [&](int x0, int y0, int z0, int bi) {
    unsigned char* hb = smem + bi * S::BUF;
    u32x4 x[2][5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int hv = (h + 4 * j) * 64 + lane;
#pragma unroll
      for (int qd = 0; qd < 2; ++qd)
        if (j < 4 || hv < C::HV) x[qd][j] = *reinterpret_cast<const u32x4*>(hb + qd * S::PLANE + hv * 16);
    }
    float sc[8], sh[8], mk[5];
    if constexpr (GN) {
      const float* gs = reinterpret_cast<const float*>(smem + S::GSS + (bi * 4 + h) * 128);
#pragma unroll
      for (int e = 0; e < 8; ++e) silu_aff_coef(gs[2 * e], gs[2 * e + 1], sc[e], sh[e]);
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int hv = (h + 4 * j) * 64 + lane;
        const int hx = hv % C::HX, hy = (hv / C::HX) % C::HY, hz = hv / (C::HX * C::HY);
        const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
        mk[j] = (hv < C::HV && ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) ? 1.f : 0.f;
      }
    } else {
      (void)x0; (void)y0; (void)z0;
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int hv = (h + 4 * j) * 64 + lane;
      if (j == 4 && hv >= C::HV) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = __uint_as_float(x[0][j][e]); v[4 + e] = __uint_as_float(x[1][j][e]); }
      if constexpr (GN) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = silu_aff(v[e], sc[e], sh[e]) * mk[j];
      }
      u32x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = pack2<bf16_t>(v[2 * e], v[2 * e + 1]);
        lo[e] = pack2<bf16_t>(v[2 * e] - lo2f<bf16_t>(hi[e]), v[2 * e + 1] - hi2f<bf16_t>(hi[e]));
      }
      *reinterpret_cast<u32x4*>(hb + hv * 16) = hi;
      *reinterpret_cast<u32x4*>(hb + S::PLANE + hv * 16) = lo;
    }
  };
  auto issue_bias = [&](const V4Tile& tt, int slot) {
    if (p.bias && h == 0)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(p.bias + (long long)tt.b * p.bias_bs + tt.ct * 64 + lane),
          (__attribute__((address_space(3))) void*)(smem + S::BIAS + slot * 256), 4, 0, 0);
  };
  V4Tile cur = tile_of(0);
  if (h == 0 && lane < 2) cnt[lane] = 0u;
  if (p.stats_wg && h == 0) reinterpret_cast<float4*>(smem + S::RUN)[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  issue_pair(0);
  issue_bias(cur, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  split(cur.x0, cur.y0, cur.z0, 0);
  split(cur.x0, cur.y0, cur.z0, 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // B0
  int gp = 0;
  for (int it = 0; it < ntile; ++it) {
    const bool more = it + 1 < ntile;
    const V4Tile nxt = more ? tile_of(it + 1) : cur;
    for (int pp = cur.c0 / 2; pp < cur.c1 / 2; ++pp) {
      const bool first = pp == cur.c0 / 2, lastp = pp + 1 == cur.c1 / 2;
      // stage gp + 1 (the tile's next pair, or the next tile's first) under this stage's MFMAs
      const int st = (gp + 1) & 1;
      const bool iss = issue_pair(st);
      if (first && more) issue_bias(nxt, (it + 1) & 1);
      if (iss) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const V4Tile& t1 = lastp ? nxt : cur;
        split(t1.x0, t1.y0, t1.z0, 2 * st);
        split(t1.x0, t1.y0, t1.z0, 2 * st + 1);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      ++gp;
    }
    cur = nxt;
  }
}

namespace {
int v5_mode() {
  static const int m = [] { const char* e = std::getenv("CWDM_V5"); return e ? std::atoi(e) : 3; }();
  return m;
}
}  // namespace

bool sg_eligible(const cwdm_conv3d_desc* d);
int v4_ksplit(const cwdm_conv3d_desc* d);
extern std::atomic<int> g_conv_path;
extern std::atomic<unsigned long long*> g_stamps;
std::atomic<int> g_v5_grid{0};
std::atomic<int> g_v5_aa{[] { const char* e = std::getenv("CWDM_V5_AA"); return e ? std::atoi(e) : 1; }()};
std::atomic<int> g_v5_aa_launches{0};
int64_t v4_items(const cwdm_conv3d_desc* d);
bool gbwd_grid_ok(const cwdm_conv3d_desc* d);
std::atomic<int> g_v5_aa_extra{0};
std::atomic<int> g_v5_aa_spin{0};
// the U-Net plan asks for per-workgroup GroupNorm partials (V4Params::stats_wg) around its convs and
// reads back how many rows a launch wrote (0: the per-tile layout of cwdm_conv3d_parts)
thread_local int g_stats_wg = 0;
thread_local int64_t g_stats_rows = 0;

namespace {
int v5_ncu() {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  return ncu;
}
// the persistent grid of an apply-ahead launch: every workgroup must be resident at once (its counter
// waits span the grid), so never more than the CUs x the instance's occupancy, whatever the debug cap
int v5_aa_grid(int64_t nblk) {
  static const int occ = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv3d_v5_kernel<bf16_t, 0, false, 8>, 512, 0) != hipSuccess)
      return 1;
    return n > 0 ? n : 1;
  }();
  const int cap = g_v5_grid.load(std::memory_order_relaxed);
  const int64_t lim = (int64_t)v5_ncu() * occ;
  return (int)std::min<int64_t>(nblk, cap > 0 ? std::min<int64_t>(cap, lim) : v5_ncu());
}
}  // namespace

// the warp-specialised kernel takes a conv of the DMA path when it is a 16-bit
// fast-epilogue conv without K split and with at least one tile per CU (CWDM_V5_MIN_TPC)
// (env CWDM_V5: 0 off, 1 GroupNorm'd inputs only, 2 every eligible conv, 3 (default)
// every eligible conv with the GroupNorm applied by the cwdm_gn_apply pre-pass: the
// in-LDS transform costs the helper waves more issue cycles than the MFMA waves
// leave them -- measured 611 vs 588 us on the 64->64 128^3-subband conv)
bool v5_eligible(const cwdm_conv3d_desc* d, bool gn) {
  const int mode = v5_mode();
  const int path = g_conv_path.load(std::memory_order_relaxed);
  if (d->dtype == CWDM_F32) {
    // the accurate fast mode (conv3d_v5s_kernel): wherever the split weights are
    // given and the shape tiles (no minimum work: it is 8x the exact-fp32 MFMA rate)
    if (!d->a_w_split || path == 1 || path == 3) return false;
    if (d->out_dtype != CWDM_F32 || d->accumulate || d->out1) return false;
    if (d->a_mode != 0 && d->a_mode != 1) return false;
    if (d->a_c0 % 16 || d->a_c1 % 16) return false;   // pairs of 8-channel fp32 chunks, never straddling the sources
    if (d->res_mode < -1 || d->res_mode > 1) return false;
    // the 1x1 skip product is added through the residual slot (conv3d_v4_forward): not both
    if (d->b_w && d->res_mode >= 0) return false;
    if (d->W < kWideMinW || d->H % 4 || d->D % 4 || d->cout % 64) return false;
    // 32-bit buffer offsets per batch: the output, and the sources (raw, or the
    // activated (c0 + c1)-channel copy of the training forward's pre-pass)
    const int64_t lim = 0xFFFFE000LL;
    if (d->D * d->H * d->W * d->cout * 4 >= lim) return false;
    const int64_t sv = d->a_mode == 1 ? d->D * d->H * d->W / 8 : d->D * d->H * d->W;
    if (d->a_gn ? sv * (d->a_c0 + d->a_c1) * 4 >= lim : (sv * d->a_c0 * 4 >= lim || sv * d->a_c1 * 4 >= lim))
      return false;
    return !(gn && d->a_mode == 1);
  }
  if (mode <= 0 || (mode == 1 && !gn) || path == 1 || path == 3) return false;
  // GroupNorm+SiLU in LDS: not for an upsampling conv (its halo repeats every
  // source voxel 8x: the pre-pass at the half resolution is 8x cheaper), and
  // not in mode 3 (pre-pass + this kernel on the activated copy)
  if (gn && (d->a_mode == 1 || mode == 3)) return false;
  if (!dtype_half(d->dtype) || sg_eligible(d)) return false;
  if (path != 2 && v4_ksplit(d) != 1) return false;   // (path 2: forced, no K split of its own)
  if (d->out_dtype != d->dtype || d->accumulate || d->out1) return false;
  if (d->a_mode != 0 && d->a_mode != 1) return false;
  if (d->res_mode < -1 || d->res_mode > 1) return false;
  if (d->W < kWideMinW || d->H % 4 || d->D % 4 || d->cout % 64) return false;
  if (d->D * d->H * d->W * d->cout * 2 >= 0xFFFFE000LL) return false;
  if (d->a_c0 + d->a_c1 < 32) return false;   // >= 2 chunks per tile: a tile's drain spans two chunks
  if (gbwd_grid_ok(d)) return false;   // the backward's fused dgrad instance is v4's
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  // tiles per CU below which v4 (two workgroups per CU) keeps the conv (env
  // CWDM_V5_MIN_TPC, A/B knob; 1 since r04: config 5's 56^3 64-channel convs,
  // 392 tiles, 57 -> 53 us on v5)
  static const double min_tpc = [] { const char* e = std::getenv("CWDM_V5_MIN_TPC"); return e ? std::atof(e) : 1.0; }();
  return path == 2 || (double)v4_items(d) >= min_tpc * ncu;
}

// sources a0 (c0 channels; chunk-major if a0_cm) and a1 (c1, channels-last);
// agn: [B][c0 + c1][2] GroupNorm scale / shift applied in LDS (null: none)
// apply-ahead (conv3d_v5_kernel<.., AA>) for a GroupNorm'd conv input: the per-chunk share AA (1, 2, 4,
// 8 steps of 256 lanes) its sweep needs, or 0 where it does not apply (env CWDM_V5_AA=0: never)
int v5_aa_units(const cwdm_conv3d_desc* d, int* lead) {
  const int mode = g_v5_aa.load(std::memory_order_relaxed);
  if (!mode || !d->a_gn || d->B != 1 || d->a_mode != 0 || !dtype_half(d->dtype)) return 0;
  const int C = d->a_c0 + d->a_c1;
  if (d->a_c0 % 8 || d->a_c1 % 8 || C % 16 || C > 2048) return 0;
  if (!v5_eligible(d, false)) return 0;
  // the helpers' share per chunk fits beside the drain from 8 input chunks (r05 stamps: the
  // 4-chunk 64-channel convs left them ~4k cycles behind the MFMA waves per chunk); env
  // CWDM_V5_AA_MINCH (A/B knob)
  static const int minch = [] { const char* e = std::getenv("CWDM_V5_AA_MINCH"); return e ? std::atoi(e) : 8; }();
  if (mode == 1 && (d->a_c0 + d->a_c1) / 16 < minch) return 0;
  const int64_t V = d->D * d->H * d->W;
  if (V * C * 2 >= 0x7FFFF000LL) return 0;
  const int tx = (int)((d->W + 31) / 32), ty = (int)(d->H / 4), tz = (int)(d->D / 4), nct = d->cout / 64;
  const int64_t nblk = (int64_t)tx * ty * tz * nct;
  const int G = v5_aa_grid(nblk);
  const int nit = (int)((nblk + G - 1) / G);
  if (nit > kV5AaCnt - 2) return 0;
  const int nch = C / 16;
  const int L = nch >= 8 ? 2 : 3;
  // the ranges of the first L iterations are a prologue nothing overlaps: worth it only where the
  // sweep is long (r05: the 128^3 128-channel conv, 32 iterations, 1650 -> 1593 us; the 64^3
  // ones, 4 iterations, all prologue, +3 %)
  if (mode == 1 && nit < 16) return 0;
  const int Q = C / 8, vps = 256 / Q;
  if (vps < 1) return 0;
  const int cs = nch >= 3 ? 1 : 0;
  int64_t steps = 0;
  for (int r = L; r < nit; ++r) {
    const int64_t len = (int64_t)v5aa_need(r, G, (int)nblk, nct, tx, ty, (int)d->D, (int)d->H, (int)d->W) -
                        v5aa_need(r - 1, G, (int)nblk, nct, tx, ty, (int)d->D, (int)d->H, (int)d->W);
    steps = std::max<int64_t>(steps, ((len + G - 1) / G + vps - 1) / vps);
  }
  const int64_t per = std::max<int64_t>(1, (steps + (nch - cs) - 1) / (nch - cs));
  if (per > 8) return 0;
  if (lead) *lead = L;
  return (int)per;
}

int v5_launch(const cwdm_conv3d_desc* d, const void* a0, int c0, const void* a1, int c1, int a0_cm,
              const float* agn, const void* res, int rmode, hipStream_t s, const V5Aa* aa) {
  const int esz = dtype_size(d->dtype);
  const int ck = 32 / esz;
  const int64_t SV = d->a_mode == 1 ? d->D * d->H * d->W / 8 : d->D * d->H * d->W;
  CWDM_REQUIRE(!agn || !a0_cm, CWDM_E_INVALID, "conv3d_v5: GroupNorm applies to raw channels-last sources only");
  V4Params p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W;
  p.tx = (p.W + 31) / 32; p.ty = p.H / 4; p.tz = p.D / 4;
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
  p.stats = d->stats;
  p.ksplit = 1; p.kper = p.nch;
  p.agn = agn;
  if (aa) {
    CWDM_REQUIRE(a0_cm && !agn && d->B == 1 && d->a_mode == 0, CWDM_E_INVALID, "conv3d_v5: apply-ahead arguments");
    p.ax0 = aa->x0; p.axc0 = aa->c0; p.ax1 = aa->x1; p.axc1 = aa->c1;
    p.agn = aa->gn;
    p.aa_lead = aa->lead;
    p.aa_units = aa->units;
    static const int prio = [] { const char* e = std::getenv("CWDM_V5_AA_PRIO"); return e ? std::atoi(e) : 0; }();
    p.aa_prio = prio;
    CWDM_REQUIRE(aa->cnt, CWDM_E_INVALID, "conv3d_v5: apply-ahead counters missing");
    p.aa_cnt = aa->cnt;
    const int spin = g_v5_aa_spin.load(std::memory_order_relaxed);
    p.aa_spin = spin > 0 ? spin : (1 << 24);
    p.aa_extra = g_v5_aa_extra.load(std::memory_order_relaxed);
  }
#ifdef CWDM_V5_DIAG
  static const int diag = [] { const char* e = std::getenv("CWDM_V5_DIAGMASK"); return e ? std::atoi(e) : 0; }();
  p.diag = diag;
#endif
  p.stamps = g_stamps.load(std::memory_order_relaxed);
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz * p.nct;
  p.nblk = (int)nblk;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  const int cap = g_v5_grid.load(std::memory_order_relaxed);
  const dim3 grid(aa ? (unsigned)v5_aa_grid(nblk) : (unsigned)std::min<long long>(nblk, cap > 0 ? cap : ncu));
  // per-workgroup statistics rows (16-bit kernel, batch 1, <= 2 channel tiles, no more rows than the
  // per-tile layout has): the finalize then reduces gridDim.x rows instead of one per tile
  if (g_stats_wg && d->stats && p.B == 1 && p.nct <= 2 &&
      (long long)grid.x <= (long long)p.tx * p.ty * p.tz) {
    p.stats_wg = 1;
    g_stats_rows = grid.x;
  }
  prof_begin(s);
  auto go = [&](auto tag) {
    using T = decltype(tag);
    if (agn) {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v5_kernel<T, 1, true>), grid, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v5_kernel<T, 0, true>), grid, dim3(512), 0, s, p);
    } else {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v5_kernel<T, 1, false>), grid, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v5_kernel<T, 0, false>), grid, dim3(512), 0, s, p);
    }
  };
  if (d->dtype == CWDM_F32) {
    p.aw = reinterpret_cast<const unsigned char*>(d->a_w_split);
    if (agn) {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v5s_kernel<1, true>), grid, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v5s_kernel<0, true>), grid, dim3(512), 0, s, p);
    } else {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v5s_kernel<1, false>), grid, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v5s_kernel<0, false>), grid, dim3(512), 0, s, p);
    }
  } else if (aa) {
    g_v5_aa_launches.fetch_add(1, std::memory_order_relaxed);
    auto go_aa = [&](auto tag) {
      using T = decltype(tag);
      // (the instance's loads per chunk >= the share: 4 or 8)
      if (aa->units <= 4) hipLaunchKernelGGL((conv3d_v5_kernel<T, 0, false, 4>), grid, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v5_kernel<T, 0, false, 8>), grid, dim3(512), 0, s, p);
    };
    if (d->dtype == CWDM_BF16) go_aa(bf16_t{});
    else go_aa(f16_t{});
  } else if (d->dtype == CWDM_BF16) {
    go(bf16_t{});
  } else {
    go(f16_t{});
  }
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * (c0 + c1));
  CWDM_LAUNCHED();
  return CWDM_OK;
}

template __global__ void conv3d_v5_kernel<bf16_t, 0, true>(V4Params);
template __global__ void conv3d_v5_kernel<bf16_t, 1, true>(V4Params);
template __global__ void conv3d_v5_kernel<bf16_t, 0, false>(V4Params);
template __global__ void conv3d_v5_kernel<bf16_t, 1, false>(V4Params);
template __global__ void conv3d_v5_kernel<f16_t, 0, true>(V4Params);
template __global__ void conv3d_v5_kernel<f16_t, 1, true>(V4Params);
template __global__ void conv3d_v5_kernel<f16_t, 0, false>(V4Params);
template __global__ void conv3d_v5_kernel<f16_t, 1, false>(V4Params);
template __global__ void conv3d_v5_kernel<bf16_t, 0, false, 4>(V4Params);
template __global__ void conv3d_v5_kernel<bf16_t, 0, false, 8>(V4Params);
template __global__ void conv3d_v5_kernel<f16_t, 0, false, 4>(V4Params);
template __global__ void conv3d_v5_kernel<f16_t, 0, false, 8>(V4Params);
template __global__ void conv3d_v5s_kernel<0, true>(V4Params);
template __global__ void conv3d_v5s_kernel<1, true>(V4Params);
template __global__ void conv3d_v5s_kernel<0, false>(V4Params);
template __global__ void conv3d_v5s_kernel<1, false>(V4Params);

}  // namespace cwdm

extern "C" int cwdm_debug_v5_aa(int on) {
  if (on < 0) return cwdm::g_v5_aa_launches.load(std::memory_order_relaxed);
  return cwdm::g_v5_aa.exchange(on > 2 ? 2 : on);
}

extern "C" int cwdm_debug_v5_aa_timeout(int extra, int spin) {
  CWDM_REQUIRE(extra >= 0 && spin >= 0, CWDM_E_INVALID, "cwdm_debug_v5_aa_timeout: extra, spin >= 0");
  cwdm::g_v5_aa_extra.store(extra);
  cwdm::g_v5_aa_spin.store(spin);
  return CWDM_OK;
}

extern "C" int cwdm_device_status(int clear) {
  unsigned v = 0;
  CWDM_HIP(hipDeviceSynchronize());
  CWDM_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(cwdm::g_cwdm_dev_err), sizeof(v), 0, hipMemcpyDeviceToHost));
  if (clear && v) {
    const unsigned z = 0;
    CWDM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(cwdm::g_cwdm_dev_err), &z, sizeof(z), 0, hipMemcpyHostToDevice));
  }
  return (int)v;
}

extern "C" int cwdm_debug_v5_grid(int n) {
  CWDM_REQUIRE(n >= 0, CWDM_E_INVALID, "cwdm_debug_v5_grid: n >= 0");
  return cwdm::g_v5_grid.exchange(n);
}
