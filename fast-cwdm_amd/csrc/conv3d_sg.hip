// Conv3d 3x3x3 (stride 1, pad 1) for the small-grid U-Net levels (16^3, 8^3:
// W = 16 or 8), bf16 or fp16, on v_mfma_f32_16x16x32_{bf16,f16}.  Same contract as the
// DMA-staged wide-grid kernel (V4Params: GroupNorm+SiLU and the 1x1 skip are
// pre-passes in conv3d_v4_forward; this kernel stages raw copies), called from
// v4_launch for shapes sg_eligible() accepts.
//
// Why a separate kernel: a 16^3 x 256-channel conv is only 4096 x 256 outputs.
// The wide kernel's 512-voxel x 64-channel tiles give 32 work items there, so
// the brick kernels split K (768 items) and pay two finishing passes over the
// fp32 slices (splitk_sum + conv3d_reduce, ~17 us per conv at 16^3, more than
// the conv's MFMA work).  Here a work item is one statistics brick of
// pick_brick (16x4x4 or 8x8x4 = 256 voxels, the partial layout of
// cwdm_conv3d_parts is unchanged) x 16 output channels with the whole K:
// 256 workgroups at 16^3, no split, no finishing pass.
//
//   * 4 waves, wave w = z-plane w of the brick (64 voxels = 4 B operands of
//     16 voxels: one x line of 16, or two lines of 8).
//   * K chunks of 32 input channels (two 16-channel sub-chunks: chunk-major
//     gn_apply output or channels-last sources, concat boundary per
//     sub-chunk); MFMA K = the chunk's 32 channels of one tap.
//   * Halo image in LDS, per 16-channel sub-chunk [HVP slots][2 quads][16 B]
//     (32-B slot pitch), double buffered, filled by LDS-DMA (out-of-volume
//     voxels read as zeros through the buffer range check).  A DMA instruction
//     covers 32 consecutive slots x both quads, i.e. whole 32-B voxel rows of
//     the chunk-major source (a quad-major image made every instruction fetch
//     64 half-used lines: ~8 B/clk per CU, tools/sg_stamps.py); a ds_read_b128
//     of 16 lanes reads 16 consecutive slots of one quad (2-way bank conflict).
//   * The chunk's A fragments (16 output channels x 32 K per tap, 27 KB) are
//     LDS-DMA'd beside its halo, double-buffered too: one workgroup per CU
//     (144 KB of LDS) has no co-resident partner to hide global-load latency,
//     so nothing in the inner loop waits on memory; one vmcnt(0) + barrier
//     per chunk.
//   * Per (dz, dx) group the operand lines are read once and feed the 3 dy
//     taps (6 reads / 12 MFMAs at W = 16, 9 / 12 at W = 8), with the group's 3
//     A fragments; the next group's reads are issued before this group's
//     MFMAs.
//   * Epilogue: + bias, + residual (same grid / nearest-upsampled), bf16
//     store, per-(brick, channel) (sum, sum^2) partials for the next
//     GroupNorm.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "conv3d_v4.hpp"

namespace cwdm {

typedef float sg_f32x4 __attribute__((ext_vector_type(4)));

template <int BX, int BY, int PAD>
struct SGCfg {
  // PAD 1: the 3x3x3 halo (648 / 600 voxels); PAD 0: the brick itself (1x1 skip)
  static constexpr int HX = BX + 2 * PAD, HY = BY + 2 * PAD, HZ = 4 + 2 * PAD, HV = HX * HY * HZ;
  static constexpr int PCS = (HV + 63) / 64;                                   // 1 KB pieces per quad's worth of slots
  static constexpr int HVP = PCS * 64;                                         // 704 slots
  static constexpr int SUB = HVP * 32;                                         // bytes per 16-channel sub-chunk image
  static constexpr int BUF = 2 * SUB;                                          // one halo buffer (32 channels)
  static constexpr int WBUF = 27 * 1024;       // one chunk's A fragments: [tap][lane][16 B]
  static constexpr int SMEM = 2 * BUF + 2 * WBUF;
  static constexpr int LPO = 16 / BX;         // x lines per 16-voxel operand
  static constexpr int NR = 3 * LPO + 3;      // distinct operand line starts per (dz, dx) group
  static_assert(BX * BY == 64, "a brick plane is 64 voxels");
};

struct SGParams {
  V4Params v;   // shape / sources / weights / epilogue as for the wide kernel (ct counts 64-row tiles)
  int ntile16;  // output channel tiles of 16
  int parts;    // statistics bricks per batch (tx * ty * tz; the last brick of an axis may be partial)
  int tx, ty;   // bricks along x and y
  // K split (the 8^3 level: 32 tiles): slice ks runs chunks [ks kper, +kper); it
  // stores its fp32 accumulators at part + (tile S + ks) 4096, and the slice
  // that arrives last at the tile's counter sums all S in slice order (the
  // result does not depend on the arrival order) and runs the epilogue
  int ksplit, kper;
  float* part;
  // per-tile arrival counters of this launch (K split only): caller memory,
  // zero when the launch starts (the last slice of a tile resets its counter, so
  // launches in stream order can share one block zeroed once: the U-Net plan
  // zeroes one per forward / backward, a lone cwdm_conv3d_forward memsets its
  // own in the workspace).  Never a process-wide array: launches on other
  // streams or plans would share tiles' counters.
  unsigned* count;
  int xcd;   // 1: XCD-aware work map (below), 0: plain (env CWDM_SG_XCD=0, A/B)
  int diag;  // timing-only diagnostics build (make SGDIAG=1, env CWDM_SG_DIAGMASK): SG_DIAG bits below
  // 3x3x3: the next chunk's fills go out after (dz, dx) group `late` - 1 of this chunk's MFMA phase
  // (0: before it).  The fills and the MFMA phase's LDS operand reads serialize on the CU's LDS
  // (tools/dma_bench.hip), so overlapping them is not free (env CWDM_SG_LATE, A/B knob)
  int late;
};
// timing-only diagnostics (results are garbage): 1 no MFMAs, 2 no halo DMA, 4 no weight DMA,
// 8 no operand LDS reads, 16 no epilogue (return after the K loop), 32 no bias loads, 64 no K-split
// hand-off (every slice runs the epilogue)
#ifdef CWDM_SG_DIAG
#define SG_DIAG(bit) ((q.diag & (bit)) != 0)
#else
#define SG_DIAG(bit) false
#endif

// counter block pre-zeroed by the caller (the U-Net plan, per forward /
// backward, thread-local for the duration of its launch list) or null
thread_local unsigned* g_sg_sync = nullptr;
constexpr int64_t kSgSyncWords = 1 << 16;   // tiles of one K-split launch (sg_split_for keeps tiles * S below)

__device__ __forceinline__ void sg_mfma(sg_f32x4& acc, const u32x4& a, const u32x4& b, bf16_t*) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                                0, 0);
}
__device__ __forceinline__ void sg_mfma(sg_f32x4& acc, const u32x4& a, const u32x4& b, f16_t*) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0, 0,
                                               0);
}

// TAPS = 27: the 3x3x3 conv; TAPS = 1: the 1x1 skip conv of a ResBlock (the
// centre tap of the same halo image and weight buffer, packed with k = 1).
// T: the 16-bit storage type (bf16 or fp16; v_mfma_f32_16x16x32_{bf16,f16})
template <typename T, int BX, int BY, int MODE, int TAPS>
__global__ void __launch_bounds__(256) conv3d_sg_kernel(SGParams q) {
  static_assert(TAPS == 27 || TAPS == 1, "3x3x3 or 1x1");
  constexpr int PAD = TAPS == 27 ? 1 : 0;
  using C = SGCfg<BX, BY, PAD>;
  const V4Params& p = q.v;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, kq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  V4_STAMP(0);
#ifdef CWDM_CONV_STAMPS
  if (p.stamps && tid == 0) {
    p.stamps[(long long)blockIdx.x * 24 + 20] = __builtin_amdgcn_s_memrealtime();
    p.stamps[(long long)blockIdx.x * 24 + 22] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
    p.stamps[(long long)blockIdx.x * 24 + 23] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
  }
#endif

  // work item -> (batch, brick, 16-channel tile); channel tile fastest.  The
  // hardware deals consecutive workgroups to the 8 XCDs round robin, so with the
  // plain map XCD j ran channel tiles j, j + 8 of EVERY brick and fetched every
  // brick's halo into its own L2 (8x the halo traffic; at 28^3 x 128 channels
  // ~128 MB per conv from MALL).  XCD-aware: XCD j runs one contiguous run of
  // work items -- whole bricks with all their channel tiles (and K slices), so
  // a halo is fetched into one L2 and the tiles' weights stay L2-resident.
  int wi = blockIdx.x;
  if (q.xcd) {
    const int n = (int)gridDim.x, xj = wi & 7, q8 = n >> 3, r8 = n & 7;
    wi = (xj < r8 ? xj * (q8 + 1) : r8 * (q8 + 1) + (xj - r8) * q8) + (wi >> 3);
  }
  const int t16 = wi % q.ntile16;
  const int ks = (wi / q.ntile16) % q.ksplit;
  const int st = wi / (q.ntile16 * q.ksplit);
  const int b = st / q.parts, brick = st - b * q.parts;
  const int tx = q.tx, ty = q.ty;
  const int x0 = (brick % tx) * BX, y0 = ((brick / tx) % ty) * BY, z0 = (brick / (tx * ty)) * 4;
  const int SH = MODE == 1 ? p.H >> 1 : p.H, SW = MODE == 1 ? p.W >> 1 : p.W;
  const int nch = p.nch / 2;  // 32-channel chunks
  const int cb0 = ks * q.kper, cb1 = min(nch, cb0 + q.kper);  // this slice's chunks

  // halo DMA of 32-channel chunk c into buffer hbuf: pieces pc = wv + 4 j (44 in
  // all: 16-channel sub-chunk 2c + pc / (2 PCS), 32-slot block pc % (2 PCS)),
  // lane = (slot 32 blk + lane / 2, quad lane & 1)
  auto issue_halo = [&](int c, int hbuf) {
    if (SG_DIAG(2)) return;
    unsigned char* hb = smem + hbuf * C::BUF;
#pragma unroll
    for (int j = 0; j < C::PCS; ++j) {
      const int pc = wv + 4 * j;
      const int sub = pc / (2 * C::PCS), blk = pc - sub * (2 * C::PCS);
      const int hv = blk * 32 + (lane >> 1);
      const int qd = 2 * sub + (lane & 1);
      if (hv >= C::HV) continue;  // padding slots
      int sv = -1;
      {
        const int hx = hv % C::HX, hy = (hv / C::HX) % C::HY, hz = hv / (C::HX * C::HY);
        int ox = x0 + hx - PAD, oy = y0 + hy - PAD, oz = z0 + hz - PAD;
        if (ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) {
          if (MODE == 1) { ox >>= 1; oy >>= 1; oz >>= 1; }
          sv = (oz * SH + oy) * SW + ox;
        }
      }
      const int sc = 2 * c + (qd >> 1);  // 16-channel sub-chunk
      const bool s0 = sc < p.nch0;
      const unsigned char* base = s0 ? reinterpret_cast<const unsigned char*>(p.a0) + (long long)b * p.a0_bstride
                                     : reinterpret_cast<const unsigned char*>(p.a1) + (long long)b * p.a1_bstride;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(s0 ? p.a0_bytes : p.a1_bytes), 0x00020000);
      const bool cm = s0 && p.a0_cm;
      const unsigned rowb = cm ? 32u : (unsigned)(s0 ? p.ac0 : p.ac1) * 2u;
      const unsigned cofs = cm ? (unsigned)sc * (unsigned)p.a0_cvox * 32u : (unsigned)((s0 ? sc : sc - p.nch0) * 32);
      const unsigned voff = sv >= 0 ? (unsigned)sv * rowb + cofs + (unsigned)((qd & 1) * 16) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(hb + pc * 1024), 16, voff,
                                               0, 0, 0);
    }
  };

  // A fragments of chunk c into weight buffer wbuf by LDS-DMA: piece = tap t
  // (wave wv issues taps wv + 4 j), lane (kq, l16) = row t16 * 16 + l16 of the
  // packed 64-row tile, sub-chunk 2c + (kq >> 1), quad kq & 1: the A operand
  // layout, so a lane's ds_read_b128 of [t][lane] is its fragment
  const int ct64 = t16 >> 2, row = (t16 & 3) * 16 + l16;
  const unsigned wlane = (unsigned)(row * 32 + (((kq & 1) ^ ((row >> 3) & 1)) << 4));
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.aw + (long long)ct64 * p.nch * TAPS * 2048), (short)0, p.nch * TAPS * 2048, 0x00020000);
  auto issue_w = [&](int c, int wbuf) {
    if (SG_DIAG(4)) return;
    unsigned char* wb = smem + 2 * C::BUF + wbuf * C::WBUF;
    const unsigned cb = (unsigned)((2 * c + (kq >> 1)) * TAPS) * 2048u + wlane;
#pragma unroll
    for (int j = 0; j < (TAPS + 3) / 4; ++j) {
      const int t = wv + 4 * j;
      if (t < TAPS)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(wb + t * 1024), 16,
                                                 cb + (unsigned)t * 2048u, 0, 0, 0);
    }
  };

  // lane read base: halo slot of (plane wv, operand line yl, x), quad kq
  const int xl = l16 % BX, yl = l16 / BX;
  const int hlane = (kq >> 1) * C::SUB + (kq & 1) * 16 + ((wv * C::HY + yl) * C::HX + xl) * 32;

  sg_f32x4 acc[4];
  {
    float bi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      bi[i] = (p.bias && q.ksplit == 1 && !SG_DIAG(32)) ? p.bias[(long long)b * p.bias_bs + t16 * 16 + 4 * kq + i] : 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = sg_f32x4{bi[0], bi[1], bi[2], bi[3]};
  }

  issue_halo(cb0, 0);
  issue_w(cb0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V4_STAMP(1);
  for (int c = cb0; c < cb1; ++c) {
    const bool has_next = c + 1 < cb1;
    const int buf = (c - cb0) & 1;
    const unsigned char* hb = smem + buf * C::BUF + hlane;
    const unsigned char* wb = smem + 2 * C::BUF + buf * C::WBUF + lane * 16;
    u32x4 av[2][C::NR], aw[2][3];
    auto read_group = [&](u32x4 (&a)[C::NR], u32x4 (&w)[3], int g) {
      if (SG_DIAG(8)) return;
      const int dz = g / 3, dx = g % 3;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) w[dy] = *reinterpret_cast<const u32x4*>(wb + (dz * 9 + dy * 3 + dx) * 1024);
#pragma unroll
      for (int s = 0; s < C::NR; ++s)
        a[s] = *reinterpret_cast<const u32x4*>(hb + ((dz * C::HY + s) * C::HX + dx) * 32);
    };
    if constexpr (TAPS == 27) {
      read_group(av[0], aw[0], 0);
    } else {
      // the brick image (no halo): operand lines 0 .. 3 of plane wv; the one A
      // fragment sits at tap slot 0
#pragma unroll
      for (int s2 = 0; s2 < 4 * C::LPO; s2 += C::LPO)
        av[0][s2] = *reinterpret_cast<const u32x4*>(hb + s2 * C::HX * 32);
      aw[0][0] = *reinterpret_cast<const u32x4*>(wb);
    }
    // the next chunk's halo and weights go to the other buffers (last read by
    // chunk c - 1, which every wave finished before the previous barrier)
    const int late = TAPS == 27 ? q.late : 0;
    if (has_next && late == 0) {
      issue_halo(c + 1, buf ^ 1);
      issue_w(c + 1, buf ^ 1);
    }
    if constexpr (TAPS == 27) {
#pragma unroll
      for (int g = 0; g < 9; ++g) {
        if (g + 1 < 9) read_group(av[(g + 1) & 1], aw[(g + 1) & 1], g + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (!SG_DIAG(1)) sg_mfma(acc[m], aw[g & 1][dy], av[g & 1][m * C::LPO + dy], (T*)nullptr);
        __builtin_amdgcn_sched_barrier(0);
        if (has_next && late == g + 1) {
          issue_halo(c + 1, buf ^ 1);
          issue_w(c + 1, buf ^ 1);
        }
      }
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) sg_mfma(acc[m], aw[0][0], av[0][m * C::LPO], (T*)nullptr);
    }
    if (has_next) {
      // the next chunk's halo and weights have landed; every wave is past this
      // chunk's reads of the buffers the chunk after next will fill
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    if (c - cb0 < 8) V4_STAMP(4 + c - cb0);
  }
  V4_STAMP(12);
  if (SG_DIAG(16)) return;

  if (q.ksplit > 1 && !SG_DIAG(64)) {
    // K split: publish this slice, the tile's last arrival finishes it.  Hand-off
    // across XCDs without fences: the in-launch split-K recipe of
    // cdna_hip_programming.md §5 item 2 ("sc1 (write-through) slab stores, which
    // need no release fence -> every wave s_waitcnt vmcnt(0) -> __syncthreads()
    // -> lane 0 relaxed agent fetch_add; the reducer then reads the slabs with
    // sc1 loads, EVERY load of them"), valid for any placement of a tile's slices
    // over XCDs.  A __threadfence() release / acquire per slice measured 2x slower
    // here.
    const int tile = st * q.ntile16 + t16;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        q.part + (long long)tile * q.ksplit * 4096, (short)0, q.ksplit * 4096 * 4, 0x00020000);
    const unsigned lofs = (unsigned)(wv * 4 * 64 + lane) * 16u;
#pragma unroll
    for (int m = 0; m < 4; ++m)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[m]), prs,
                                             (unsigned)ks * 16384u + lofs + (unsigned)m * 1024u, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* flag = reinterpret_cast<unsigned*>(smem);
    if (tid == 0)
      *flag = __hip_atomic_fetch_add(&q.count[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    V4_STAMP(13);
    if (*flag != (unsigned)(q.ksplit - 1)) {
      V4_STAMP(15);
#ifdef CWDM_CONV_STAMPS
      if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 24 + 21] = __builtin_amdgcn_s_memrealtime();
#endif
      return;
    }
    if (tid == 0) __hip_atomic_store(&q.count[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float bi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bi[i] = p.bias ? p.bias[(long long)b * p.bias_bs + t16 * 16 + 4 * kq + i] : 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      sg_f32x4 sum = __builtin_bit_cast(sg_f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, lofs + m * 1024u, 0, 16));
      for (int k = 1; k < q.ksplit; ++k)
        sum += __builtin_bit_cast(sg_f32x4,
                                  __builtin_amdgcn_raw_buffer_load_b128(prs, (unsigned)k * 16384u + lofs + m * 1024u, 0, 16));
      acc[m] = sum + sg_f32x4{bi[0], bi[1], bi[2], bi[3]};
    }
    V4_STAMP(14);
  }

  // epilogue: lane (l16, kq) of operand m holds channels t16 16 + 4 kq + i of
  // voxel (x0 + xl, y0 + m LPO + yl, z0 + wv)
  // (a partial brick at the grid's edge: voxels outside D x H x W computed
  // zero-padded and dropped here -- no store, no residual load, no statistics)
  const int ox = x0 + xl, oz = z0 + wv;
  const long long HW = (long long)p.H * p.W;
  float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};
  const int co = t16 * 16 + 4 * kq;
  bool inb[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) inb[m] = ox < p.W && (y0 + m * C::LPO + yl) < p.H && oz < p.D;
  // out_f32 (the accurate fast mode's K-expanded split convs, sg_fp32x): fp32 output AND residual
  uint2 rq[4];
  float4 rf[4];
  if (p.rmode >= 0) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int oy = y0 + m * C::LPO + yl;
      long long rvox = ((long long)b * p.D + oz) * HW + (long long)oy * p.W + ox;
      if (p.rmode == 1)
        rvox = (((long long)b * (p.D >> 1) + (oz >> 1)) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1);
      rq[m] = uint2{0u, 0u};
      rf[m] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (inb[m]) {
        if (p.out_f32) rf[m] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.res) + rvox * p.cout + co);
        else rq[m] = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(p.res) + rvox * p.cout + co);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int oy = y0 + m * C::LPO + yl;
    const long long vox = ((long long)b * p.D + oz) * HW + (long long)oy * p.W + ox;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[m][i];
    if (p.rmode >= 0) {
      if (p.out_f32) {
        v[0] += rf[m].x; v[1] += rf[m].y; v[2] += rf[m].z; v[3] += rf[m].w;
      } else {
        v[0] += lo2f<T>(rq[m].x); v[1] += hi2f<T>(rq[m].x);
        v[2] += lo2f<T>(rq[m].y); v[3] += hi2f<T>(rq[m].y);
      }
    }
    if (inb[m]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ssum[i] += v[i];
        ssq[i] += v[i] * v[i];
      }
      if (p.out_f32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + vox * p.cout + co) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint2 sq;
        sq.x = pack2<T>(v[0], v[1]);
        sq.y = pack2<T>(v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.out) + vox * p.cout + co) = sq;
      }
    }
  }
  if (p.stats) {
    // rows of 16 lanes hold 4 channels for 16 voxels: DPP row sums, then the 4
    // plane waves through the halo padding slots of buffer 0
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ssum[i] = row16_sum(ssum[i]);
      ssq[i] = row16_sum(ssq[i]);
    }
    __syncthreads();  // every wave is done with the halo buffers
    float* R = reinterpret_cast<float*>(smem);  // [wave][16 sums | 16 squares]
    if (l16 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        R[wv * 32 + 4 * kq + i] = ssum[i];
        R[wv * 32 + 16 + 4 * kq + i] = ssq[i];
      }
    }
    __syncthreads();
    if (tid < 16) {
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        s += R[w * 32 + tid];
        s2 += R[w * 32 + 16 + tid];
      }
      const long long pidx = ((long long)b * q.parts + brick) * p.cout + t16 * 16 + tid;
      p.stats[pidx * 2 + 0] = s;
      p.stats[pidx * 2 + 1] = s2;
    }
  }
  V4_STAMP(15);
#ifdef CWDM_CONV_STAMPS
  if (p.stamps && tid == 0) p.stamps[(long long)blockIdx.x * 24 + 21] = __builtin_amdgcn_s_memrealtime();
#endif
}

template __global__ void conv3d_sg_kernel<bf16_t, 16, 4, 0, 27>(SGParams);
template __global__ void conv3d_sg_kernel<bf16_t, 16, 4, 1, 27>(SGParams);
template __global__ void conv3d_sg_kernel<bf16_t, 16, 4, 0, 1>(SGParams);
template __global__ void conv3d_sg_kernel<bf16_t, 8, 8, 0, 27>(SGParams);
template __global__ void conv3d_sg_kernel<bf16_t, 8, 8, 1, 27>(SGParams);
template __global__ void conv3d_sg_kernel<bf16_t, 8, 8, 0, 1>(SGParams);
template __global__ void conv3d_sg_kernel<f16_t, 16, 4, 0, 27>(SGParams);
template __global__ void conv3d_sg_kernel<f16_t, 16, 4, 1, 27>(SGParams);
template __global__ void conv3d_sg_kernel<f16_t, 16, 4, 0, 1>(SGParams);
template __global__ void conv3d_sg_kernel<f16_t, 8, 8, 0, 27>(SGParams);
template __global__ void conv3d_sg_kernel<f16_t, 8, 8, 1, 27>(SGParams);
template __global__ void conv3d_sg_kernel<f16_t, 8, 8, 0, 1>(SGParams);

extern std::atomic<int> g_conv_path;
// set by the U-Net plan around the accurate fast mode's K-expanded small-grid convs: a 16-bit conv
// with fp32 output takes this kernel, its residual fp32 too (SgFp32xScope)
thread_local bool g_sg_fp32x = false;

namespace {
bool sg_shape_ok(const cwdm_conv3d_desc* d) {
  if (g_conv_path.load(std::memory_order_relaxed) == 1) return false;
  if (!dtype_half(d->dtype) || d->accumulate || d->out1 || d->cout % 64) return false;
  if (d->out_dtype != d->dtype && !(d->out_dtype == CWDM_F32 && g_sg_fp32x)) return false;
  // W < kWideMinW (the wide kernels take the rest): 16 x 4 x 4 bricks for W >= 16,
  // 8 x 8 x 4 below (pick_brick's statistics bricks), the last brick of an axis partial
  return d->W >= 1 && d->W < kWideMinW && d->H >= 1 && d->D >= 1;
}

// statistics bricks of a small grid: (bx, tx, ty, tz), parts = tx ty tz (== cwdm_conv3d_parts)
struct SgGeom { int bx, tx, ty, tz; int64_t parts() const { return (int64_t)tx * ty * tz; } };
SgGeom sg_geom(const cwdm_conv3d_desc* d) {
  const int bx = d->W >= 16 ? 16 : 8, by = 64 / bx;
  return SgGeom{bx, (int)ceil_div(d->W, bx), (int)ceil_div(d->H, by), (int)ceil_div(d->D, 4)};
}
}  // namespace

// shapes the small-grid kernel takes: bf16, plain bf16 output (no fp32 / dual /
// accumulating output), same-grid or upsampled source and residual, W = 16
// (16x4x4 statistics bricks) or W = 8 (8x8x4), 32-channel K chunks.  At 8^3
// there are only 32 tiles: K split across workgroups (sg_ksplit), finished by
// the last slice of each tile.
bool sg_eligible(const cwdm_conv3d_desc* d) {
  if (!sg_shape_ok(d) || !d->a_w) return false;
  if (d->a_mode != 0 && d->a_mode != 1) return false;
  if (d->res_mode < -1 || d->res_mode > 1) return false;
  if ((d->a_c0 + d->a_c1) % 32 || d->a_c0 % 16) return false;
  const int64_t V = d->D * d->H * d->W;
  const int64_t SV = d->a_mode == 1 ? V / 8 : V;
  return SV * (d->a_c0 + d->a_c1) * 2 < 0xFFFFE000LL && d->B * (V / 256) * (d->cout / 16) < (1LL << 31);
}

// the 1x1 skip segment alone (segment B of a desc, channels-last sources)
bool sg_skip_eligible(const cwdm_conv3d_desc* d) {
  if (!sg_shape_ok(d) || !d->b_w) return false;
  if ((d->b_c0 + d->b_c1) % 32 || d->b_c0 % 16) return false;
  const int64_t V = d->D * d->H * d->W;
  return V * (d->b_c0 + d->b_c1) * 2 < 0xFFFFE000LL && d->B * (V / 256) * (d->cout / 16) < (1LL << 31);
}

// K slices of a launch: enough work items for the chip (~256), at least one
// 32-channel chunk per slice (the 16^3 level has 256 tiles: no split)
namespace {
int sg_split_for(const cwdm_conv3d_desc* d, int cin, bool skip = false) {
  const int64_t parts = sg_geom(d).parts();
  const int64_t tiles = d->B * parts * (d->cout / 16);
  const int nch = cin / 32;
  // work-item target (env CWDM_SG_TARGET, A/B knob; 192 since r04: the 8^3
  // level splits K 4 ways instead of 8, 66.28 -> 66.54 steps/s on one box,
  // config 5 unchanged -- profiles/r04/g_sg_target_ab.txt); the 1x1 skips' own
  // (env CWDM_SG_SKIP_TARGET, A/B knob, default the same)
  static const int64_t target3 = [] { const char* e = std::getenv("CWDM_SG_TARGET"); return e ? std::atoll(e) : 192LL; }();
  static const int64_t target1 = [] { const char* e = std::getenv("CWDM_SG_SKIP_TARGET"); return e ? std::atoll(e) : target3; }();
  const int64_t target = skip ? target1 : target3;
  if (tiles >= target || nch < 2) return 1;
  int S = (int)std::min<int64_t>((target + tiles - 1) / tiles, nch);
  const int per = (nch + S - 1) / S;
  S = (nch + per - 1) / per;
  return (tiles * S < (1 << 16) && S > 1) ? S : 1;
}
}  // namespace

int sg_ksplit(const cwdm_conv3d_desc* d) { return sg_eligible(d) ? sg_split_for(d, d->a_c0 + d->a_c1) : 1; }
// voxels per batch of one K-split slice: the small-grid kernel stores whole
// (possibly partial) bricks of 256 voxels, the wide kernel the grid itself
int64_t ksplit_slice_voxels(const cwdm_conv3d_desc* d) {
  return sg_shape_ok(d) ? sg_geom(d).parts() * 256 : d->D * d->H * d->W;
}
int sg_skip_ksplit(const cwdm_conv3d_desc* d) { return sg_skip_eligible(d) ? sg_split_for(d, d->b_c0 + d->b_c1, true) : 1; }

// bytes of the K-split counter block a lone launch keeps behind its slices (0 without a split)
int64_t sg_sync_bytes(int ksplit) { return ksplit > 1 ? kSgSyncWords * 4 : 0; }
// the U-Net plan's zeroed sync block: the small-grid K-split counters, then the
// warp-specialised conv's apply-ahead sweep counters (kV5AaWords)
int64_t plan_sync_bytes() { return kSgSyncWords * 4 + kV5AaWords * 4; }
unsigned* plan_aa_counters() { return g_sg_sync ? g_sg_sync + kSgSyncWords : nullptr; }

namespace {
// counters of a K-split launch: the plan's pre-zeroed block, else `own` (the
// workspace tail behind the slices), zeroed here by a memset node
int sg_counters(SGParams& q, void* own, hipStream_t s) {
  q.count = nullptr;
  if (q.ksplit == 1) return CWDM_OK;
  const int64_t tiles = (int64_t)q.v.B * q.parts * q.ntile16;
  CWDM_REQUIRE(tiles <= kSgSyncWords, CWDM_E_UNSUPPORTED, "conv3d (small grid): too many K-split tiles");
  if (g_sg_sync) {
    q.count = g_sg_sync;
    return CWDM_OK;
  }
  CWDM_REQUIRE(own, CWDM_E_INVALID, "conv3d (small grid): K-split counters missing");
  q.count = reinterpret_cast<unsigned*>(own);
  CWDM_HIP(hipMemsetAsync(own, 0, (size_t)((tiles * 4 + 15) & ~15LL), s));
  return CWDM_OK;
}

template <typename T>
void sg_go_t(const SGParams& q, const cwdm_conv3d_desc* d, int taps, hipStream_t s) {
  const dim3 grid((unsigned)(d->B * q.parts * q.ntile16 * q.ksplit));
  const bool w8 = sg_geom(d).bx == 8;
  if (w8 && taps == 1) {
    hipLaunchKernelGGL((conv3d_sg_kernel<T, 8, 8, 0, 1>), grid, dim3(256), 0, s, q);
  } else if (w8) {
    if (q.v.amode == 1) hipLaunchKernelGGL((conv3d_sg_kernel<T, 8, 8, 1, 27>), grid, dim3(256), 0, s, q);
    else hipLaunchKernelGGL((conv3d_sg_kernel<T, 8, 8, 0, 27>), grid, dim3(256), 0, s, q);
  } else if (taps == 1) {
    hipLaunchKernelGGL((conv3d_sg_kernel<T, 16, 4, 0, 1>), grid, dim3(256), 0, s, q);
  } else if (q.v.amode == 1) {
    hipLaunchKernelGGL((conv3d_sg_kernel<T, 16, 4, 1, 27>), grid, dim3(256), 0, s, q);
  } else {
    hipLaunchKernelGGL((conv3d_sg_kernel<T, 16, 4, 0, 27>), grid, dim3(256), 0, s, q);
  }
}

int sg_go(const SGParams& q0, const cwdm_conv3d_desc* d, int taps, double flops, hipStream_t s) {
  static const int xcd_map = [] { const char* e = std::getenv("CWDM_SG_XCD"); return !(e && e[0] == '0'); }();
  SGParams q = q0;
  q.xcd = xcd_map;
  // default 4: after the 4th of 9 groups (r06 same box: 16^3 convs 567 -> 523 us per step, 8^3 347 -> 332,
  // 15.36 -> 15.28 ms; conv_bench 16^3 -8 %, all-after-the-phase (9) -5 %)
  static const int late = [] { const char* e = std::getenv("CWDM_SG_LATE"); return e ? std::atoi(e) : 4; }();
  q.late = late < 0 ? 0 : (late > 9 ? 9 : late);
#ifdef CWDM_SG_DIAG
  static const int diag = [] { const char* e = std::getenv("CWDM_SG_DIAGMASK"); return e ? std::atoi(e) : 0; }();
  q.diag = diag;
#endif
  prof_begin(s);
  if (d->dtype == CWDM_F16) sg_go_t<f16_t>(q, d, taps, s);
  else sg_go_t<bf16_t>(q, d, taps, s);
  prof_end(s, flops);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
}  // namespace

// partial: fp32 scratch of sg_ksplit(d) x B x V x cout (the K-split slices) followed
// by sg_sync_bytes of counters, else unused
int sg_launch(const V4Params& v, const cwdm_conv3d_desc* d, void* partial, hipStream_t s) {
  SGParams q{};
  q.v = v;
  q.ntile16 = d->cout / 16;
  const SgGeom gm = sg_geom(d);
  q.parts = (int)gm.parts();
  q.tx = gm.tx; q.ty = gm.ty;
  q.ksplit = sg_ksplit(d);
  q.kper = ((d->a_c0 + d->a_c1) / 32 + q.ksplit - 1) / q.ksplit;
  q.part = reinterpret_cast<float*>(partial);
  CWDM_REQUIRE(q.ksplit == 1 || partial, CWDM_E_INVALID, "conv3d (small grid): K-split scratch missing");
  int rc;
  if ((rc = sg_counters(q, q.ksplit > 1 ? reinterpret_cast<unsigned char*>(partial) +
                                              (int64_t)q.ksplit * d->B * ksplit_slice_voxels(d) * d->cout * 4
                                        : nullptr, s)))
    return rc;
  return sg_go(q, d, 27, 2.0 * d->B * d->D * d->H * d->W * (double)d->cout * 27.0 * (d->a_c0 + d->a_c1), s);
}

// out = W_skip . [b0 | b1] (bf16, no bias / residual / statistics): the skip
// pre-pass of conv3d_v4_forward; partial: fp32 scratch of sg_skip_ksplit(d) x B x V x cout
int sg_skip_launch(const cwdm_conv3d_desc* d, void* out, void* partial, hipStream_t s) {
  SGParams q{};
  V4Params& p = q.v;
  const int64_t V = d->D * d->H * d->W;
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W;
  p.cout = d->cout; p.nct = d->cout / 64;
  p.nch0 = d->b_c0 / 16; p.nch = (d->b_c0 + d->b_c1) / 16;
  p.a0 = d->b0; p.ac0 = d->b_c0; p.a1 = d->b1; p.ac1 = d->b_c1;
  p.a0_bstride = V * d->b_c0 * 2; p.a1_bstride = V * d->b_c1 * 2;
  p.a0_bytes = (unsigned)(V * d->b_c0 * 2); p.a1_bytes = (unsigned)(V * d->b_c1 * 2);
  p.amode = 0; p.a0_cm = 0; p.a0_cvox = (int)V;
  p.aw = reinterpret_cast<const unsigned char*>(d->b_w);
  p.bias = nullptr; p.res = nullptr; p.rmode = -1;
  p.out = out; p.stats = nullptr;
  p.out_f32 = (d->out_dtype == CWDM_F32) ? 1 : 0;   // (the accurate fast mode's K-expanded skip, sg_shape_ok)
  q.ntile16 = d->cout / 16;
  const SgGeom gm = sg_geom(d);
  q.parts = (int)gm.parts();
  q.tx = gm.tx; q.ty = gm.ty;
  q.ksplit = sg_skip_ksplit(d);
  q.kper = ((d->b_c0 + d->b_c1) / 32 + q.ksplit - 1) / q.ksplit;
  q.part = reinterpret_cast<float*>(partial);
  CWDM_REQUIRE(q.ksplit == 1 || partial, CWDM_E_INVALID, "conv3d (small grid): K-split scratch missing");
  int rc;
  if ((rc = sg_counters(q, q.ksplit > 1 ? reinterpret_cast<unsigned char*>(partial) +
                                              (int64_t)q.ksplit * d->B * ksplit_slice_voxels(d) * d->cout * 4
                                        : nullptr, s)))
    return rc;
  return sg_go(q, d, 1, 2.0 * d->B * V * (double)d->cout * (d->b_c0 + d->b_c1), s);
}

}  // namespace cwdm
