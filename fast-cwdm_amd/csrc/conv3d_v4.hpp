// Conv3d 3x3x3 (stride 1, pad 1) implicit GEMM, DMA-staged variant for the
// wide U-Net levels (W % 32 == 0, H % 4 == 0, D % 4 == 0, cout % 64 == 0).
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
//     fragments (16 B of one output channel) straight into VGPRs, two groups
//     ahead, through a 3-deep register ring with counted vmcnt waits.
//   * The halo is double-buffered (the next chunk's DMA is issued at the top
//     of the current chunk): one raw s_barrier per chunk, no exposed DMA
//     latency.  Two workgroups share a CU (80 KB LDS each, <= 256 registers
//     per lane), so one workgroup's barrier and epilogue hide under the
//     other's MFMAs.
//   * Epilogue from registers: + bias, + residual (same / upsampled grid),
//     store (or accumulate), per-channel (sum, sum^2) partials for the next
//     GroupNorm, reduced across lanes with DPP and across waves in LDS.
#pragma once
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
  const unsigned char* aw;            // packed weights, NT = 64
  const float* bias; long long bias_bs;
  const void* res; int rmode;         // -1 none, 0 same grid, 1 upsampled
  void* out; int out_f32;
  float* stats;
  void* out1; int out_c0;
  int accumulate;
};

struct V4Cfg {
  static constexpr int HX = 34, HY = 6, HZ = 6, HV = HX * HY * HZ;  // 1224 halo voxels
  static constexpr int HVP = 1280;                                   // slots per quad plane (20 pieces)
  static constexpr int PIECES = 2 * HVP / 64;                        // 40 DMA pieces per chunk
  static constexpr int HALO_B = 2 * HVP * 16;                        // 40960 per buffer
  static constexpr int SMEM = 2 * HALO_B;                            // double-buffered halo: 80 KB
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
#define V4_WAIT_W(n, w) \
  asm volatile("s_waitcnt vmcnt(" #n ")" : "+v"((w)[0]), "+v"((w)[1]), "+v"((w)[2]) :: "memory")

// sum of v over the 32 lanes of each half-wave (lanes 0-31 / 32-63), result in
// every lane of the half
__device__ __forceinline__ float halfwave_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));  // quad_perm 1,0,3,2
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));  // quad_perm 2,3,0,1
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true)); // row_half_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true)); // row_mirror
  v += __shfl_xor(v, 16, 64);
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

template <typename T, int MODE>
__global__ void __launch_bounds__(256, 2) conv3d_v4_kernel(V4Params p) {
  using C = V4Cfg;
  constexpr int CK = ConvTr<T>::CK;
  constexpr int ESZ = sizeof(T);
  __shared__ __attribute__((aligned(1024))) unsigned char smem[C::SMEM];

  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, hh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int f = wv & 1, vg = wv >> 1;

  // XCD-aware, bijective block -> (spatial tile, channel tile) map: each XCD
  // gets a contiguous run of tiles (x fastest), so halo neighbours share its L2
  const int nblk = gridDim.x;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ct = wg % p.nct;
  const int st = wg / p.nct;
  const int tiles = p.tx * p.ty * p.tz;
  const int b = st / tiles;
  const int sl = st - b * tiles;
  const int x0 = (sl % p.tx) * 32, y0 = ((sl / p.tx) % p.ty) * 4, z0 = (sl / (p.tx * p.ty)) * 4;

  // ---- per-lane source voxel of this wave's 10 halo pieces (chunk-invariant)
  const int SH = MODE == 1 ? p.H >> 1 : p.H, SW = MODE == 1 ? p.W >> 1 : p.W;
  int svox[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const int pc = wv + 4 * j;                 // piece id (wave-uniform)
    const int hv = (pc % 20) * 64 + lane;      // slot in the quad plane
    int sv = -1;
    if (hv < C::HV) {
      const int hx = hv % C::HX, hy = (hv / C::HX) % C::HY, hz = hv / (C::HX * C::HY);
      int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
      if (ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D) {
        if (MODE == 1) { ox >>= 1; oy >>= 1; oz >>= 1; }
        sv = (oz * SH + oy) * SW + ox;
      }
    }
    svox[j] = sv;
  }
  const unsigned char* a0b = reinterpret_cast<const unsigned char*>(p.a0) + (long long)b * p.a0_bstride;
  const unsigned char* a1b = p.a1 ? reinterpret_cast<const unsigned char*>(p.a1) + (long long)b * p.a1_bstride : a0b;
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a0b, (short)0, (int)p.a0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)a1b, (short)0, (int)p.a1_bytes, 0x00020000);

  // issue the 10 halo pieces of chunk c into halo buffer c & 1
  auto issue_halo = [&](int c) {
    const bool s0 = c < p.nch0;
    const int cs = s0 ? p.ac0 : p.ac1;
    const int cb = (s0 ? c : c - p.nch0) * CK;
    const unsigned rowb = (unsigned)cs * ESZ;
    unsigned char* hb = smem + (c & 1) * C::HALO_B;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int pc = wv + 4 * j;
      const int qd = pc / 20;
      const unsigned voff = svox[j] >= 0 ? (unsigned)svox[j] * rowb + (unsigned)(cb * ESZ + qd * 16) : 0xFFFFFFF0u;
      unsigned char* dst = hb + pc * 1024;
      if (s0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs0, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs1, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0, 0);
    }
  };
  // weight fragments of group G (chunk G / 9, (dz, dx) = G % 9): the 3 dy taps,
  // this lane's row (output channel) lr of the wave's 32-channel slice, quad hh
  const int total = 9 * p.nch;
  const unsigned char* wlane =
      p.aw + (long long)ct * p.nch * 27 * 2048 + f * 1024 + lr * 32 + ((hh ^ ((lr >> 3) & 1)) << 4);
  auto load_w = [&](u32x4 (&w)[3], int G) {
    G = G < total ? G : total - 1;  // past the end: harmless reload keeps the wait counts uniform
    const int c = G / 9, g = G - 9 * c;
    const unsigned char* src = wlane + ((long long)c * 27 + (g / 3) * 9 + (g % 3)) * 2048;
    v4_gload(w[0], src);
    v4_gload(w[1], src + 3 * 2048);
    v4_gload(w[2], src + 6 * 2048);
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][m][i] = 0.f;

  // lane read base: halo voxel (z = 2 vg, line 0, x = lr) of quad plane hh
  const int hlane = hh * (C::HVP * 16) + ((2 * vg) * (C::HX * C::HY) + lr) * 16;

  u32x4 wr[3][3];
  load_w(wr[0], 0);
  load_w(wr[1], 1);
  issue_halo(0);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[0][2]), "+v"(wr[1][0]),
               "+v"(wr[1][1]), "+v"(wr[1][2])::"memory");
  __builtin_amdgcn_s_barrier();
  for (int c = 0; c < p.nch; ++c) {
    const unsigned char* hb = smem + (c & 1) * C::HALO_B + hlane;
    // 18 steps per chunk: step K = (group K / 2, plane K % 2).  The 6 halo
    // lines of step K + 1 are read before the 12 MFMAs of step K (software
    // pipeline, pinned by sched_barrier), so every MFMA block finds its
    // operands already in registers.
    u32x4 av[2][6];
    v4_read_step<0>(av[0], hb);
#define V4_STEP(K)                                                                                            \
    {                                                                                                         \
      constexpr int GI = (K) / 2, PL = (K) % 2;                                                               \
      if (PL == 0) {                                                                                          \
        if (GI == 0 && c + 1 < p.nch) issue_halo(c + 1);                                                      \
        load_w(wr[(GI + 2) % 3], 9 * c + GI + 2);                                                             \
      }                                                                                                       \
      if ((K) < 17) v4_read_step<((K) + 1) % 18>(av[((K) + 1) & 1], hb);                                      \
      if (PL == 0 && GI >= 2) V4_WAIT_W(6, wr[GI % 3]);                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                                      \
      _Pragma("unroll") for (int dy = 0; dy < 3; ++dy)                                                        \
      _Pragma("unroll") for (int m = 0; m < 4; ++m)                                                           \
        v4_mfma<T>(acc[PL][m], wr[GI % 3][dy], av[(K) & 1][m + dy]);                                          \
      __builtin_amdgcn_sched_barrier(0);                                                                      \
    }
    V4_STEP(0) V4_STEP(1) V4_STEP(2) V4_STEP(3) V4_STEP(4) V4_STEP(5)
    V4_STEP(6) V4_STEP(7) V4_STEP(8) V4_STEP(9) V4_STEP(10) V4_STEP(11)
    V4_STEP(12) V4_STEP(13) V4_STEP(14) V4_STEP(15) V4_STEP(16) V4_STEP(17)
#undef V4_STEP
    // next chunk: its halo (issued at group 0) and its first two weight groups
    // (issued at groups 7, 8) must have landed; then every wave is past this
    // chunk's reads of the buffer the following chunk's halo will overwrite
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[0][2]), "+v"(wr[1][0]),
                 "+v"(wr[1][1]), "+v"(wr[1][2])::"memory");
    __builtin_amdgcn_s_barrier();
  }

  // ---------------- epilogue (from registers) ----------------
  const int cbase = ct * 64 + f * 32 + 4 * hh;   // + 8 j + k
  float bia[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int co = cbase + 8 * (i >> 2) + (i & 3);
    bia[i] = p.bias ? p.bias[(long long)b * p.bias_bs + co] : 0.f;
  }
  float ssum[16], ssq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { ssum[i] = 0.f; ssq[i] = 0.f; }
  const int ox = x0 + lr;
#pragma unroll
  for (int pl = 0; pl < 2; ++pl) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int oy = y0 + m, oz = z0 + 2 * vg + pl;
      const long long vox = (((long long)b * p.D + oz) * p.H + oy) * p.W + ox;
      long long rvox = vox;
      if (p.rmode == 1)
        rvox = (((long long)b * (p.D >> 1) + (oz >> 1)) * (p.H >> 1) + (oy >> 1)) * (p.W >> 1) + (ox >> 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = cbase + 8 * j;
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = acc[pl][m][4 * j + k] + bia[4 * j + k];
        if (p.rmode >= 0) {
          const T* r = reinterpret_cast<const T*>(p.res) + rvox * p.cout + co;
          if constexpr (sizeof(T) == 2) {
            const uint2 rq = *reinterpret_cast<const uint2*>(r);
            v[0] += __uint_as_float(rq.x << 16); v[1] += __uint_as_float(rq.x & 0xffff0000u);
            v[2] += __uint_as_float(rq.y << 16); v[3] += __uint_as_float(rq.y & 0xffff0000u);
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
        if (p.out_f32) {
          float* o = reinterpret_cast<float*>(obase) + vox * ostride + oc;
          if (p.accumulate) {
            const float4 oq = *reinterpret_cast<const float4*>(o);
            v[0] += oq.x; v[1] += oq.y; v[2] += oq.z; v[3] += oq.w;
          }
          *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        } else if constexpr (sizeof(T) == 2) {
          bf16_t* o = reinterpret_cast<bf16_t*>(obase) + vox * ostride + oc;
          if (p.accumulate) {
            const uint2 oq = *reinterpret_cast<const uint2*>(o);
            v[0] += __uint_as_float(oq.x << 16); v[1] += __uint_as_float(oq.x & 0xffff0000u);
            v[2] += __uint_as_float(oq.y << 16); v[3] += __uint_as_float(oq.y & 0xffff0000u);
          }
          uint2 sq;
          sq.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
          sq.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
          *reinterpret_cast<uint2*>(o) = sq;
        } else {
          float* o = reinterpret_cast<float*>(obase) + vox * ostride + oc;
          if (p.accumulate) {
            const float4 oq = *reinterpret_cast<const float4*>(o);
            v[0] += oq.x; v[1] += oq.y; v[2] += oq.z; v[3] += oq.w;
          }
          *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ssum[4 * j + k] += v[k];
          ssq[4 * j + k] += v[k] * v[k];
        }
      }
    }
  }
  if (p.stats) {
    // lanes of a half-wave hold the same 16 channels for 32 different voxels
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ssum[i] = halfwave_sum(ssum[i]);
      ssq[i] = halfwave_sum(ssq[i]);
    }
    float* R = reinterpret_cast<float*>(smem);  // [vg][64 ch][2]
    if (lr == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int cl = f * 32 + 4 * hh + 8 * (i >> 2) + (i & 3);
        R[(vg * 64 + cl) * 2 + 0] = ssum[i];
        R[(vg * 64 + cl) * 2 + 1] = ssq[i];
      }
    }
    __syncthreads();
    if (tid < 64) {
      const int c = ct * 64 + tid;
      const long long pidx = ((long long)b * tiles + sl) * p.cout + c;
      p.stats[pidx * 2 + 0] = R[tid * 2 + 0] + R[(64 + tid) * 2 + 0];
      p.stats[pidx * 2 + 1] = R[tid * 2 + 1] + R[(64 + tid) * 2 + 1];
    }
  }
}

}  // namespace cwdm
