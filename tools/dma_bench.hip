// Per-CU LDS fill rate by instruction form (why the small-grid conv's chunk fetch runs at ~8.6 B/clk
// per CU, tools/sg_stamps.py): one 256-thread workgroup per CU (144 KB of LDS, as the small-grid
// conv), every wave issues NI 1-KB fills per round (16 B per lane), waits vmcnt(0), barrier; R rounds.
// Forms: 0 buffer_load_dwordx4 ... lds (per-lane voffset), 1 global_load_lds_dwordx4 (per-lane address),
// 2 global_load_dwordx4 to VGPRs + ds_write_b128, 3 form 0 with each lane on its own 128-B line.
// Source: a buffer of SRC bytes read round-robin (2 MB: L2-resident; 64 MB: Infinity Cache; 1 GB: HBM).
// build: hipcc --offload-arch=gfx950 -O3 tools/dma_bench.hip -o tools/dma_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// NR > 0: after issuing a round's fills every wave also runs NR ds_read_b128 of the previous round's
// image (the small-grid conv's MFMA-phase operand traffic) before it waits for the fills
template <int FORM, int NI, int NR = 0>
__global__ void __launch_bounds__(256) fill(const unsigned char* src, unsigned long long src_bytes, int rounds,
                                            unsigned* sink) {
  __shared__ __attribute__((aligned(1024))) unsigned char sm[144 * 1024];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)0x7FFFFFF0, 0x00020000);
  // this workgroup's window: 64 KB * NI per round, advancing
  unsigned long long base = ((unsigned long long)blockIdx.x * 4 * NI * 1024) % src_bytes;
  unsigned acc = 0;
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int pc = wv * NI + j;                      // piece index within the round (1 KB each)
      unsigned long long off = (base + (unsigned long long)pc * 1024 + (FORM == 3 ? lane * 128 : lane * 16)) % src_bytes;
      unsigned char* dst = sm + (pc % 144) * 1024;
      if constexpr (FORM == 0 || FORM == 3) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, (unsigned)off, 0, 0, 0);
      } else if constexpr (FORM == 1) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off),
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      } else {
        const u32x4 v = *reinterpret_cast<const u32x4*>(src + off);
        *reinterpret_cast<u32x4*>(dst + lane * 16) = v;
      }
    }
    if constexpr (NR > 0) {
      u32x4 t = {0u, 0u, 0u, 0u};
#pragma unroll 8
      for (int k = 0; k < NR; ++k) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(sm + ((wv * NR + k) * 1024 + lane * 16) % (144 * 1024));
        t ^= v;
      }
      acc += t[0] ^ t[1] ^ t[2] ^ t[3];
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    acc += *reinterpret_cast<const unsigned*>(sm + (tid * 64) % (144 * 1024));
    base = (base + (unsigned long long)gridDim.x * 4 * NI * 1024) % src_bytes;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int FORM, int NI, int NR = 0>
double run(const unsigned char* src, unsigned long long bytes, int grid, unsigned* sink) {
  const int rounds = 200;
  hipLaunchKernelGGL((fill<FORM, NI, NR>), dim3(grid), dim3(256), 0, 0, src, bytes, 4, sink);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL((fill<FORM, NI, NR>), dim3(grid), dim3(256), 0, 0, src, bytes, rounds, sink);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double per_cu = (double)rounds * 4 * NI * 1024 / (ms * 1e-3);   // bytes/s per workgroup (= per CU)
  return per_cu / 1e9;
}

int main() {
  unsigned char* src;
  const unsigned long long big = 1ull << 30;
  hipMalloc(&src, big);
  hipMemset(src, 1, big);
  unsigned* sink;
  hipMalloc(&sink, 64);
  const unsigned long long sizes[] = {2ull << 20, 64ull << 20, 1ull << 30};
  const char* names[] = {"2MB(L2)", "64MB(MALL)", "1GB(HBM)"};
  for (int si = 0; si < 3; ++si) {
    for (int grid : {256, 128}) {
      printf("%-11s grid %3d  GB/s per CU | NI=4: buf %.1f glb %.1f reg %.1f scat %.1f | NI=16: buf %.1f glb %.1f reg %.1f scat %.1f\n",
             names[si], grid, run<0, 4>(src, sizes[si], grid, sink), run<1, 4>(src, sizes[si], grid, sink),
             run<2, 4>(src, sizes[si], grid, sink), run<3, 4>(src, sizes[si], grid, sink),
             run<0, 16>(src, sizes[si], grid, sink), run<1, 16>(src, sizes[si], grid, sink),
             run<2, 16>(src, sizes[si], grid, sink), run<3, 16>(src, sizes[si], grid, sink));
    }
  }
  // contention: 16 fills per wave in flight while the wave reads NR x 1 KB of LDS (the small-grid conv
  // reads ~81 per wave per chunk in its MFMA phase), 64 MB source
  printf("64MB(MALL)  grid 256  NI=16 buf, LDS reads per wave per round: 0 %.1f | 32 %.1f | 81 %.1f | 160 %.1f GB/s per CU\n",
         run<0, 16, 0>(src, sizes[1], 256, sink), run<0, 16, 32>(src, sizes[1], 256, sink),
         run<0, 16, 81>(src, sizes[1], 256, sink), run<0, 16, 160>(src, sizes[1], 256, sink));
  printf("2MB(L2)     grid 256  NI=16 buf, LDS reads per wave per round: 0 %.1f | 32 %.1f | 81 %.1f | 160 %.1f GB/s per CU\n",
         run<0, 16, 0>(src, sizes[0], 256, sink), run<0, 16, 32>(src, sizes[0], 256, sink),
         run<0, 16, 81>(src, sizes[0], 256, sink), run<0, 16, 160>(src, sizes[0], 256, sink));
  return 0;
}
