// MFMA shape under DVFS on this chip (MI355X_MICROARCH.md 'DVFS give-back' item 7):
// v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_16x16x32_bf16 at the same output
// tile per wave (64 x 64 outputs: 4 accumulators of 32x32 or 16 of 16x16), the
// same K per step and the same LDS read bytes (operands re-read from LDS every
// step, 2 waves per SIMD like the DMA conv kernel), on random bf16 data.
// Evidence for the next conv-kernel step.
// build: hipcc -O3 --offload-arch=gfx950 tools/mfma_shape_bench.hip -o tools/mfma_shape_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

constexpr int LDSB = 32 * 1024;

// per step: K = 32 per output element (two K-16 MFMAs of 32x32 or one K-32 of 16x16)
template <int SHAPE>
__global__ void __launch_bounds__(256, 2) shape_kernel(const u32x4* __restrict__ src, int steps, float* out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDSB];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < LDSB / 16; i += 256) reinterpret_cast<u32x4*>(lds)[i] = src[(blockIdx.x * 97 + i) % 65536];
  __syncthreads();
  const int wv = tid >> 6;
  const unsigned char* base = lds + wv * 4096 + lane * 16;
  if constexpr (SHAPE == 32) {
    f32x16 acc[2][2];
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
    for (int s = 0; s < steps; ++s) {
      const int o = (s & 7) * 1024;
      u32x4 A[2][2], B[2][2];  // [k half][m / n tile]
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          A[k][t] = *reinterpret_cast<const u32x4*>(base + ((o + k * 2048 + t * 512) & (LDSB - 4096 - 1)));
          B[k][t] = *reinterpret_cast<const u32x4*>(base + ((o + k * 2048 + t * 512 + 256) & (LDSB - 4096 - 1)));
        }
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, A[k][a]),
                                                                __builtin_bit_cast(bf16x8, B[k][b]), acc[a][b], 0, 0, 0);
    }
    float r = 0.f;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int i = 0; i < 16; ++i) r += acc[a][b][i];
    out[blockIdx.x * 256 + tid] = r;
  } else {
    f32x4 acc[4][4];
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b)
        for (int i = 0; i < 4; ++i) acc[a][b][i] = 0.f;
    for (int s = 0; s < steps; ++s) {
      const int o = (s & 7) * 1024;
      u32x4 A[4], B[4];  // 16 x 32 operands: same bytes per step as the 32x32 form
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        A[t] = *reinterpret_cast<const u32x4*>(base + ((o + t * 512) & (LDSB - 4096 - 1)));
        B[t] = *reinterpret_cast<const u32x4*>(base + ((o + t * 512 + 256) & (LDSB - 4096 - 1)));
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, A[a]),
                                                              __builtin_bit_cast(bf16x8, B[b]), acc[a][b], 0, 0, 0);
    }
    float r = 0.f;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b)
        for (int i = 0; i < 4; ++i) r += acc[a][b][i];
    out[blockIdx.x * 256 + tid] = r;
  }
}

int main() {
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<unsigned> h(65536 * 4);
  unsigned x = 12345u;
  for (auto& v : h) {  // random bf16 pairs in about [-2, 2]
    x = x * 1664525u + 1013904223u;
    unsigned lo = 0x3f80u | ((x >> 9) & 0x7fu) | ((x >> 8) & 0x8000u);
    x = x * 1664525u + 1013904223u;
    unsigned hi = 0x3f80u | ((x >> 9) & 0x7fu) | ((x >> 8) & 0x8000u);
    v = lo | (hi << 16);
  }
  u32x4* d;
  float* o;
  CHECK(hipMalloc(&d, h.size() * 4));
  CHECK(hipMalloc(&o, (size_t)2 * ncu * 256 * 4));
  CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const int steps = 40000;
  const dim3 grid(2 * ncu);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    for (int shape : {32, 16}) {
      for (int w = 0; w < 2; ++w) {  // warm, then timed
        CHECK(hipEventRecord(e0));
        if (shape == 32) hipLaunchKernelGGL(shape_kernel<32>, grid, dim3(256), 0, 0, d, steps, o);
        else hipLaunchKernelGGL(shape_kernel<16>, grid, dim3(256), 0, 0, d, steps, o);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
      }
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      // per wave per step: 64 x 64 outputs x K 32 = 131072 MAC
      const double flops = 2.0 * 131072.0 * steps * 4 * grid.x;
      printf("rep %d shape %dx%d: %.3f ms  %.1f TFLOP/s\n", rep, shape, shape, ms, flops / ms / 1e9);
    }
  }
  return 0;
}
