// Launch-cost probe: chains of dependent empty (or near-empty) kernels in a HIP graph, by static LDS
// size and grid, timed per kernel with rocprofv3 --kernel-trace (or hipEvents over the chain).
// build: hipcc --offload-arch=gfx950 -O3 tools/launch_bench.hip -o tools/launch_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int LDS>
__global__ void __launch_bounds__(256) k_lds(float* out, int n) {
  __shared__ float sm[LDS / 4];
  const int t = threadIdx.x;
  sm[t] = (float)t;
  __syncthreads();
  if (blockIdx.x == 0 && t == 0 && n < 0) out[0] = sm[(t + 1) % (LDS / 4)];
}

template <int LDS>
float chain(int grid, int reps, float* out) {
  hipStream_t s;
  hipStreamCreate(&s);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_lds<LDS>, dim3(grid), dim3(256), 0, s, out, i);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, s);
  for (int k = 0; k < 5; ++k) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  hipStreamDestroy(s);
  return 1000.f * ms / (5 * reps);
}

int main() {
  float* out;
  hipMalloc(&out, 64);
  const int grids[] = {32, 128, 256, 512, 1024};
  for (int g : grids) {
    printf("grid %4d: lds 1K %.2f us  32K %.2f us  64K %.2f us  96K %.2f us  144K %.2f us per kernel\n", g,
           chain<1024>(g, 200, out), chain<32768>(g, 200, out), chain<65536>(g, 200, out), chain<98304>(g, 200, out),
           chain<147456>(g, 200, out));
  }
  return 0;
}
