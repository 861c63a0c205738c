// Shared helpers for libcwdm (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/cwdm.h"

namespace cwdm {

// ---- error channel (thread-local, read by cwdm_last_error) ---------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define CWDM_HIP(expr)                                                        \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess)                                                     \
      return ::cwdm::fail(CWDM_E_HIP, std::string(#expr) + ": " +            \
                                          hipGetErrorString(e_));             \
  } while (0)

#define CWDM_REQUIRE(cond, code, msg)                                         \
  do {                                                                        \
    if (!(cond)) return ::cwdm::fail(code, msg);                              \
  } while (0)

// After a kernel launch: report launch-configuration errors without syncing.
#define CWDM_LAUNCHED() CWDM_HIP(hipGetLastError())

// ---- per-conv profiling hook (cwdm_unet_set_profiling) --------------------
// The plan arms it around one conv call; the launch sites of the MFMA conv
// kernels (DMA-staged, brick/wide, head) record an event pair around their own
// launch and the algorithmic flops it covers -- so the bench's roofline times
// exactly those kernels, not the GroupNorm pre-passes or split-K finishes.
struct ProfHook {
  hipEvent_t ev[2][2];
  double flops[2];
  int n = 0;  // brackets used (<= 2 MFMA kernels per conv call)
};
inline thread_local ProfHook* g_prof = nullptr;
inline void prof_begin(hipStream_t s) {
  if (g_prof && g_prof->n < 2) (void)hipEventRecord(g_prof->ev[g_prof->n][0], s);
}
inline void prof_end(hipStream_t s, double flops) {
  if (g_prof && g_prof->n < 2) {
    (void)hipEventRecord(g_prof->ev[g_prof->n][1], s);
    g_prof->flops[g_prof->n] = flops;
    ++g_prof->n;
  }
}

// ---- bf16 <-> f32 (storage = raw 16 bits) --------------------------------
typedef unsigned short bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even, NaN preserved (plain cast lowers to v_cvt_pk_bf16_f32)
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int kDtype = CWDM_F32;
  __device__ __forceinline__ static float load(const float* p) { return *p; }
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int kDtype = CWDM_BF16;
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Division by a launch constant without the integer-division sequence: q =
// (mulhi(n, m) + n) >> s with s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1
// (exact for n < 2^31; the sum then stays below 2^32).  For the index
// arithmetic of the streaming kernels, where 64-bit divisions cost as much
// issue as the memory traffic they move.
struct FastDiv {
  unsigned d, m, s;
};
inline FastDiv make_fastdiv(unsigned d) {
  unsigned s = 0;
  while ((1ull << s) < d) ++s;
  return {d, (unsigned)(((1ull << 32) * ((1ull << s) - d)) / d + 1), s};
}
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.s; }

}  // namespace cwdm
