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

// ---- fp16 (IEEE binary16, storage = _Float16) --------------------------------
typedef _Float16 f16_t;
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

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
template <> struct Elem<f16_t> {
  static constexpr int kDtype = CWDM_F16;
  __device__ __forceinline__ static float to_f(f16_t v) { return (float)v; }
  __device__ __forceinline__ static f16_t from_f(float v) { return (f16_t)v; }  // round to nearest even
};

// ---- 16-bit pairs in one 32-bit word (element 0 in the low half) -------------
// the bf16 forms are the bit tricks the kernels used from the start; the fp16
// forms convert (v_cvt_f32_f16 / a packed round-to-nearest-even convert)
template <typename T> __device__ __forceinline__ float lo2f(unsigned u);
template <typename T> __device__ __forceinline__ float hi2f(unsigned u);
template <> __device__ __forceinline__ float lo2f<bf16_t>(unsigned u) { return __uint_as_float(u << 16); }
template <> __device__ __forceinline__ float hi2f<bf16_t>(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
template <> __device__ __forceinline__ float lo2f<f16_t>(unsigned u) {
  return (float)__builtin_bit_cast(f16_t, (unsigned short)(u & 0xffffu));
}
template <> __device__ __forceinline__ float hi2f<f16_t>(unsigned u) {
  return (float)__builtin_bit_cast(f16_t, (unsigned short)(u >> 16));
}
template <typename T> __device__ __forceinline__ unsigned pack2(float a, float b);
template <> __device__ __forceinline__ unsigned pack2<bf16_t>(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}
template <> __device__ __forceinline__ unsigned pack2<f16_t>(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2_t));
}

// storage dtype <-> element size / K chunk (32 bytes of input channels per voxel)
inline int dtype_size(int dtype) { return dtype == CWDM_F32 ? 4 : 2; }
inline bool dtype_half(int dtype) { return dtype == CWDM_BF16 || dtype == CWDM_F16; }
inline bool dtype_compute(int dtype) { return dtype == CWDM_F32 || dtype == CWDM_BF16 || dtype == CWDM_F16; }

// host dispatch over the three compute dtypes: f(T{}) with T = float / bf16_t / f16_t
template <typename F>
inline int dispatch_dtype(int dtype, F&& f) {
  if (dtype == CWDM_BF16) return f(bf16_t{});
  if (dtype == CWDM_F16) return f(f16_t{});
  return f(float{});
}

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


// one conv weight pack of a batched launch (conv3d.hip pack_batch_run; the
// U-Net plan collects its packs through g_pack_batch).  No implicit padding:
// tables are compared bytewise to skip re-uploads.
struct PackJob {
  const float* w;
  void* out;
  long long total;
  int cout, cin, ntaps, NT, transpose, cin_real, s2_ci0, pad;
  long long blk0;
};
static_assert(sizeof(PackJob) == 64, "PackJob layout");

// host side of the fused GroupNorm backward reduce (see V4Params::gx0): the
// plan fills it before a dgrad conv and reads back used / nblk
struct GbwdFuse {
  const void* x0; const void* x1; int c0;   // the GroupNorm input (channels-last; x1: channels [c0, C))
  const float* ss; const float* mr; int groups;
  float* part; long long part_bytes;        // [B][nblk][C][2] partials out
  bool used; int nblk;
};
extern thread_local GbwdFuse* g_gbwd;

// the U-Net plan's backward: the SiLU(GroupNorm) backward's apply pass of a
// skip block's GN1, fused into its 1x1 skip dgrad (pointwise.hip pw_kernel):
// dx = W_skip^T dY (+ dx) + k0 SiLU'(x sc + sh) du + k1 x + k2, written once
struct GapplyFuse {
  const void* x0; const void* x1;  // the GroupNorm input = the skip conv's input (split as the dgrad's outputs)
  const void* du;                  // [B][V][N] gradient of the SiLU output
  const float* ss;                 // [B][N][2] scale / shift
  const float* coef;               // [B][N][4] k0, k1, k2 (gn_bwd_finalize)
  bool used;
};
extern thread_local GapplyFuse* g_gapply;

// The U-Net plan's forward: a GroupNorm finalize (statistics partials -> scale /
// shift, cwdm_gn_finalize) offered to the consumer conv.  Where the conv's
// GroupNorm+SiLU pre-pass runs at a small grid it computes the finalize itself
// (gn_fin_apply, conv3d_v4.hip: each workgroup reduces the partials of its 16
// channels); any other route runs cwdm_gn_finalize first (gnfin_flush).  Either
// way ss / mr are written for later readers (the backward).
struct GnFinFuse {
  const float* s0; long long p0; int c0;
  const float* s1; long long p1; int c1;
  const float* gamma; const float* beta;
  int groups; long long voxels; float eps;
  float* ss;   // [B][C][2] -- the a_gn pointer of the consumer conv
  float* mr;   // [B][groups][2]
  long long B;
  bool used;
};
extern thread_local GnFinFuse* g_gnfin;
// run the offered finalize now if it is pending for d (d->a_gn == its ss)
int gnfin_flush(const cwdm_conv3d_desc* d, hipStream_t s);
}  // namespace cwdm
