// Conv3d host side: weight packing, launch planning (brick, split-K) and the C ABI.
// Kernels: conv3d_kernels.hpp, instantiated in conv3d_inst_*.hip.
#include <algorithm>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "conv3d_kernels.hpp"

namespace cwdm {
extern template int launch_wide<bf16_t, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<bf16_t, 32, 4, 2, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<bf16_t, 16, 4, 4, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<bf16_t, 8, 8, 4, 1>(const ConvParams&, hipStream_t);
extern template int launch_wide<bf16_t, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<bf16_t, 32, 4, 2, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<bf16_t, 16, 4, 4, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<bf16_t, 8, 8, 4, 2>(const ConvParams&, hipStream_t);
extern template int launch_wide<f16_t, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<f16_t, 32, 4, 2, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<f16_t, 16, 4, 4, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<f16_t, 8, 8, 4, 1>(const ConvParams&, hipStream_t);
extern template int launch_wide<f16_t, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<f16_t, 32, 4, 2, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<f16_t, 16, 4, 4, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<f16_t, 8, 8, 4, 2>(const ConvParams&, hipStream_t);
extern template int launch_wide<float, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<float, 32, 4, 2, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<float, 16, 4, 4, 1>(const ConvParams&, hipStream_t);
extern template int launch_conv<float, 8, 8, 4, 1>(const ConvParams&, hipStream_t);
extern template int launch_wide<float, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<float, 32, 4, 2, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<float, 16, 4, 4, 2>(const ConvParams&, hipStream_t);
extern template int launch_conv<float, 8, 8, 4, 2>(const ConvParams&, hipStream_t);
// ---- weight packing: OIDHW fp32 -> [ct][chunk][tap][n][2 quads, swizzled] ----
// stride-2 conv as a stride-1 conv over the space-to-depth input (stride2.hip):
// expanded weight We[co][ph ci0 + ci][t] of w[co][ci][k] (ci0 original input channels)
__device__ __forceinline__ int s2_k(int t, int p) { return t == 1 ? 1 + p : ((t == 0 && p == 1) ? 0 : -1); }
__device__ __forceinline__ float s2_weight(const float* w, int ci0, int co, int ci_e, int t) {
  const int ph = ci_e / ci0, ci = ci_e % ci0;
  const int kz = s2_k(t / 9, ph >> 2), ky = s2_k((t / 3) % 3, (ph >> 1) & 1), kx = s2_k(t % 3, ph & 1);
  if (kz < 0 || ky < 0 || kx < 0) return 0.f;
  return w[((long long)co * ci0 + ci) * 27 + (kz * 3 + ky) * 3 + kx];
}

// element i of a packed weight image (output-indexed)
template <typename T>
__device__ __forceinline__ void pack_elem(const float* __restrict__ w, int cout, int cin, int ntaps, int NT,
                                          T* __restrict__ out, int transpose, int cin_real, int s2_ci0, long long i) {
  constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ;
  const int nch = cin / CK;
  const int e = i % EPQ;
  long long r = i / EPQ;
  const int qp = r % 2;
  r /= 2;
  const int n = r % NT;
  r /= NT;
  const int tap = r % ntaps;
  r /= ntaps;
  const int chunk = r % nch;
  const int ct = r / nch;
  const int q = qp ^ ((n >> 3) & 1);
  const int co = ct * NT + n, ci = chunk * CK + q * EPQ + e;
  float v = 0.f;
  // transpose: pack the input-gradient conv of a (cin -> cout) conv, i.e. weights
  // W'[co'=ci][ci'=co][tap] = W[co][ci][ntaps-1-tap] (w is then cin x cout OIDHW)
  if (co < cout && ci < cin_real) {
    if (s2_ci0) v = transpose ? s2_weight(w, s2_ci0, ci, co, ntaps - 1 - tap) : s2_weight(w, s2_ci0, co, ci, tap);
    else if (transpose) v = w[((long long)ci * cout + co) * ntaps + (ntaps - 1 - tap)];
    else v = w[((long long)co * cin + ci) * ntaps + tap];
  }
  out[i] = Elem<T>::from_f(v);
}

template <typename T>
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ w, int cout, int cin, int ntaps, int NT,
                                                   int nct, T* __restrict__ out, int transpose, int cin_real,
                                                   int s2_ci0) {
  constexpr int CK = ConvTr<T>::CK;
  const long long total = (long long)nct * (cin / CK) * ntaps * NT * CK;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) pack_elem<T>(w, cout, cin, ntaps, NT, out, transpose, cin_real, s2_ci0, i);
}

// every conv of a U-Net pack in one launch: block -> job by a binary search
// over the jobs' first blocks (uniform per block), 1024 elements per block
template <typename T>
__global__ void __launch_bounds__(256) pack_batch_kernel(const PackJob* __restrict__ jobs, int njobs) {
  const long long bid = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].blk0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const PackJob j = jobs[lo];
  const long long base = (bid - j.blk0) * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // 4 independent gathers in flight per thread
    const long long i = base + k * 256 + threadIdx.x;
    if (i < j.total)
      pack_elem<T>(j.w, j.cout, j.cin, j.ntaps, j.NT, reinterpret_cast<T*>(j.out), j.transpose, j.cin_real,
                   j.s2_ci0, i);
  }
}

template <typename T, int NF>
int dispatch_brick(const ConvParams& p, const Brick& br, hipStream_t s) {
  if (br.bx == 32 && br.bz == 4) return launch_wide<T, NF>(p, s);
  if (br.bx == 32) return launch_conv<T, 32, 4, 2, NF>(p, s);
  if (br.bx == 16) return launch_conv<T, 16, 4, 4, NF>(p, s);
  return launch_conv<T, 8, 8, 4, NF>(p, s);
}

// K-split factor: small grids (the U-Net's 32^3 .. 8^3 levels) get split-K so
// that a launch has ~768 workgroups to spread over 256 CUs.
inline int pick_ksplit(long long nblk, int total_chunks) {
  static const long long target = [] { const char* e = std::getenv("CWDM_KSPLIT_TARGET"); return e ? std::atoll(e) : 768LL; }();
  if (nblk >= 512 || nblk >= target || total_chunks <= 1) return 1;
  int S = (int)((target + nblk - 1) / nblk);
  if (S > total_chunks) S = total_chunks;
  const int per = (total_chunks + S - 1) / S;
  return (total_chunks + per - 1) / per;
}

int ck_of(int dtype) { return 32 / dtype_size(dtype); }

}  // namespace cwdm

using namespace cwdm;

extern "C" int64_t cwdm_conv3d_packed_bytes(int cout, int cin, int ksize, int dtype) {
  if (cout <= 0 || cin <= 0 || (ksize != 1 && ksize != 3)) return -1;
  const int ck = ck_of(dtype);
  if (cin % ck) return -1;
  const int NT = 32 * pick_nf(cout);
  const int nct = (int)ceil_div(cout, NT);
  const int ntaps = ksize * ksize * ksize;
  if (!dtype_compute(dtype)) return -1;
  const int esz = dtype_size(dtype);
  return (int64_t)nct * (cin / ck) * ntaps * NT * ck * esz;
}

static int pack_impl(const float* w, int cout, int cin, int ksize, int dtype, void* packed, int transpose,
                     cwdm_stream_t stream, int s2_ci0 = 0);
namespace cwdm {
extern thread_local std::vector<PackJob>* g_pack_batch;
}

extern "C" int cwdm_conv3d_pack(const float* w, int cout, int cin, int ksize, int dtype, void* packed,
                                cwdm_stream_t stream) {
  return pack_impl(w, cout, cin, ksize, dtype, packed, 0, stream);
}

extern "C" int cwdm_conv3d_pack_s2(const float* w, int cout, int cin, int dtype, void* packed, int transpose,
                                   cwdm_stream_t stream) {
  // forward: a (cout -> 8 cin) conv over the space-to-depth input; transpose: its dgrad (8 cin outputs)
  return transpose ? pack_impl(w, 8 * cin, cout, 3, dtype, packed, 1, stream, cin)
                   : pack_impl(w, cout, 8 * cin, 3, dtype, packed, 0, stream, cin);
}

extern "C" int cwdm_conv3d_pack_dgrad(const float* w, int cout, int cin, int ksize, int dtype, void* packed,
                                      cwdm_stream_t stream) {
  // the dgrad conv maps cout channels back to cin: packed as a (cout -> cin) conv
  // (its input channels are padded with zeros up to the chunk size, e.g. the
  // 8-channel output head)
  return pack_impl(w, cin, cout, ksize, dtype, packed, 1, stream);
}

static int pack_impl(const float* w, int cout, int cin, int ksize, int dtype, void* packed, int transpose,
                     cwdm_stream_t stream, int s2_ci0) {
  CWDM_REQUIRE(w && packed, CWDM_E_INVALID, "cwdm_conv3d_pack: null pointer");
  CWDM_REQUIRE(ksize == 1 || ksize == 3, CWDM_E_UNSUPPORTED, "cwdm_conv3d_pack: kernel size must be 1 or 3");
  CWDM_REQUIRE(dtype_compute(dtype), CWDM_E_INVALID, "cwdm_conv3d_pack: bad dtype");
  const int ck = ck_of(dtype);
  const int cin_real = cin;
  if (transpose) cin = (int)ceil_div(cin, ck) * ck;
  CWDM_REQUIRE(cin % ck == 0, CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_pack: input channels must be a multiple of " + std::to_string(ck));
  const int NT = 32 * pick_nf(cout);
  const int nct = (int)ceil_div(cout, NT);
  const int ntaps = ksize * ksize * ksize;
  const long long total = (long long)nct * (cin / ck) * ntaps * NT * ck;
  if (g_pack_batch) {  // the U-Net plan collects its packs and launches them together (pack_batch_run)
    g_pack_batch->push_back(PackJob{w, packed, total, cout, cin, ntaps, NT, transpose, cin_real, s2_ci0, 0, 0});
    return CWDM_OK;
  }
  dim3 grid((unsigned)ceil_div(total, 256));
  return dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL(pack_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, w, cout, cin, ntaps, NT, nct,
                       reinterpret_cast<T*>(packed), transpose, cin_real, s2_ci0);
    CWDM_LAUNCHED();
    return CWDM_OK;
  });
}

namespace cwdm {
thread_local std::vector<PackJob>* g_pack_batch = nullptr;

// one launch for the collected packs; the job table goes to `table` (device,
// >= jobs.size() entries), uploaded only when it differs from `cache`
int pack_batch_run(std::vector<PackJob>& jobs, int dtype, PackJob* table, std::vector<PackJob>& cache,
                   hipStream_t s) {
  if (jobs.empty()) return CWDM_OK;
  long long blk = 0;
  for (auto& j : jobs) {
    j.blk0 = blk;
    blk += ceil_div(j.total, 1024);
  }
  CWDM_REQUIRE(blk < (1LL << 31), CWDM_E_UNSUPPORTED, "pack batch: too many blocks");
  if (cache.size() != jobs.size() || std::memcmp(cache.data(), jobs.data(), jobs.size() * sizeof(PackJob))) {
    CWDM_HIP(hipMemcpyAsync(table, jobs.data(), jobs.size() * sizeof(PackJob), hipMemcpyHostToDevice, s));
    CWDM_HIP(hipStreamSynchronize(s));  // (pageable source; only when the layout changed)
    cache = jobs;
  }
  return dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL(pack_batch_kernel<T>, dim3((unsigned)blk), dim3(256), 0, s, table, (int)jobs.size());
    CWDM_LAUNCHED();
    return CWDM_OK;
  });
}
}  // namespace cwdm

namespace {
struct Plan1 { Brick br; int nf, nct, S; long long nblk; int64_t ws; };
Plan1 plan_conv(const cwdm_conv3d_desc* d) {
  Plan1 q;
  q.br = pick_brick(d->D, d->H, d->W);
  q.nf = pick_nf(d->cout);
  q.nct = (int)ceil_div(d->cout, 32 * q.nf);
  q.nblk = (long long)d->B * ceil_div(d->W, q.br.bx) * ceil_div(d->H, q.br.by) * ceil_div(d->D, q.br.bz) * q.nct;
  const int ck = ck_of(d->dtype);
  const int total = (d->a_c0 + d->a_c1) / ck + (d->b_w ? (d->b_c0 + d->b_c1) / ck : 0);
  q.S = pick_ksplit(q.nblk, total);
  q.ws = q.S > 1 ? (int64_t)q.S * d->B * d->D * d->H * d->W * d->cout * 4 : 0;
  return q;
}
}  // namespace

namespace cwdm {
bool v4_eligible(const cwdm_conv3d_desc* d);
int64_t v4_workspace_bytes(const cwdm_conv3d_desc* d);
int conv3d_v4_forward(const cwdm_conv3d_desc* d, hipStream_t s);
int legacy_conv3d_forward(const cwdm_conv3d_desc* d, cwdm_stream_t stream);
bool head_eligible(const cwdm_conv3d_desc* d);
int head_conv_forward(const cwdm_conv3d_desc* d, hipStream_t s);
bool pw_eligible(const cwdm_conv3d_desc* d);
int pw_forward(const cwdm_conv3d_desc* d, hipStream_t s);
}  // namespace cwdm

extern "C" int64_t cwdm_conv3d_workspace_bytes(const cwdm_conv3d_desc* d) {
  if (!d || d->B <= 0 || d->D <= 0 || d->H <= 0 || d->W <= 0 || d->cout <= 0) return -1;
  const int64_t legacy = plan_conv(d).ws;
  return v4_eligible(d) ? std::max(legacy, v4_workspace_bytes(d)) : legacy;
}

extern "C" int64_t cwdm_conv3d_parts(int dtype, int64_t D, int64_t H, int64_t W, int cout) {
  (void)dtype; (void)cout;
  Brick br = pick_brick(D, H, W);
  return ceil_div(D, br.bz) * ceil_div(H, br.by) * ceil_div(W, br.bx);
}

extern "C" int cwdm_conv3d_forward(const cwdm_conv3d_desc* d, cwdm_stream_t stream) {
  CWDM_REQUIRE(d && d->out && (d->a_w || d->b_w), CWDM_E_INVALID, "cwdm_conv3d_forward: null pointer");
  CWDM_REQUIRE(!d->a_w || (d->a0 && d->a_c0 > 0), CWDM_E_INVALID, "cwdm_conv3d_forward: segment A input missing");
  CWDM_REQUIRE(dtype_compute(d->dtype), CWDM_E_INVALID, "cwdm_conv3d_forward: bad dtype");
  CWDM_REQUIRE(d->B > 0 && d->D > 0 && d->H > 0 && d->W > 0 && d->cout > 0, CWDM_E_SHAPE,
               "cwdm_conv3d_forward: empty shape");
  const int ck = ck_of(d->dtype);
  CWDM_REQUIRE(!d->a_w || (d->a_c0 % ck == 0 && d->a_c1 % ck == 0 && (d->a_c1 == 0 || d->a1)), CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_forward: segment A channels must be multiples of " + std::to_string(ck));
  if (d->b_w)
    CWDM_REQUIRE(d->b0 && d->b_c0 > 0 && d->b_c0 % ck == 0 && d->b_c1 % ck == 0 && (d->b_c1 == 0 || d->b1),
                 CWDM_E_UNSUPPORTED, "cwdm_conv3d_forward: segment B channels must be multiples of " + std::to_string(ck));
  CWDM_REQUIRE(d->a_mode >= 0 && d->a_mode <= 2 && d->res_mode >= -1 && d->res_mode <= 2, CWDM_E_INVALID,
               "cwdm_conv3d_forward: bad resample mode");
  if (d->a_mode == 1 || d->res_mode == 1)
    CWDM_REQUIRE(d->D % 2 == 0 && d->H % 2 == 0 && d->W % 2 == 0, CWDM_E_SHAPE,
                 "cwdm_conv3d_forward: upsample needs an even output grid");
  CWDM_REQUIRE(d->res_mode < 0 || d->res, CWDM_E_INVALID, "cwdm_conv3d_forward: residual pointer missing");
  CWDM_REQUIRE(d->out_dtype == CWDM_F32 || d->out_dtype == d->dtype, CWDM_E_INVALID,
               "cwdm_conv3d_forward: output dtype must be fp32 or the compute dtype");
  if (head_eligible(d)) return head_conv_forward(d, (hipStream_t)stream);
  if (pw_eligible(d)) return pw_forward(d, (hipStream_t)stream);
  if (v4_eligible(d)) {
    const int64_t need = v4_workspace_bytes(d);
    if (need == 0 || (d->workspace && d->ws_bytes >= need)) return conv3d_v4_forward(d, (hipStream_t)stream);
  }
  return legacy_conv3d_forward(d, stream);
}

// the brick / split-K kernels of conv3d_kernels.hpp (every shape and mode)
int cwdm::legacy_conv3d_forward(const cwdm_conv3d_desc* d, cwdm_stream_t stream) {
  const Plan1 pl = plan_conv(d);
  const int nf = pl.nf;
  CWDM_REQUIRE(nf == 2 || d->cout % 32 == 0 || d->cout < 32, CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_forward: cout must be a multiple of 32 or below 32");
  ConvParams p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W;
  const Brick br = pl.br;
  p.tx = (int)ceil_div(d->W, br.bx); p.ty = (int)ceil_div(d->H, br.by); p.tz = (int)ceil_div(d->D, br.bz);
  p.cout = d->cout; p.nct = (int)ceil_div(d->cout, 32 * nf);
  p.a0 = d->a0; p.ac0 = d->a_c0; p.a1 = d->a1; p.ac1 = d->a_c1; p.amode = d->a_mode; p.agn = d->a_gn; p.aw = d->a_w;
  p.b0 = d->b0; p.bc0 = d->b_c0; p.b1 = d->b1; p.bc1 = d->b_c1; p.bw = d->b_w;
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.res = d->res; p.rmode = d->res_mode;
  p.out = d->out; p.out_f32 = (d->out_dtype == CWDM_F32 && d->dtype != CWDM_F32) ? 1 : (d->dtype == CWDM_F32);
  p.stats = d->stats;
  p.out1 = d->out1;
  p.out_c0 = d->out_c0;
  p.accumulate = d->accumulate;
  if (!d->a_w) { p.ac0 = 0; p.ac1 = 0; p.a0 = nullptr; p.a1 = nullptr; }
  if (d->out1)
    CWDM_REQUIRE(d->out_c0 > 0 && d->out_c0 < d->cout && d->out_c0 % 8 == 0, CWDM_E_UNSUPPORTED,
                 "cwdm_conv3d_forward: dual-output split must be a multiple of 8 channels");
  p.ksplit = 1;
  p.partial = nullptr;
  if (pl.S > 1 && d->workspace && d->ws_bytes >= pl.ws) {
    p.ksplit = pl.S;
    p.partial = reinterpret_cast<float*>(d->workspace);
  }
  hipStream_t s = (hipStream_t)stream;
  return dispatch_dtype(d->dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    return nf == 2 ? dispatch_brick<T, 2>(p, br, s) : dispatch_brick<T, 1>(p, br, s);
  });
}

