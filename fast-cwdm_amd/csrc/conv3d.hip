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

// Tiled variant for the jobs without the stride-2 fold: a workgroup takes one
// (32 output channels, one input chunk) tile of a job, every tap.  The tile's
// weights come in as contiguous runs of w (forward: per co, the chunk's CK x
// ntaps floats; transposed: per ci, 32 co x ntaps floats) into LDS, and go out
// as 16-byte vectors of the packed layout (one (n, quad) per lane, consecutive
// lanes consecutive in memory).  pack_batch_kernel's output-indexed gather read
// one float per 108-byte tap row and wrote 2 bytes per lane: ~0.4 ms for the
// 81.5 M-parameter U-Net's 326 MB of weights, twice per training step.
template <typename T>
__global__ void __launch_bounds__(256) pack_tile_kernel(const PackJob* __restrict__ jobs, int njobs) {
  constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ;
  __shared__ __attribute__((aligned(16))) float sm[32 * CK * 27];
  const long long bid = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].blk0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const PackJob j = jobs[lo];
  const int nch = j.cin / CK, nsubs = j.NT / 32, nt = j.ntaps;
  long long r = bid - j.blk0;
  const int chunk = (int)(r % nch);
  r /= nch;
  const int nsub = (int)(r % nsubs);
  const int ct = (int)(r / nsubs);
  const int co0 = ct * j.NT + nsub * 32, ci0 = chunk * CK;
  const int tid = threadIdx.x;
  // rows of L floats: forward, row = co_l (32 rows, w[co0 + row][ci0 ..][*]);
  // transposed, row = ci_l (CK rows, w[ci0 + row][co0 ..][*], nk valid floats)
  const int rows = j.transpose ? CK : 32, L = j.transpose ? 32 * nt : CK * nt;
  const int nk = j.transpose ? min(32, j.cout - co0) * nt : L;
  auto src_of = [&](int row) -> const float* {
    return j.transpose ? j.w + ((long long)(ci0 + row) * j.cout + co0) * nt
                       : j.w + ((long long)(co0 + row) * j.cin + ci0) * nt;
  };
  auto row_ok = [&](int row) { return j.transpose ? ci0 + row < j.cin_real : co0 + row < j.cout; };
  // 16-byte loads when every run starts 16-byte aligned: 4 x 16 B in flight per
  // lane (4-byte loads left ~1 KB in flight per wave: 1.2 TB/s)
  const bool v4 = ((size_t)j.w & 15) == 0 && L % 4 == 0 && nk % 4 == 0 &&
                  (j.transpose ? (long long)j.cout * nt % 4 == 0 : (long long)j.cin * nt % 4 == 0);
  if (v4) {
    const int L4 = L / 4, n4 = rows * L4;
    for (int i0 = tid; i0 < n4; i0 += 4 * 256) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < n4) {
          const int row = i / L4, k4 = i - row * L4;
          if (row_ok(row) && 4 * k4 < nk) v[u] = reinterpret_cast<const float4*>(src_of(row))[k4];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        if (i < n4) reinterpret_cast<float4*>(sm)[i] = v[u];
      }
    }
  } else {
    for (int row = 0; row < rows; ++row) {
      const float* src = src_of(row);
      const bool ok = row_ok(row);
      for (int k = tid; k < L; k += 256) sm[row * L + k] = (ok && k < nk) ? src[k] : 0.f;
    }
  }
  __syncthreads();
  T* out = reinterpret_cast<T*>(j.out);
  for (int v = tid; v < nt * 64; v += 256) {
    const int qp = v & 1, nl = (v >> 1) & 31, tap = v >> 6;
    const int q = qp ^ ((nl >> 3) & 1);
    T tmp[EPQ] __attribute__((aligned(16)));
#pragma unroll
    for (int e = 0; e < EPQ; ++e) {
      const int cil = q * EPQ + e;
      const float x = j.transpose ? sm[(cil * 32 + nl) * nt + (nt - 1 - tap)] : sm[(nl * CK + cil) * nt + tap];
      tmp[e] = Elem<T>::from_f(x);
    }
    const long long off = (((((long long)ct * nch + chunk) * nt + tap) * j.NT + nsub * 32 + nl) * 2 + qp) * EPQ;
    *reinterpret_cast<uint4*>(out + off) = *reinterpret_cast<const uint4*>(tmp);
  }
}

// Split-bf16 packing of an fp32 conv for the accurate fast mode (conv3d_v5.hip,
// cwdm_conv3d_desc.a_w_split): the bf16 layout of a virtual conv with 3 cin
// inputs -- per pair of fp32 K chunks (a: channels 16 p .. + 7, b: + 8 .. + 15)
// three bf16 chunks: A = [hi(w_a) | hi(w_a)] and B = [hi(w_b) | hi(w_b)] over a
// chunk's (hi(x) | lo(x)) halo planes, C = [lo(w_a) | lo(w_b)] over (hi(x_a) |
// hi(x_b)); hi = bf16(w), lo = bf16(w - hi): hi.hi + lo.hi + hi.lo of every
// product, fp32-accumulated.  Quad slots swizzled by bit 3 of the output row as
// in pack_impl (only C's two quads differ).
__global__ void __launch_bounds__(256) pack_split_kernel(const float* __restrict__ w, int cout, int cin, int NT,
                                                         bf16_t* __restrict__ out, long long total) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int nvc = 3 * (cin / 16);  // virtual 16-channel chunks
  const int e = (int)(i % 8);
  long long r = i / 8;
  const int qp = (int)(r % 2);
  r /= 2;
  const int n = (int)(r % NT);
  r /= NT;
  const int tap = (int)(r % 27);
  r /= 27;
  const int vc = (int)(r % nvc);
  const int ct = (int)(r / nvc);
  const int pair = vc / 3, kind = vc % 3;
  const int q = qp ^ ((n >> 3) & 1);   // the logical K half this slot carries
  const int co = ct * NT + n, ci = pair * 16 + (kind == 2 ? 8 * q : 8 * kind) + e;
  float v = 0.f;
  if (co < cout) {
    const float x = w[((long long)co * cin + ci) * 27 + tap];
    const float hi = bf2f(f2bf(x));
    v = kind == 2 ? x - hi : hi;
  }
  out[i] = f2bf(v);
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

extern "C" int64_t cwdm_conv3d_packed_split_bytes(int cout, int cin) {
  if (cout <= 0 || cout % 64 || cin <= 0 || cin % 16) return -1;
  return cwdm_conv3d_packed_bytes(cout, 3 * cin, 3, CWDM_BF16);
}

extern "C" int cwdm_conv3d_pack_split(const float* w, int cout, int cin, void* packed, cwdm_stream_t stream) {
  CWDM_REQUIRE(w && packed, CWDM_E_INVALID, "cwdm_conv3d_pack_split: null pointer");
  CWDM_REQUIRE(cout > 0 && cout % 64 == 0 && cin > 0 && cin % 16 == 0, CWDM_E_UNSUPPORTED,
               "cwdm_conv3d_pack_split: cout % 64 == 0, cin % 16 == 0");
  const int NT = 64;
  const long long total = (long long)(cout / NT) * (3 * cin / 16) * 27 * NT * 16;
  hipLaunchKernelGGL(pack_split_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, w,
                     cout, cin, NT, reinterpret_cast<bf16_t*>(packed), total);
  CWDM_LAUNCHED();
  return CWDM_OK;
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
  // the tiled kernel's jobs (no stride-2 fold, ntaps <= 27) first, then the gather kernel's
  static const bool tiled_on = [] { const char* e = std::getenv("CWDM_PACK_TILED"); return !(e && e[0] == '0'); }();
  auto tiled = [&](const PackJob& j) { return tiled_on && j.s2_ci0 == 0 && j.ntaps <= 27 && j.NT % 32 == 0; };
  std::stable_partition(jobs.begin(), jobs.end(), tiled);
  size_t nt = 0;
  while (nt < jobs.size() && tiled(jobs[nt])) ++nt;
  const int ck = ck_of(dtype);
  long long tb = 0, blk = 0;
  for (size_t i = 0; i < jobs.size(); ++i) {
    auto& j = jobs[i];
    if (i < nt) {
      j.blk0 = tb;
      tb += ceil_div(j.cout, j.NT) * (j.NT / 32) * (long long)(j.cin / ck);
    } else {
      j.blk0 = blk;
      blk += ceil_div(j.total, 1024);
    }
  }
  CWDM_REQUIRE(blk < (1LL << 31) && tb < (1LL << 31), CWDM_E_UNSUPPORTED, "pack batch: too many blocks");
  if (cache.size() != jobs.size() || std::memcmp(cache.data(), jobs.data(), jobs.size() * sizeof(PackJob))) {
    CWDM_HIP(hipMemcpyAsync(table, jobs.data(), jobs.size() * sizeof(PackJob), hipMemcpyHostToDevice, s));
    CWDM_HIP(hipStreamSynchronize(s));  // (pageable source; only when the layout changed)
    cache = jobs;
  }
  return dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if (nt > 0) {
      hipLaunchKernelGGL(pack_tile_kernel<T>, dim3((unsigned)tb), dim3(256), 0, s, table, (int)nt);
      CWDM_LAUNCHED();
    }
    if (nt < jobs.size()) {
      hipLaunchKernelGGL(pack_batch_kernel<T>, dim3((unsigned)blk), dim3(256), 0, s, table + nt,
                         (int)(jobs.size() - nt));
      CWDM_LAUNCHED();
    }
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
bool v5_eligible(const cwdm_conv3d_desc* d, bool gn);
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
  return (v4_eligible(d) || (d->a_w_split && v5_eligible(d, false))) ? std::max(legacy, v4_workspace_bytes(d)) : legacy;
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
  // (an offered GroupNorm finalize, GnFinFuse, runs first on every route but the
  // DMA-staged one, whose pre-pass may take it)
  int rc;
  if (head_eligible(d)) {
    if ((rc = gnfin_flush(d, (hipStream_t)stream))) return rc;
    return head_conv_forward(d, (hipStream_t)stream);
  }
  if (pw_eligible(d)) {
    if ((rc = gnfin_flush(d, (hipStream_t)stream))) return rc;
    return pw_forward(d, (hipStream_t)stream);
  }
  // (the accurate fast mode's split-bf16 kernel takes fp32 shapes of any size: the same host path)
  if (v4_eligible(d) || (d->a_w_split && v5_eligible(d, false))) {
    const int64_t need = v4_workspace_bytes(d);
    if (need == 0 || (d->workspace && d->ws_bytes >= need)) return conv3d_v4_forward(d, (hipStream_t)stream);
  }
  if ((rc = gnfin_flush(d, (hipStream_t)stream))) return rc;
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

