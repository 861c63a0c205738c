// Host side of the DMA-staged conv3d (conv3d_v4.hpp) and its pre-passes:
//   * cwdm_gn_apply: SiLU(GroupNorm(x)) of one or two channels-last sources
//     written once into a workspace tensor (the conv then stages raw copies),
//   * the 1x1 skip segment (ResBlock skip_connection) runs first as a B-only
//     conv into a workspace tensor that the 3x3x3 conv adds as its residual.
#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "conv3d_v4.hpp"

namespace cwdm {

template __global__ void conv3d_v4_kernel<bf16_t, 0, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 0, true, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 0, true, false, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 0, true, true, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 1, true, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 1, true>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 0, false>(V4Params);
template __global__ void conv3d_v4_kernel<bf16_t, 1, false>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 0, true>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 0, true, true>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 0, true, false, true>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 0, true, true, true>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 1, true, true>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 1, true>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 0, false>(V4Params);
template __global__ void conv3d_v4_kernel<f16_t, 1, false>(V4Params);
template __global__ void conv3d_v4_kernel<float, 0, false>(V4Params);
template __global__ void conv3d_v4_kernel<float, 1, false>(V4Params);

namespace {

// out[v][c] = SiLU(x[v][c] * sc[b][c] + sh[b][c]); a thread handles one
// 8-channel group of VPT voxels a quarter of the volume apart (each load /
// store instruction still covers consecutive voxels across the lanes), so
// VPT loads are in flight together and the scale/shift reload only when the
// batch index changes.  32-bit item indices (host-checked: B * V * C / 8 < 2^31;
// the 64-bit version's three 64-bit divisions per voxel cost as much issue as
// the traffic it moves).
// cm: write the chunk-major layout [B][C / CK][V][CK] the DMA-staged conv reads
// as contiguous halo rows (CK = 16 bf16 / 8 fp32 channels = 32 bytes per voxel)
template <typename T, int VPT>
__global__ void __launch_bounds__(256) gn_apply_kernel(const T* __restrict__ x0, int c0, const T* __restrict__ x1,
                                                      int c1, const float* __restrict__ gn, FastDiv dvpb,
                                                      FastDiv dg8, unsigned nvox, unsigned nq, T* __restrict__ out,
                                                      int cm) {
  const int C = c0 + c1;
  const unsigned i0 = blockIdx.x * 256u + threadIdx.x;   // (voxel slot, group)
  const unsigned vq = fdiv(i0, dg8);                     // voxels vq, vq + nq, ...
  if (vq >= nq) return;
  const int c = (int)(i0 - vq * dg8.d) * 8;
  constexpr int CK = 32 / sizeof(T);
  const bool first = c < c0;
  const T* xs = first ? x0 + c : x1 + (c - c0);
  const unsigned xc = first ? c0 : c1;
  float xv[VPT][8];
  unsigned vs[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const unsigned v = vq + k * nq < nvox ? vq + k * nq : nvox - 1;
    vs[k] = v;
    const T* src = xs + (size_t)v * xc;
    if constexpr (sizeof(T) == 2) {
      unpack<T>(*reinterpret_cast<const u32x4*>(src), xv[k]);
    } else {
      unpack<float>(*reinterpret_cast<const u32x4*>(src), xv[k]);
      unpack<float>(*reinterpret_cast<const u32x4*>(src + 4), xv[k] + 4);
    }
  }
  unsigned bprev = 0xFFFFFFFFu;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    if (vq + k * nq >= nvox) break;
    const unsigned v = vs[k];
    const unsigned b = fdiv(v, dvpb);
    if (b != bprev) {
      const float4* g4 = reinterpret_cast<const float4*>(gn + ((size_t)b * C + c) * 2);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float4 t = g4[e];  // (sc, sh) of channels c + 2e, c + 2e + 1
        silu_aff_coef(t.x, t.y, sc[2 * e], sh[2 * e]);
        silu_aff_coef(t.z, t.w, sc[2 * e + 1], sh[2 * e + 1]);
      }
      bprev = b;
    }
    float y[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = silu_aff(xv[k][e], sc[e], sh[e]);
    T* dst = cm ? out + ((size_t)(b * (unsigned)(C / CK) + (unsigned)(c / CK)) * dvpb.d + (v - b * dvpb.d)) * CK + (c % CK)
                : out + (size_t)v * C + c;
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<u32x4*>(dst) = pack<T>(y);
    } else {
      *reinterpret_cast<u32x4*>(dst) = pack<float>(y);
      *reinterpret_cast<u32x4*>(dst + 4) = pack<float>(y + 4);
    }
  }
}

// GroupNorm finalize + SiLU(GN(x)) pre-pass in one launch (small grids,
// GnFinFuse): workgroup (16-channel chunk j, voxel block, batch entry) first
// reduces the statistics partials of its 16 channels -- parts x 16 (sum, sum^2)
// pairs, 128 contiguous bytes per part -- in fp64 (thread (part slice r,
// channel cl) over parts r, r + 16, ..., then the 16 slices and the group's
// channels in order), derives (scale, shift) as gn_finalize does, and applies
// them to its voxels, writing the chunk-major layout (32 bytes of the chunk per
// voxel).  Workgroups of voxel block 0 also write ss / mr for later readers.
// 16-bit types; a chunk lies in one source (c0 % 16 == 0); cpg divides 16.
struct GnFinApplyArgs {
  const void* x0; int c0; const void* x1; int c1;
  const float* s0; long long p0; const float* s1; long long p1;
  const float* gamma; const float* beta; int groups; double n; float eps;
  float* ss; float* mr; void* out;
  int V, vblk;   // voxels per batch entry, voxels per workgroup
};

template <typename T>
__global__ void __launch_bounds__(256) gn_fin_apply_kernel(GnFinApplyArgs a) {
  const int j = blockIdx.x, vb = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int C = a.c0 + a.c1, cpg = C / a.groups, c16 = 16 * j;
  const bool first = c16 < a.c0;
  const int cs = first ? a.c0 : a.c1, cl0 = first ? c16 : c16 - a.c0;
  const long long P = first ? a.p0 : a.p1;
  const float2* part = reinterpret_cast<const float2*>(first ? a.s0 : a.s1) + (long long)b * P * cs + cl0;
  __shared__ double r1[256], r2[256];
  __shared__ float tab[32];
  {
    const int cl = t & 15, r = t >> 4;
    double s = 0.0, q = 0.0;
    for (long long k = r; k < P; k += 16) {
      const float2 u = part[k * cs + cl];
      s += (double)u.x;
      q += (double)u.y;
    }
    r1[t] = s;
    r2[t] = q;
  }
  __syncthreads();
  if (t < 16) {
    double s = 0.0, q = 0.0;
    for (int r = 0; r < 16; ++r) { s += r1[r * 16 + t]; q += r2[r * 16 + t]; }
    r1[t] = s;   // (slot t of slice 0 is read only by this thread)
    r2[t] = q;
  }
  __syncthreads();
  if (t < 16) {
    const int g0 = (t / cpg) * cpg;   // the group's first channel within the chunk
    double s = 0.0, q = 0.0;
    for (int k = 0; k < cpg; ++k) { s += r1[g0 + k]; q += r2[g0 + k]; }
    const double mean = s / a.n;
    double var = q / a.n - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)a.eps));
    const float meanf = (float)mean;
    const int c = c16 + t;
    const float sc = a.gamma[c] * rstd;
    const float sh = a.beta[c] - meanf * sc;
    tab[2 * t] = sc;
    tab[2 * t + 1] = sh;
    if (vb == 0) {
      a.ss[((long long)b * C + c) * 2] = sc;
      a.ss[((long long)b * C + c) * 2 + 1] = sh;
      if (t % cpg == 0 && a.mr) {
        const int g = c / cpg;
        a.mr[((long long)b * a.groups + g) * 2] = meanf;
        a.mr[((long long)b * a.groups + g) * 2 + 1] = rstd;
      }
    }
  }
  __syncthreads();
  const int h = t & 1, vs = t >> 1;
  float sa[8], sb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) silu_aff_coef(tab[2 * (8 * h + e)], tab[2 * (8 * h + e) + 1], sa[e], sb[e]);
  const T* xs = reinterpret_cast<const T*>(first ? a.x0 : a.x1) + (long long)b * a.V * cs + cl0 + 8 * h;
  T* out = reinterpret_cast<T*>(a.out) + (((long long)b * (C / 16) + j) * a.V) * 16 + 8 * h;
  const int v0 = vb * a.vblk, v1 = min(a.V, v0 + a.vblk);
  for (int v = v0 + vs; v < v1; v += 128) {
    float f[8];
    unpack<T>(*reinterpret_cast<const u32x4*>(xs + (long long)v * cs), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = silu_aff(f[e], sa[e], sb[e]);
    *reinterpret_cast<u32x4*>(out + (long long)v * 16) = pack<T>(f);
  }
}

inline int64_t align256(int64_t n) { return (n + 255) & ~(int64_t)255; }

int64_t src_voxels(const cwdm_conv3d_desc* d) {
  const int64_t V = d->D * d->H * d->W;
  return d->a_mode == 1 ? V / 8 : V;
}

}  // namespace

// kernel-path policy (cwdm_conv3d_set_path): 0 auto, 1 legacy only, 2 DMA kernels wherever the shape allows,
// 3 as 2 without the warp-specialised kernel
std::atomic<int> g_conv_path{[] {
  const char* e = std::getenv("CWDM_CONV_PATH");
  return e ? std::atoi(e) : 0;
}()};

std::atomic<unsigned long long*> g_stamps{nullptr};

bool sg_eligible(const cwdm_conv3d_desc* d);
bool sg_skip_eligible(const cwdm_conv3d_desc* d);
int sg_launch(const V4Params& v, const cwdm_conv3d_desc* d, void* partial, hipStream_t s);
int64_t ksplit_slice_voxels(const cwdm_conv3d_desc* d);
bool pw_eligible(const cwdm_conv3d_desc* d);
int pw_forward(const cwdm_conv3d_desc* d, hipStream_t s);
bool pw_split_eligible(const cwdm_conv3d_desc* d);
int pw_split_forward(const cwdm_conv3d_desc* d, hipStream_t s);
int sg_ksplit(const cwdm_conv3d_desc* d);
int sg_skip_launch(const cwdm_conv3d_desc* d, void* out, void* partial, hipStream_t s);
int sg_skip_ksplit(const cwdm_conv3d_desc* d);
int64_t sg_sync_bytes(int ksplit);
bool v5_eligible(const cwdm_conv3d_desc* d, bool gn);
int v5_launch(const cwdm_conv3d_desc* d, const void* a0, int c0, const void* a1, int c1, int a0_cm,
              const float* agn, const void* res, int rmode, hipStream_t s, const V5Aa* aa = nullptr);
int v5_aa_units(const cwdm_conv3d_desc* d, int* lead);
unsigned* plan_aa_counters();

int64_t v4_items(const cwdm_conv3d_desc* d) {
  return d->B * ((d->W + 31) / 32) * (d->H / 4) * (d->D / 4) * (d->cout / 64);
}

// work items a launch aims for before it splits K (env CWDM_V4_KSPLIT_TARGET)
int64_t v4_ksplit_target() {
  static const int64_t t = [] {
    const char* e = std::getenv("CWDM_V4_KSPLIT_TARGET");
    // 64 (r04; was 128): config 5's 28^3 64-channel down-block convs (49 tiles)
    // then run unsplit on 32-channel tiles: 44 -> 19 us against the split legacy path
    return e ? (int64_t)std::atoll(e) : (int64_t)64;
  }();
  return t;
}

// K split of a grid with fewer tiles than two workgroups per CU (the 32^3
// level): enough K slices for ~512 work items, at least two chunks per slice
int v4_ksplit(const cwdm_conv3d_desc* d) {
  if (sg_eligible(d)) return sg_ksplit(d);  // the small-grid kernel's own K split (8^3 level)
  const int ck = 32 / dtype_size(d->dtype);
  const int nch = (d->a_c0 + d->a_c1) / ck;
  const int64_t nblk = v4_items(d);
  const int64_t target = v4_ksplit_target();
  if (nblk >= target || nch < 2) return 1;
  // 16-bit: v4_launch doubles the work items with 32-channel tiles (no finishing
  // passes) -- enough at config 5's 28^3 level (98 -> 196)
  if (dtype_half(d->dtype) && 2 * nblk >= target && d->cout % 64 == 0) return 1;
  int S = (int)std::min<int64_t>((target + nblk - 1) / nblk, nch / 2);
  if (S < 1) S = 1;
  const int per = (nch + S - 1) / S;
  return (nch + per - 1) / per;
}

bool v4_eligible(const cwdm_conv3d_desc* d) {
  const int path = g_conv_path.load(std::memory_order_relaxed);
  if (path == 1) return false;
  // the 1x1 skip product is added through the residual slot: not both
  if (d->b_w && d->res_mode >= 0) return false;
  if (sg_eligible(d)) return true;  // 16^3 / 8^3 levels: conv3d_sg.hip behind the same pre-passes
  if (!dtype_compute(d->dtype)) return false;
  // W >= kWideMinW: the statistics partials follow cwdm_conv3d_parts' 32-wide x tiles (pick_brick)
  if (!d->a_w || d->W < kWideMinW || d->H % 4 || d->D % 4 || d->cout % 64) return false;
  if (d->a_mode != 0 && d->a_mode != 1) return false;
  if (d->res_mode < -1 || d->res_mode > 1) return false;
  if (d->out1 && d->out_c0 % 8) return false;
  const int64_t nblk = v4_items(d);
  // work items: K slices, or (16-bit, no split, < 256 tiles) v4_launch's 32-channel tiles
  const int S = v4_ksplit(d);
  const int64_t items = nblk * S * (S == 1 && dtype_half(d->dtype) && nblk < 256 ? 2 : 1);
  if (items < std::min<int64_t>(384, v4_ksplit_target()) && path < 2) return false;  // too few work items even K-split: the brick kernels
  const int esz = dtype_size(d->dtype);
  const int64_t sv = src_voxels(d);
  // the DMA range check works on 32-bit byte offsets per batch
  const int64_t lim = 0xFFFFE000LL;
  if (d->a_gn) return sv * (d->a_c0 + d->a_c1) * esz < lim;
  return sv * d->a_c0 * esz < lim && sv * d->a_c1 * esz < lim;
}

int64_t v4_workspace_bytes(const cwdm_conv3d_desc* d) {
  const int esz = dtype_size(d->dtype);
  int64_t ws = 0;
  if (d->a_gn) ws += align256(d->B * src_voxels(d) * (d->a_c0 + d->a_c1) * esz);
  if (d->b_w) ws += align256(d->B * d->D * d->H * d->W * d->cout * esz);
  // K-split slices of the conv, or of its 1x1 skip pre-pass (which runs first: one region serves both)
  int S = v4_ksplit(d);
  if (d->b_w) {
    cwdm_conv3d_desc e = *d;
    e.a_w = nullptr;
    S = std::max(S, sg_skip_ksplit(&e));
  }
  // (+ the small-grid kernel's K-split arrival counters behind the slices)
  if (S > 1) ws += align256(S * d->B * ksplit_slice_voxels(d) * d->cout * 4) + sg_sync_bytes(S);
  // (+ a lone launch's apply-ahead sweep counters, last: conv3d_v4_forward)
  if (d->a_gn) ws += kV5AaWords * 4;
  return ws;
}

int legacy_conv3d_forward(const cwdm_conv3d_desc* d, cwdm_stream_t stream);

// the U-Net plan's backward: fuse the reduce pass of the SiLU(GroupNorm)
// backward that follows this dgrad conv into its epilogue (GbwdFuse, conv3d_v4.hpp
// V4Params::gx0); taken only by the 16-bit fast epilogue without K split
thread_local GbwdFuse* g_gbwd = nullptr;
thread_local GnFinFuse* g_gnfin = nullptr;

int gnfin_flush(const cwdm_conv3d_desc* d, hipStream_t s) {
  GnFinFuse* f = g_gnfin;
  if (!f || f->used || !d->a_gn || f->ss != d->a_gn) return CWDM_OK;
  f->used = true;
  return cwdm_gn_finalize(f->s0, f->p0, f->c0, f->s1, f->p1, f->c1, f->gamma, f->beta, f->groups, f->B, f->voxels,
                          f->eps, f->ss, f->mr, s);
}

namespace {
// the fused finalize + pre-pass applies: 16-bit, every 16-channel chunk in one
// source and whole groups, few partials per chunk (the small grids: <= 256 parts)
bool gn_fin_fusable(const GnFinFuse& f, int dtype, int c0, int c1) {
  const int C = c0 + c1;
  if (!dtype_half(dtype) || C % 16 || c0 % 16 || f.c0 != c0 || f.c1 != c1 || f.groups <= 0 || C % f.groups) return false;
  const int cpg = C / f.groups;
  // the largest grid, in voxels, whose finalize the pre-pass takes (env CWDM_GNFIN_MAXV, A/B knob):
  // 32^3 -- with per-workgroup partials the 64^3 / 128^3 finalizes qualify too, but the fused pass
  // (~512 workgroups, each re-reducing its chunk's partials) streams the big grids far below the plain
  // pre-pass: r06 same box, 15.33 ms per step without the fusion there vs 15.52 (64^3) / 15.96 (128^3)
  static const long long maxv = [] { const char* e = std::getenv("CWDM_GNFIN_MAXV"); return e ? std::atoll(e) : 32768LL; }();
  return cpg <= 16 && 16 % cpg == 0 && f.p0 <= 256 && (c1 == 0 || f.p1 <= 256) && f.voxels <= maxv;
}

int gn_fin_apply(const GnFinFuse& f, const void* x0, int c0, const void* x1, int c1, int64_t B, int64_t V, int dtype,
                 void* out, hipStream_t s) {
  GnFinApplyArgs a{};
  a.x0 = x0; a.c0 = c0; a.x1 = x1; a.c1 = c1;
  a.s0 = f.s0; a.p0 = f.p0; a.s1 = f.s1; a.p1 = f.p1;
  a.gamma = f.gamma; a.beta = f.beta; a.groups = f.groups;
  a.n = (double)((c0 + c1) / f.groups) * (double)f.voxels; a.eps = f.eps;
  a.ss = f.ss; a.mr = f.mr; a.out = out;
  CWDM_REQUIRE(V < (1LL << 31) && V * (c0 + c1) < (1LL << 31), CWDM_E_UNSUPPORTED, "gn_fin_apply: grid too large");
  a.V = (int)V;
  // ~512 workgroups in all
  const int nchunk = (c0 + c1) / 16;
  long long nvb = std::max<long long>(1, 512 / (nchunk * B));
  a.vblk = (int)std::max<long long>(128, ceil_div(V, nvb));
  nvb = ceil_div(V, (long long)a.vblk);
  CWDM_REQUIRE(B < 65536 && nvb < 65536, CWDM_E_UNSUPPORTED, "gn_fin_apply: grid too large");
  const dim3 grid((unsigned)nchunk, (unsigned)nvb, (unsigned)B);
  if (dtype == CWDM_F16) hipLaunchKernelGGL(gn_fin_apply_kernel<f16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(gn_fin_apply_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
}  // namespace

// the backward's dgrad conv whose epilogue may take the GroupNorm-backward
// reduce (v4 only): only where the conv leaves VALU room -- at 128^3 the
// epilogue's ~13 VALU + 2 transcendentals per output element cost the
// MFMA-bound kernel more (+30 %) than the separate reduce pass it saves; at
// 32^3 it is a net win (same-box kernel traces).  At 64^3 it was too
// against v4's plain dgrad (r03), but the warp-specialised kernel now takes those
// dgrads faster than the fused v4 instance runs: 12 launches 3096 us fused vs 2547 +
// 371 us of separate reduces (r06, profiles/r06/w_gbwd_maxw_ab.txt).  Env
// CWDM_GBWD_MAXW, default 32.  Elsewhere the dgrad is an ordinary conv (v5 may take it).
bool gbwd_grid_ok(const cwdm_conv3d_desc* d) {
  static const int gb_maxw = [] { const char* e = std::getenv("CWDM_GBWD_MAXW"); return e ? std::atoi(e) : 32; }();
  return g_gbwd && !g_gbwd->used && dtype_half(d->dtype) && d->W <= gb_maxw && d->a_mode == 0 && d->res_mode < 0 &&
         !d->stats;
}

int gn_apply(const void* x0, int c0, const void* x1, int c1, const float* gn, int64_t B, int64_t vpb, int dtype,
             void* out, hipStream_t s, int cm = 0) {
  constexpr int VPT = 4;
  const int G8 = (c0 + c1) / 8;
  CWDM_REQUIRE(B * vpb * G8 < (1LL << 31) - 256 * VPT, CWDM_E_UNSUPPORTED,
               "gn_apply: more than 2^31 channel groups in one launch");
  const int64_t nvox = B * vpb, nq = ceil_div(nvox, VPT);
  const dim3 grid((unsigned)ceil_div(nq * G8, 256));
  const FastDiv dvpb = make_fastdiv((unsigned)vpb), dg8 = make_fastdiv((unsigned)G8);
  return dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL((gn_apply_kernel<T, VPT>), grid, dim3(256), 0, s, reinterpret_cast<const T*>(x0), c0,
                       reinterpret_cast<const T*>(x1), c1, gn, dvpb, dg8, (unsigned)nvox, (unsigned)nq,
                       reinterpret_cast<T*>(out), cm);
    CWDM_LAUNCHED();
    return CWDM_OK;
  });
}

// launch of the DMA-staged kernel on prepared sources: a0 (c0 channels,
// chunk-major if a0_cm) and a1 (c1 channels, channels-last), residual res/rmode;
// partial: fp32 scratch of v4_ksplit(d) output slices (unused without a K split)
int v4_launch(const cwdm_conv3d_desc* d, const void* a0, int c0, const void* a1, int c1, int a0_cm,
              const void* res, int rmode, void* partial, hipStream_t s) {
  const int esz = dtype_size(d->dtype);
  const int ck = 32 / esz;
  const int64_t SV = src_voxels(d);
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
  p.out_f32 = (d->out_dtype == CWDM_F32 && d->dtype != CWDM_F32) ? 1 : 0;
  p.stats = d->stats;
  p.out1 = d->out1; p.out_c0 = d->out_c0;
  p.accumulate = d->accumulate;
  p.stamps = g_stamps.load(std::memory_order_relaxed);
  if (sg_eligible(d)) return sg_launch(p, d, partial, s);
  // the warp-specialised kernel (conv3d_v5.hip) where it applies (not the
  // backward's fused GroupNorm-reduce dgrad, not the stamps diagnostics build)
  if (v5_eligible(d, false))   // (refuses the dgrad that takes the fused GroupNorm-backward reduce)
    return v5_launch(d, a0, c0, a1, c1, a0_cm, nullptr, res, rmode, s);
  const int S = v4_ksplit(d);
  p.ksplit = S;
  p.kper = (p.nch + S - 1) / S;
  if (S > 1) {
    CWDM_REQUIRE(partial, CWDM_E_INVALID, "conv3d: K-split scratch missing");
    p.ks_stride = (long long)p.B * p.D * p.H * p.W * p.cout;
    p.bias = nullptr; p.res = nullptr; p.rmode = -1; p.stats = nullptr;
    p.out = partial; p.out_f32 = 1; p.out1 = nullptr; p.out_c0 = 0; p.accumulate = 0;
  }
  // fewer 64-channel tiles than CUs (the 32^3 level): 32-channel tiles, one
  // z-plane per wave (twice the work items; the statistics bricks are the same)
  static const bool ct32_on = [] { const char* e = std::getenv("CWDM_V4_CT32"); return !(e && e[0] == '0'); }();
  const bool ct32 = ct32_on && dtype_half(d->dtype) && S == 1 && !p.out_f32 && !p.accumulate && !p.out1 &&
                    (long long)p.B * p.tx * p.ty * p.tz * p.nct < 256 &&
                    (long long)p.D * p.H * p.W * p.cout * 2 < 0xFFFFE000LL;
  if (ct32) p.nct = d->cout / 32;
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz * p.nct * S;
  p.nblk = (int)nblk;
  // persistent: two workgroups per CU (80 KB LDS, <= 256 registers per lane each)
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  // workgroups per CU slot of the persistent grid (env CWDM_V4_GRID_MULT, A/B knob)
  static const long long gmul = [] { const char* e = std::getenv("CWDM_V4_GRID_MULT"); return e ? std::atoll(e) : 4LL; }();
  const dim3 grid((unsigned)std::min<long long>(nblk, gmul * ncu));
  // half a tile: ~17k cycles per chunk and ~12k for the epilogue when shared (tools/conv_stamps.py)
  // CWDM_CONV_STAGGER=-1 restores the half-tile delay; measured (r01 v7 kernel,
  // bench.py A/B on one MI355X): no delay 57.15 vs half-tile 56.80 steps/s
  static const int stagger_env = [] { const char* e = std::getenv("CWDM_CONV_STAGGER"); return e ? std::atoi(e) : 0; }();
  p.stagger_cycles = nblk > 2LL * ncu ? (stagger_env >= 0 ? stagger_env : (p.nch * 17000 + 12000) / 2) : 0;
  // the fast epilogue addresses output / residual through 32-bit buffer offsets per batch
  const bool fast = !p.out_f32 && !p.accumulate && !p.out1 &&
                    (long long)p.D * p.H * p.W * p.cout * 2 < 0xFFFFE000LL;
  prof_begin(s);
  auto launch16 = [&](auto tag) {
    using T = decltype(tag);
    if (p.gx0) {   // fused GroupNorm-backward reduce (dgrad, same-grid source: amode 0)
      if (ct32) hipLaunchKernelGGL((conv3d_v4_kernel<T, 0, true, true, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v4_kernel<T, 0, true, false, true>), grid, dim3(256), 0, s, p);
    } else if (ct32) {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<T, 1, true, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v4_kernel<T, 0, true, true>), grid, dim3(256), 0, s, p);
    } else if (fast) {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<T, 1, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v4_kernel<T, 0, true>), grid, dim3(256), 0, s, p);
    } else {
      if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<T, 1, false>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv3d_v4_kernel<T, 0, false>), grid, dim3(256), 0, s, p);
    }
  };
  // (gbwd_grid_ok: where the fused reduce pays)
  if (gbwd_grid_ok(d) && (ct32 || fast) && S == 1 && rmode < 0 && !p.stats && p.amode == 0) {
    GbwdFuse& g = *g_gbwd;
    const int nc = ct32 ? 32 : 64;
    const int C = d->cout;
    const long long need = (long long)p.B * p.tx * p.ty * p.tz * C * 8;
    if (g.groups > 0 && C % g.groups == 0 && C / g.groups >= 2 && g.c0 % nc == 0 && g.c0 <= C &&
        (g.c0 == C || g.x1) && need <= g.part_bytes) {
      p.gx0 = g.x0; p.gx1 = g.x1; p.gc0 = g.c0;
      p.gss = g.ss; p.gmr = g.mr; p.ggroups = g.groups;
      p.gdiv = make_fastdiv((unsigned)(C / g.groups));
      p.stats = g.part;
      g.used = true;
      g.nblk = p.tx * p.ty * p.tz;
    }
  }
  if (d->dtype == CWDM_BF16) {
    launch16(bf16_t{});
  } else if (d->dtype == CWDM_F16) {
    launch16(f16_t{});
  } else {
    if (p.amode == 1) hipLaunchKernelGGL((conv3d_v4_kernel<float, 1, false>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv3d_v4_kernel<float, 0, false>), grid, dim3(256), 0, s, p);
  }
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * (c0 + c1));
  CWDM_LAUNCHED();
  if (S > 1) {
    // finish: slice sum over the whole chip, then the per-tile epilogue
    const long long n4 = p.ks_stride / 4;
    float* part = reinterpret_cast<float*>(partial);
    hipLaunchKernelGGL(splitk_sum_kernel<0>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, s, part, S, n4);
    CWDM_LAUNCHED();
    ConvParams q{};
    q.B = p.B; q.D = p.D; q.H = p.H; q.W = p.W;
    q.tx = p.tx; q.ty = p.ty; q.tz = p.tz;
    q.cout = p.cout; q.nct = p.nct;
    q.bias = d->bias; q.bias_bs = d->bias_bstride;
    q.res = res; q.rmode = rmode;
    q.out = d->out; q.out_f32 = (d->out_dtype == CWDM_F32 && d->dtype != CWDM_F32) ? 1 : (d->dtype == CWDM_F32);
    q.stats = d->stats;
    q.out1 = d->out1; q.out_c0 = d->out_c0;
    q.accumulate = d->accumulate;
    q.ksplit = 1;
    q.partial = part;
    const dim3 rg((unsigned)v4_items(d));
    dispatch_dtype(d->dtype, [&](auto tag) -> int {
      using T = decltype(tag);
      hipLaunchKernelGGL((conv3d_reduce_kernel<T, 32, 4, 4, 2>), rg, dim3(256), 0, s, q, 1);
      return CWDM_OK;
    });
    CWDM_LAUNCHED();
  }
  return CWDM_OK;
}

thread_local void* g_act_keep = nullptr;  // set by the U-Net plan's training forward (ActKeepScope)
thread_local int g_act_kept = 0;

int conv3d_v4_forward(const cwdm_conv3d_desc* d, hipStream_t s) {
  const int esz = dtype_size(d->dtype);
  unsigned char* ws = reinterpret_cast<unsigned char*>(d->workspace);
  const int64_t SV = src_voxels(d);
  const void* a0 = d->a0;
  const void* a1 = d->a1;
  int c0 = d->a_c0, c1 = d->a_c1;
  int a0_cm = 0;
  int rc;
  // GroupNorm + SiLU inside the warp-specialised conv (no activated copy):
  // inference only -- the training forward keeps the activated input for wgrad
  const float* agn = nullptr;
  if (d->a_gn && !g_act_keep && v5_eligible(d, true)) agn = d->a_gn;
  // or the warp-specialised conv writes the activated copy itself, ahead of its sweep (apply-ahead:
  // no pre-pass over HBM; the training forward keeps the copy it writes)
  V5Aa aa{};
  aa.units = (d->a_gn && !agn) ? v5_aa_units(d, &aa.lead) : 0;
  // an offered GroupNorm finalize (GnFinFuse): fused into the pre-pass below where it fits, else run now
  GnFinFuse* fin = (g_gnfin && !g_gnfin->used && d->a_gn && g_gnfin->ss == d->a_gn) ? g_gnfin : nullptr;
  if (fin && (agn || aa.units || !gn_fin_fusable(*fin, d->dtype, c0, c1))) {
    if ((rc = gnfin_flush(d, s))) return rc;
    fin = nullptr;
  }
  if (d->a_gn && !agn) {
    // the activated input: in the workspace, or (training) where the plan keeps
    // it for the backward's DMA-staged wgrad
    void* act = ws;
    if (g_act_keep) {
      act = g_act_keep;
      g_act_kept = 1;
    } else {
      ws += align256(d->B * SV * (c0 + c1) * esz);
    }
    if (aa.units) {
      aa.x0 = a0; aa.c0 = c0; aa.x1 = a1; aa.c1 = c1; aa.gn = d->a_gn;
      // the sweep counters: the plan's zeroed sync block, else this launch's workspace tail (zeroed here)
      aa.cnt = plan_aa_counters();
      if (!aa.cnt) {
        const int64_t need = v4_workspace_bytes(d);
        CWDM_REQUIRE(d->workspace && d->ws_bytes >= need, CWDM_E_WORKSPACE, "conv3d (apply-ahead): workspace too small");
        aa.cnt = reinterpret_cast<unsigned*>(reinterpret_cast<unsigned char*>(d->workspace) + need - kV5AaWords * 4);
        CWDM_HIP(hipMemsetAsync(aa.cnt, 0, kV5AaWords * 4, s));
      }
    } else if (fin) {
      fin->used = true;
      if ((rc = gn_fin_apply(*fin, a0, c0, a1, c1, d->B, SV, d->dtype, act, s))) return rc;
    } else if ((rc = gn_apply(a0, c0, a1, c1, d->a_gn, d->B, SV, d->dtype, act, s, 1))) {
      return rc;
    }
    a0 = act; c0 = c0 + c1; a1 = nullptr; c1 = 0;
    a0_cm = 1;
  }
  const void* res = d->res;
  int rmode = d->res_mode;
  if (d->b_w) {
    void* skip = ws;
    ws += align256(d->B * d->D * d->H * d->W * d->cout * esz);
    cwdm_conv3d_desc e = *d;
    e.a0 = nullptr; e.a1 = nullptr; e.a_c0 = 0; e.a_c1 = 0; e.a_gn = nullptr; e.a_w = nullptr; e.a_mode = 0;
    e.bias = nullptr; e.bias_bstride = 0; e.stats = nullptr;
    e.out = skip; e.out_dtype = d->dtype; e.out1 = nullptr; e.out_c0 = 0; e.accumulate = 0;
    e.workspace = nullptr; e.ws_bytes = 0;
    if (sg_skip_eligible(&e)) {
      if ((rc = sg_skip_launch(&e, skip, ws, s))) return rc;   // ws: the K-split region, free until the conv
    } else if (pw_eligible(&e)) {
      if ((rc = pw_forward(&e, s))) return rc;
    } else if (pw_split_eligible(&e)) {
      if ((rc = pw_split_forward(&e, s))) return rc;
    } else if ((rc = legacy_conv3d_forward(&e, (cwdm_stream_t)s))) {
      return rc;
    }
    res = skip; rmode = 0;
  }
  if (agn) return v5_launch(d, a0, c0, a1, c1, 0, agn, res, rmode, s);
  if (aa.units) return v5_launch(d, a0, c0, nullptr, 0, 1, nullptr, res, rmode, s, &aa);
  return v4_launch(d, a0, c0, a1, c1, a0_cm, res, rmode, v4_ksplit(d) > 1 ? ws : nullptr, s);
}

// ---------------------------------------------------------------------------
// ResBlock with a 1x1 skip_connection (unet.py:264-271): x is read once for
// both users.  One pass writes act = SiLU(GN1(x)) (chunk-major, conv1's input)
// and skip = W_skip . x (channels-last, conv2's residual; its bias is folded
// into conv2's).  Per block of 128 voxels the workgroup copies the x rows into
// LDS with coalesced 16-byte loads (rows padded by 16 B: conflict-free column
// reads); then each wave takes 32 voxels: lane (v, hh) reads quad hh of every
// 16-channel chunk of voxel v, transforms it for act (stored 1 KB-contiguous per
// wave instruction) and feeds it raw as the MFMA B operand against W_skip (A
// operand, the conv packing of a 1x1 kernel, staged once per workgroup) -- the
// conv kernel's accumulator layout.
// ---------------------------------------------------------------------------
struct ApplySkipParams {
  const void* x0; int c0; const void* x1; int c1;
  const float* gn;     // [B][C][2] scale / shift
  long long vpb;       // voxels per batch (% 128 == 0)
  long long nvox;      // B * vpb
  int B;
  void* act;           // chunk-major [B][C / CK][vpb][CK]
  const unsigned char* ws;  // packed 1x1 weights, NT = 64 rows per channel tile
  int cout;            // 32 NF
  void* skip;          // [B][vpb][cout]
};

template <typename T, int NF, int QT>
__global__ void __launch_bounds__(256) gn_apply_skip_kernel(ApplySkipParams p) {
  constexpr int CK = ConvTr<T>::CK, EPQ = ConvTr<T>::EPQ, ES = sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int C = p.c0 + p.c1, nk = C / CK;
  const int wbytes = NF * 32 * C * ES;
  const int RS = C * ES + 16;                      // padded LDS row of one voxel
  for (int i = threadIdx.x * 16; i < wbytes; i += 256 * 16)
    *reinterpret_cast<u32x4*>(lds + i) = *reinterpret_cast<const u32x4*>(p.ws + i);
  float* gl = reinterpret_cast<float*>(lds + wbytes);
  for (int i = threadIdx.x; i < p.B * C * 2; i += 256) gl[i] = p.gn[i];
  unsigned char* xt = lds + wbytes + ((p.B * C * 8 + 15) & ~15);
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, hh = lane >> 5, wv = tid >> 6;
  const int q0 = p.c0 * ES / 16, q1 = p.c1 * ES / 16;   // 16-byte quads per row of each source
  const int nq0 = 128 * q0, nqt = (q0 + q1) / 2;        // quads of source 0 per block; per thread
  const long long nblocks = p.nvox / 128;
  // the next block's 128 x rows are loaded into registers while this block
  // computes (consecutive lanes read consecutive 16-byte quads), then copied
  // to LDS: HBM latency hides under the MFMA / store work
  u32x4 pf[QT];
  // quad i = tid + 256 j of a block: source 0 rows first (nq0 quads), then
  // source 1; its global offset within the block's rows is i (or i - nq0) x 16
  // bytes, its LDS offset (row vl, column) is fixed per thread: computed once,
  // so the block loop carries no integer division
  int loff[QT];
#pragma unroll
  for (int j = 0; j < QT; ++j) {
    const int i = tid + 256 * j;
    int vl, col;
    if (i < nq0) { vl = i / q0; col = i - vl * q0; }
    else { const int i1 = i - nq0; vl = i1 / q1; col = q0 + (i1 - vl * q1); }
    loff[j] = vl * RS + col * 16;
  }
  const unsigned char* xb0 = reinterpret_cast<const unsigned char*>(p.x0);
  const unsigned char* xb1 = reinterpret_cast<const unsigned char*>(p.x1);
  auto fetch = [&](long long blk) {
    const unsigned char* s0 = xb0 + blk * 128 * q0 * 16;
    const unsigned char* s1 = xb1 + blk * 128 * q1 * 16 - (long long)nq0 * 16;
#pragma unroll
    for (int j = 0; j < QT; ++j) {
      if (j >= nqt) break;
      const int i = tid + 256 * j;
      pf[j] = *reinterpret_cast<const u32x4*>((i < nq0 ? s0 : s1) + (long long)i * 16);
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < QT; ++j) {
      if (j >= nqt) break;
      *reinterpret_cast<u32x4*>(xt + loff[j]) = pf[j];
    }
  };
  if ((long long)blockIdx.x < nblocks) fetch(blockIdx.x);
  for (long long blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const long long v0 = blk * 128;
    __syncthreads();  // previous block's column reads are done (and W / gn staged, first time)
    put();
    __syncthreads();
    if (blk + gridDim.x < nblocks) fetch(blk + gridDim.x);
    const int vl = wv * 32 + lr;
    const long long v = v0 + vl;
    const int b = (int)(v0 / p.vpb);
    const long long vb = v - (long long)b * p.vpb;
    f32x16 acc[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[f][i] = 0.f;
    for (int k = 0; k < nk; ++k) {
      const u32x4 q = *reinterpret_cast<const u32x4*>(xt + vl * RS + k * 32 + hh * 16);
      float xv[EPQ], y[EPQ];
      unpack<T>(q, xv);
      const float* gs = gl + ((long long)b * C + k * CK + hh * EPQ) * 2;
#pragma unroll
      for (int e = 0; e < EPQ; ++e) y[e] = silu(xv[e] * gs[2 * e] + gs[2 * e + 1]);
      T* dst = reinterpret_cast<T*>(p.act) + (((long long)b * nk + k) * p.vpb + vb) * CK + hh * EPQ;
      *reinterpret_cast<u32x4*>(dst) = pack<T>(y);
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int n = (f & 1) * 32 + lr;
        const u32x4 a = *reinterpret_cast<const u32x4*>(
            lds + (((f >> 1) * nk + k) * 64 + n) * 32 + ((hh ^ ((n >> 3) & 1)) << 4));
        mfma_acc(acc[f], a, q, (T*)nullptr);
      }
    }
    // skip store: lane (v, hh) holds channels 32 f + 8 j + 4 hh + 0..3 of voxel v
#pragma unroll
    for (int f = 0; f < NF; ++f) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        T* o = reinterpret_cast<T*>(p.skip) + v * p.cout + f * 32 + 8 * j + 4 * hh;
        if constexpr (sizeof(T) == 2) {
          uint2 w;
          w.x = pack2<T>(acc[f][4 * j], acc[f][4 * j + 1]);
          w.y = pack2<T>(acc[f][4 * j + 2], acc[f][4 * j + 3]);
          *reinterpret_cast<uint2*>(o) = w;
        } else {
          *reinterpret_cast<float4*>(o) = make_float4(acc[f][4 * j], acc[f][4 * j + 1], acc[f][4 * j + 2], acc[f][4 * j + 3]);
        }
      }
    }
  }
}

int64_t apply_skip_lds_bytes(int dtype, int C, int cout, int64_t B) {
  const int es = dtype_size(dtype);
  return (int64_t)cout * C * es + ((B * C * 8 + 15) & ~15) + 128LL * (C * es + 16);
}

bool apply_skip_ok(int dtype, int C, int cout, int64_t B, int64_t vpb) {
  const int ck = 32 / dtype_size(dtype);
  const int qt = C * dtype_size(dtype) / 32;   // prefetch registers per thread (kernel's QT)
  return dtype_compute(dtype) && (cout == 64 || cout == 128) && vpb % 128 == 0 &&
         C % ck == 0 && qt <= 16 && apply_skip_lds_bytes(dtype, C, cout, B) <= 160 * 1024;
}

int gn_apply_skip(const void* x0, int c0, const void* x1, int c1, const float* gn, int64_t B, int64_t vpb, int dtype,
                  const void* wskip, int cout, void* act, void* skip, hipStream_t s) {
  CWDM_REQUIRE(apply_skip_ok(dtype, c0 + c1, cout, B, vpb), CWDM_E_UNSUPPORTED, "gn_apply_skip: unsupported shape");
  ApplySkipParams p{};
  p.x0 = x0; p.c0 = c0; p.x1 = x1; p.c1 = c1; p.gn = gn; p.vpb = vpb; p.nvox = B * vpb; p.B = (int)B;
  p.act = act; p.ws = reinterpret_cast<const unsigned char*>(wskip); p.cout = cout; p.skip = skip;
  const int64_t lds = apply_skip_lds_bytes(dtype, c0 + c1, cout, B);
  const int64_t nblocks = p.nvox / 128;
  static const int64_t cap = [] { const char* e = std::getenv("CWDM_SKIP_GRID"); return e ? (int64_t)std::atoll(e) : (int64_t)512; }();
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(nblocks, cap)));
  auto go = [&](auto kern) -> int {
    CWDM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, grid, dim3(256), (unsigned)lds, s, p);
    return CWDM_OK;
  };
  int rc;
  rc = dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    return cout == 64 ? go(gn_apply_skip_kernel<T, 2, 16>) : go(gn_apply_skip_kernel<T, 4, 16>);
  });
  if (rc) return rc;
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace cwdm

using namespace cwdm;

extern "C" int cwdm_gn_apply(const void* x0, int c0, const void* x1, int c1, const float* gn, int64_t B,
                             int64_t voxels, int dtype, void* out, cwdm_stream_t stream) {
  CWDM_REQUIRE(x0 && gn && out && (c1 == 0 || x1), CWDM_E_INVALID, "cwdm_gn_apply: null pointer");
  CWDM_REQUIRE(c0 > 0 && c0 % 8 == 0 && c1 % 8 == 0 && B > 0 && voxels > 0, CWDM_E_SHAPE,
               "cwdm_gn_apply: channels must be multiples of 8");
  CWDM_REQUIRE(dtype_compute(dtype), CWDM_E_INVALID, "cwdm_gn_apply: bad dtype");
  return gn_apply(x0, c0, x1, c1, gn, B, voxels, dtype, out, (hipStream_t)stream);
}

extern "C" int cwdm_conv3d_set_path(int path) {
  CWDM_REQUIRE(path >= 0 && path <= 3, CWDM_E_INVALID, "cwdm_conv3d_set_path: path must be 0, 1, 2 or 3");
  return g_conv_path.exchange(path);
}

// diagnostics: the DMA-staged conv kernel writes 24 u64 per workgroup (s_memtime
// at start / after the prologue / after each of the first 16 chunks / at the end,
// and HW_ID, XCC_ID) into buf (device memory, >= 24 * workgroups); null disables
extern "C" int cwdm_debug_conv_stamps(void* buf) {
  g_stamps.store(reinterpret_cast<unsigned long long*>(buf));
  return CWDM_OK;
}

// diagnostics / tests: the fused GroupNorm finalize + pre-pass (gn_fin_apply_kernel)
// on its own, so it can be compared with cwdm_gn_finalize + cwdm_gn_apply in one
// process (the plan picks it per conv; CWDM_GNFIN is read once)
extern "C" int cwdm_debug_gn_fin_apply(const float* stats0, int64_t parts0, int c0, const float* stats1,
                                       int64_t parts1, int c1, const float* gamma, const float* beta, int groups,
                                       int64_t B, int64_t voxels, float eps, const void* x0, const void* x1,
                                       int dtype, float* scale_shift, float* mean_rstd, void* out_cm,
                                       cwdm_stream_t stream) {
  CWDM_REQUIRE(stats0 && x0 && gamma && beta && scale_shift && mean_rstd && out_cm && (c1 == 0 || (stats1 && x1)),
               CWDM_E_INVALID, "cwdm_debug_gn_fin_apply: null pointer");
  CWDM_REQUIRE(B > 0 && voxels > 0 && parts0 > 0 && (c1 == 0 || parts1 > 0), CWDM_E_SHAPE,
               "cwdm_debug_gn_fin_apply: empty shape");
  GnFinFuse f{};
  f.s0 = stats0; f.p0 = parts0; f.c0 = c0;
  f.s1 = stats1; f.p1 = parts1; f.c1 = c1;
  f.gamma = gamma; f.beta = beta; f.groups = groups; f.voxels = voxels; f.eps = eps;
  f.ss = scale_shift; f.mr = mean_rstd; f.B = B;
  CWDM_REQUIRE(gn_fin_fusable(f, dtype, c0, c1), CWDM_E_UNSUPPORTED,
               "cwdm_debug_gn_fin_apply: not a fusable shape (16-bit, 16-channel chunks, <= 16 channels per "
               "group dividing 16, <= 256 partials)");
  return gn_fin_apply(f, x0, c0, x1, c1, B, voxels, dtype, out_cm, (hipStream_t)stream);
}
