// Backward kernels of the U-Net ResBlock path besides the convolutions
// (training, guided_diffusion/train_util.py:396-462 -> loss.backward()):
//   * SiLU(GroupNorm(x)) backward (nn.py:17-19, :93-100) with the adjoint of
//     the resampling that followed it in the forward (upsample / AvgPool2),
//     in three passes: per-block channel partials of (sum dz, sum dz*xhat),
//     an fp64 finalize into per-(b, c) affine coefficients + dgamma/dbeta,
//     and an elementwise apply that recomputes dz;
//   * the residual-path resample adjoint, per-channel sums (bias and emb
//     gradients), the timestep-embedding MLP / emb-projection backward;
//   * the AdamW step (torch.optim.AdamW, train_util.py:111).
#include <cmath>
#include <type_traits>

#include "common.hpp"

namespace cwdm {
namespace {

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <typename T> __device__ __forceinline__ void load8(const T* p, float* f);
template <> __device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const u4 a = *reinterpret_cast<const u4*>(p), b = *reinterpret_cast<const u4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[i] = __uint_as_float(a[i]); f[4 + i] = __uint_as_float(b[i]); }
}
template <> __device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float* f) {
  const u4 a = *reinterpret_cast<const u4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(a[i] << 16); f[2 * i + 1] = __uint_as_float(a[i] & 0xffff0000u); }
}
template <> __device__ __forceinline__ void load8<f16_t>(const f16_t* p, float* f) {
  const u4 a = *reinterpret_cast<const u4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = lo2f<f16_t>(a[i]); f[2 * i + 1] = hi2f<f16_t>(a[i]); }
}
template <typename T> __device__ __forceinline__ void store8(T* p, const float* f);
template <> __device__ __forceinline__ void store8<float>(float* p, const float* f) {
  u4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) { a[i] = __float_as_uint(f[i]); b[i] = __float_as_uint(f[4 + i]); }
  *reinterpret_cast<u4*>(p) = a;
  *reinterpret_cast<u4*>(p + 4) = b;
}
template <> __device__ __forceinline__ void store8<bf16_t>(bf16_t* p, const float* f) {
  u4 a;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = pack2<bf16_t>(f[2 * i], f[2 * i + 1]);   // v_cvt_pk_bf16_f32 (RNE, as f2bf)
  *reinterpret_cast<u4*>(p) = a;
}
template <> __device__ __forceinline__ void store8<f16_t>(f16_t* p, const float* f) {
  u4 a;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = pack2<f16_t>(f[2 * i], f[2 * i + 1]);
  *reinterpret_cast<u4*>(p) = a;
}

// gradient of the SiLU output at voxel (z, y, x) of the GN grid, channels [c, c+8).
// MODE is a template parameter: with a runtime three-way branch here the
// gfx950 compiler (ROCm 7.2 clang) dropped the channel offset on the MODE-2
// path of resample_add (an undefined register in the address -> aperture
// violation), so every caller is instantiated per mode.
template <typename T, int MODE>
__device__ __forceinline__ void load_du(const T* du, int C, int c, int b, unsigned v, int d, int h, int w, float* f) {
  if constexpr (MODE == 0) {
    load8<T>(du + ((long long)b * ((long long)d * h * w) + v) * C + c, f);
  } else {
    const unsigned x = v % (unsigned)w, yz = v / (unsigned)w;
    const unsigned y = yz % (unsigned)h, z = yz / (unsigned)h;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = 0.f;
      const int D2 = 2 * d, H2 = 2 * h, W2 = 2 * w;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float g[8];
        load8<T>(du + ((((long long)b * D2 + 2 * z + (k >> 2)) * H2 + 2 * y + ((k >> 1) & 1)) * W2 + 2 * x + (k & 1)) * C +
                     c,
                 g);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += g[e];
      }
    } else {
      load8<T>(du + ((((long long)b * (d >> 1) + (z >> 1)) * (h >> 1) + (y >> 1)) * (w >> 1) + (x >> 1)) * C + c, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= 0.125f;
    }
  }
}

// d/dz SiLU(z) * du, the sigmoid from the hardware exp2 / reciprocal like the
// forward's silu() (1-2 ulp): the IEEE expf + division sequence made the
// GroupNorm backward passes issue-bound instead of HBM-bound
__device__ __forceinline__ float dsilu(float z, float du) {
  const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -1.4426950408889634f));
  return du * (s * (1.0f + z * (1.0f - s)));
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) gn_bwd_reduce_kernel(const T* __restrict__ x0, int c0, const T* __restrict__ x1,
                                                           int c1, const T* __restrict__ du,
                                                           const float* __restrict__ ss,
                                                           const float* __restrict__ mr, int groups, int d, int h,
                                                           int w, long long vpb, float* __restrict__ part) {
  __shared__ float red[256 * 16];
  const int C = c0 + c1, ncg = C >> 3, nslots = 256 / ncg;
  const int b = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int cg = threadIdx.x % ncg, slot = threadIdx.x / ncg;
  const long long V = (long long)d * h * w;
  const int c = cg * 8, cpg = C / groups;
  float A[8], Bs[8], sc[8], sh[8], mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    A[e] = 0.f; Bs[e] = 0.f;
    sc[e] = ss[((long long)b * C + c + e) * 2];
    sh[e] = ss[((long long)b * C + c + e) * 2 + 1];
    const int g = (c + e) / cpg;
    mu[e] = mr[((long long)b * groups + g) * 2];
    rs[e] = mr[((long long)b * groups + g) * 2 + 1];
  }
  const T* xs = c < c0 ? x0 : x1;
  const int xc = c < c0 ? c0 : c1, xo = c < c0 ? c : c - c0;
  if (slot < nslots) {
    const long long v0 = blk * vpb, v1 = v0 + vpb < V ? v0 + vpb : V;
    // UNR voxels per trip, all their loads issued before the arithmetic
    constexpr int UNR = MODE == 1 ? 1 : 4;
    for (long long vb = v0 + slot; vb < v1; vb += (long long)UNR * nslots) {
      float xv[UNR][8], g[UNR][8];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long long v = vb + (long long)u * nslots < v1 ? vb + (long long)u * nslots : vb;
        load8<T>(xs + ((long long)b * V + v) * xc + xo, xv[u]);
        load_du<T, MODE>(du, C, c, b, (unsigned)v, d, h, w, g[u]);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (vb + (long long)u * nslots >= v1) break;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = dsilu(xv[u][e] * sc[e] + sh[e], g[u][e]);
          A[e] += dz;
          Bs[e] += dz * ((xv[u][e] - mu[e]) * rs[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[threadIdx.x * 16 + e] = slot < nslots ? A[e] : 0.f;
    red[threadIdx.x * 16 + 8 + e] = slot < nslots ? Bs[e] : 0.f;
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += 256) {
    const int g8 = cc >> 3, e = cc & 7;
    float sa = 0.f, sb = 0.f;
    for (int s = 0; s < nslots; ++s) {
      sa += red[(s * ncg + g8) * 16 + e];
      sb += red[(s * ncg + g8) * 16 + 8 + e];
    }
    part[(((long long)b * nblk + blk) * C + cc) * 2] = sa;
    part[(((long long)b * nblk + blk) * C + cc) * 2 + 1] = sb;
  }
}

// One workgroup per group g (all batch entries in order): the group's channels'
// partial sums over the nblk blocks (sub threads per channel, 8 loads in flight
// each, fixed order), the group terms, the apply coefficients and dgamma /
// dbeta.  (One workgroup for all channels ran 10 us per call, 71 calls per
// training step.)
__global__ void __launch_bounds__(256) gn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                             int B, const float* __restrict__ gamma,
                                                             const float* __restrict__ mr, int groups,
                                                             long long V, float* __restrict__ coef,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             int acc_affine) {
  __shared__ double rA[256], rB[256], cA[1024], cB[1024], dG[1024], dB[1024], gs[2];
  const int g = blockIdx.x, cpg = C / groups, c0 = g * cpg;
  const int t = threadIdx.x;
  for (int c = t; c < cpg; c += 256) { dG[c] = 0.0; dB[c] = 0.0; }
  for (int b = 0; b < B; ++b) {
    for (int w0 = 0; w0 < cpg; w0 += 256) {
      const int cw = min(256, cpg - w0), sub = 256 / cw;
      const int cl = t % cw, j = t / cw;
      double a = 0.0, bb = 0.0;
      if (j < sub) {
        const float2* pc = reinterpret_cast<const float2*>(part + ((long long)b * nblk * C + c0 + w0 + cl) * 2);
        int i = j;
        for (; i + 7 * sub < nblk; i += 8 * sub) {
          float2 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = pc[(long long)(i + u * sub) * C];
#pragma unroll
          for (int u = 0; u < 8; ++u) { a += (double)v[u].x; bb += (double)v[u].y; }
        }
        for (; i < nblk; i += sub) {
          const float2 v = pc[(long long)i * C];
          a += (double)v.x;
          bb += (double)v.y;
        }
      }
      rA[t] = a; rB[t] = bb;
      __syncthreads();
      if (t < cw) {
        double sa = 0.0, sb = 0.0;
        for (int k = 0; k < sub; ++k) { sa += rA[k * cw + t]; sb += rB[k * cw + t]; }
        cA[w0 + t] = sa; cB[w0 + t] = sb;
        dG[w0 + t] += sb; dB[w0 + t] += sa;
      }
      __syncthreads();
    }
    if (t == 0) {
      double a = 0.0, bb = 0.0;
      for (int c = 0; c < cpg; ++c) {
        a += (double)gamma[c0 + c] * cA[c];
        bb += (double)gamma[c0 + c] * cB[c];
      }
      gs[0] = a; gs[1] = bb;
    }
    __syncthreads();
    const double N = (double)cpg * (double)V;
    const double mu = mr[((long long)b * groups + g) * 2], rs = mr[((long long)b * groups + g) * 2 + 1];
    for (int c = t; c < cpg; c += 256) {
      const double k1 = rs * gamma[c0 + c];
      const double k2 = -rs * rs * gs[1] / N;
      const double k3 = -rs * gs[0] / N + rs * rs * gs[1] * mu / N;
      coef[((long long)b * C + c0 + c) * 4 + 0] = (float)k1;
      coef[((long long)b * C + c0 + c) * 4 + 1] = (float)k2;
      coef[((long long)b * C + c0 + c) * 4 + 2] = (float)k3;
    }
    __syncthreads();
  }
  for (int c = t; c < cpg; c += 256) {
    // acc_affine: a GroupNorm whose parameters serve two calls (WavUNetModel's reused blocks)
    const int cc = c0 + c;
    dgamma[cc] = acc_affine ? dgamma[cc] + (float)dG[c] : (float)dG[c];
    dbeta[cc] = acc_affine ? dbeta[cc] + (float)dB[c] : (float)dB[c];
  }
}

template <typename T> __device__ __forceinline__ float stored(float v) {
  if constexpr (sizeof(T) == 2) return Elem<T>::to_f(Elem<T>::from_f(v));
  else return v;
}

// Batch blockIdx.y.  A workgroup of blockDim.x = (256 / ncg) * ncg threads
// (ncg = C / 8 channel groups) keeps each thread on ONE channel group (tid %
// ncg), so its 8 channels' scale / shift and coefficients sit in registers for
// the whole grid-stride loop over voxels (a per-item reload of the 40
// coefficient words cost more issue than the tensor traffic).
// chs (optional): per-channel sums of the written dx (the value as stored),
// atomically added to chs[b * chs_stride + c] -- the emb-projection gradient of
// the block's conv1 output (sum over voxels of d h1) without a second read of dx.
template <typename T, int MODE>
__global__ void __launch_bounds__(256) gn_bwd_apply_kernel(const T* __restrict__ x0, int c0, const T* __restrict__ x1,
                                                          int c1, const T* __restrict__ du,
                                                          const float* __restrict__ ss,
                                                          const float* __restrict__ coef, int d, int h, int w,
                                                          T* __restrict__ dx0, int acc0, T* __restrict__ dx1,
                                                          int acc1, float* __restrict__ chs, long long chs_stride) {
  const int C = c0 + c1, ncg = C >> 3;
  const unsigned V = (unsigned)d * h * w;   // < 2^31 (host-checked)
  const int b = blockIdx.y;
  const int nvb = blockDim.x / ncg;         // voxels per workgroup trip
  const int cg = threadIdx.x % ncg, c = cg * 8;
  const bool first = c < c0;
  const T* xs = first ? x0 : x1;
  T* dx = first ? dx0 : dx1;
  const int xc = first ? c0 : c1, xo = first ? c : c - c0;
  const int acc = first ? acc0 : acc1;
  float k_sc[8], k_sh[8], k0[8], k1[8], k2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const long long bc = (long long)b * C + c + e;
    k_sc[e] = ss[bc * 2]; k_sh[e] = ss[bc * 2 + 1];
    k0[e] = coef[bc * 4]; k1[e] = coef[bc * 4 + 1]; k2[e] = coef[bc * 4 + 2];
  }
  const T* xb = xs + (size_t)b * V * xc + xo;
  T* ob = dx + (size_t)b * V * xc + xo;
  float sum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sum[e] = 0.f;
  const unsigned vstep = gridDim.x * (unsigned)nvb;
  // UNR voxels per trip: all loads first, then the arithmetic and stores
  constexpr int UNR = MODE == 1 ? 1 : 2;
  for (unsigned v0 = blockIdx.x * (unsigned)nvb + threadIdx.x / ncg; v0 < V; v0 += UNR * vstep) {
    float xv[UNR][8], g[UNR][8], o[UNR][8];
    if constexpr (sizeof(T) == 2) {
      // 16-bit: the loads stay packed until the arithmetic (the unpacked copies of x, du
      // and dx held beside the packed ones took bf16 to 150-168 VGPRs: 3 waves per SIMD)
      u4 xr[UNR], gr[UNR], orr[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const unsigned v = v0 + u * vstep < V ? v0 + u * vstep : v0;
        xr[u] = *reinterpret_cast<const u4*>(xb + (size_t)v * xc);
        if constexpr (MODE == 0) gr[u] = *reinterpret_cast<const u4*>(du + ((size_t)b * V + v) * C + c);
        else load_du<T, MODE>(du, C, c, b, v, d, h, w, g[u]);
        orr[u] = u4{0u, 0u, 0u, 0u};
        if (acc) orr[u] = *reinterpret_cast<const u4*>(ob + (size_t)v * xc);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          xv[u][2 * i] = lo2f<T>(xr[u][i]); xv[u][2 * i + 1] = hi2f<T>(xr[u][i]);
          if constexpr (MODE == 0) { g[u][2 * i] = lo2f<T>(gr[u][i]); g[u][2 * i + 1] = hi2f<T>(gr[u][i]); }
          o[u][2 * i] = lo2f<T>(orr[u][i]); o[u][2 * i + 1] = hi2f<T>(orr[u][i]);
        }
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const unsigned v = v0 + u * vstep < V ? v0 + u * vstep : v0;
        load8<T>(xb + (size_t)v * xc, xv[u]);
        load_du<T, MODE>(du, C, c, b, v, d, h, w, g[u]);
        if (acc) load8<T>(ob + (size_t)v * xc, o[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (v0 + u * vstep >= V) break;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = dsilu(xv[u][e] * k_sc[e] + k_sh[e], g[u][e]);
        const float r = k0[e] * dz + k1[e] * xv[u][e] + k2[e];
        o[u][e] = acc ? o[u][e] + r : r;
      }
      store8<T>(ob + (size_t)(v0 + u * vstep) * xc, o[u]);
      if (chs) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sum[e] += stored<T>(o[u][e]);
      }
    }
  }
  if (!chs) return;
  __shared__ float red[256 * 8];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = sum[e];
  __syncthreads();
  // this workgroup's channel sums -> its row of the partials [B][gridDim.x][C]
  // (chs_reduce_kernel adds them in workgroup order: deterministic)
  for (int cc = threadIdx.x; cc < C; cc += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nvb; ++k) s += red[(k * ncg + (cc >> 3)) * 8 + (cc & 7)];
    chs[((long long)b * gridDim.x + blockIdx.x) * C + cc] = s;
  }
}

// out[b * stride + c] += sum_k part[b][k][c], k in order (fixed-order finish of
// per-workgroup channel sums: the result does not depend on arrival order)
// Fixed-order finish of [B][nk][C] partial rows: a 1024-thread block per 64
// channels; thread (channel cl, row r) sums rows r, r + 16, ... with 8
// interleaved accumulators (loads in flight, not a serial chain), then the 16
// row sums are added in row order -- deterministic for a given nk.  (One
// thread per channel walking all nk rows took ~90 us per call.)
__global__ void __launch_bounds__(1024) chs_reduce_kernel(const float* __restrict__ part, int nk, int C,
                                                         float* __restrict__ out_bc, long long bc_stride,
                                                         float* __restrict__ out_c, float* __restrict__ out_c2,
                                                         int B) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float tot = 0.f;
  for (int b = 0; b < B; ++b) {
    float a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.f;
    if (c < C) {
      const float* p = part + (long long)b * nk * C + c;
      int k = r;
      for (; k + 16 * 7 < nk; k += 16 * 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += p[(long long)(k + 16 * e) * C];
      }
#pragma unroll
      for (int e = 0; e < 7; ++e)
        if (k + 16 * e < nk) a[e] += p[(long long)(k + 16 * e) * C];
    }
    red[r][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (r == 0 && c < C) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) s += red[q][cl];
      if (out_bc) out_bc[(long long)b * bc_stride + c] += s;
      tot += s;
    }
    __syncthreads();
  }
  if (r == 0 && c < C) {
    if (out_c) out_c[c] += tot;
    if (out_c2) out_c2[c] += tot;
  }
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) resample_add_kernel(T* __restrict__ dst, const T* __restrict__ src, int C,
                                                          int d, int h, int w, int acc, FastDiv dncg) {
  const int ncg = C >> 3;
  const long long V = (long long)d * h * w;
  const int b = blockIdx.y;
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i >= (unsigned)(V * ncg)) return;   // < 2^31 (host-checked)
  const unsigned v = fdiv(i, dncg);
  const int c = (int)(i - v * dncg.d) * 8;
  float g[8], o[8];
  load_du<T, MODE>(src, C, c, b, v, d, h, w, g);
  T* p = dst + ((long long)b * V + v) * C + c;
  if (acc) {
    load8<T>(p, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += g[e];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e];
  }
  store8<T>(p, o);
}

template <typename T>
__global__ void __launch_bounds__(256) channel_sum_kernel(const T* __restrict__ src, long long V, int C, int cs,
                                                         long long vpb, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int ncg = (C + 7) >> 3, nslots = 256 / ncg;
  const int b = blockIdx.y, blk = blockIdx.x;
  const int cg = threadIdx.x % ncg, slot = threadIdx.x / ncg;
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  if (slot < nslots) {
    const long long v0 = blk * vpb, v1 = v0 + vpb < V ? v0 + vpb : V;
#pragma unroll 4
    for (long long v = v0 + slot; v < v1; v += nslots) {
      float f[8];
      load8<T>(src + ((long long)b * V + v) * cs + cg * 8, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += f[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = slot < nslots ? a[e] : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int k = 0; k < nslots; ++k) s += red[(k * ncg + (c >> 3)) * 8 + (c & 7)];
    // [B][gridDim.x][C] partials; chs_reduce_kernel adds them in workgroup order
    part[((long long)b * gridDim.x + blk) * C + c] = s;
  }
}

// maxabs (optional): max |p| before the update and max |g| (TrainLoop.run_step's norm/param_max and
// norm/grad_max, train_util.py:370-375 of the reference) from the same pass, as the bit patterns of
// non-negative floats -- unsigned order = float order, a NaN above +inf, so NaN propagates -- one
// atomic max per workgroup (exact whatever the order)
// DEV (the sync-free loss-scaled step): the step count lives on the device (dstep, the
// steps taken so far) and found_inf (GradScaler's, after unscale_) skips the whole
// update, as GradScaler.step skips optimizer.step; the bias corrections are the host's
// double-precision formulas on the device count (adamw_step_inc advances it afterwards)
template <bool DEV>
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n,
                                                   float decay, float w1, float b2, float w2, float neg_step,
                                                   float bc2_sqrt, float eps, unsigned* __restrict__ maxabs,
                                                   const double* __restrict__ dstep, const float* __restrict__ found_inf,
                                                   double lr, double beta1, double beta2) {
  if constexpr (DEV) {
    if (found_inf && *found_inf != 0.f) return;
    const double sd = *dstep + 1.0;
    const double bc1 = 1.0 - pow(beta1, sd), bc2 = 1.0 - pow(beta2, sd);
    neg_step = (float)(-(lr / bc1));
    bc2_sqrt = (float)sqrt(bc2);
  }
  const long long stride = (long long)gridDim.x * blockDim.x;
  unsigned mp = 0u, mg = 0u;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i];
    const float p0 = p[i];
    mp = max(mp, __float_as_uint(fabsf(p0)));
    mg = max(mg, __float_as_uint(fabsf(gi)));
    float pi = p0 * decay;
    const float mi = m[i] + w1 * (gi - m[i]);
    const float vi = v[i] * b2 + w2 * (gi * gi);
    const float den = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + neg_step * (mi / den);
    p[i] = pi; m[i] = mi; v[i] = vi;
  }
  if (!maxabs) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mp = max(mp, (unsigned)__shfl_xor((int)mp, o, 64));
    mg = max(mg, (unsigned)__shfl_xor((int)mg, o, 64));
  }
  __shared__ unsigned red[2][4];
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = mp; red[1][threadIdx.x >> 6] = mg; }
  __syncthreads();
  if (threadIdx.x == 0) {
    mp = max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3]));
    mg = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
    atomicMax(maxabs, mp);
    atomicMax(maxabs + 1, mg);
  }
}

__global__ void adamw_step_inc(double* __restrict__ dstep, const float* __restrict__ found_inf) {
  if (threadIdx.x == 0 && !(found_inf && *found_inf != 0.f)) *dstep = *dstep + 1.0;
}

__device__ __forceinline__ float silu_ref(float v) { return v / (1.0f + expf(-v)); }
__device__ __forceinline__ float dsilu_ref(float z) {
  const float s = 1.0f / (1.0f + expf(-z));
  return s * (1.0f + z * (1.0f - s));
}

// emb projection of one ResBlock (rows [0, n) of the block; dEb stride R), one element per
// thread of workgroup blk (of 1024 threads)
__device__ __forceinline__ void emb_bwd_w(const float* __restrict__ dEb, int R, int n, int B,
                                          const float* __restrict__ temb, int E, float* __restrict__ dw,
                                          float* __restrict__ db, float* __restrict__ dcb, int acc, int blk) {
  const long long i = (long long)blk * 1024 + threadIdx.x;
  if (i >= (long long)n * E) return;
  const int r = (int)(i / E), e = (int)(i % E);
  float s = 0.f, sb = 0.f;
  for (int b = 0; b < B; ++b) {
    const float g = dEb[(long long)b * R + r];
    s += g * silu_ref(temb[(long long)b * E + e]);
    sb += g;
  }
  dw[i] = acc ? dw[i] + s : s;
  if (e == 0) {
    db[r] = acc ? db[r] + sb : sb;
    if (dcb) dcb[r] = acc ? dcb[r] + sb : sb;
  }
}

// dsil[b][e] += sum_r W[r][e] * dEb[b][r]: one 1024-thread block per (16 e, b),
// 64 row groups over all n rows, the group sums added in group order -- one
// writer per element, a fixed summation order (no atomics: deterministic)
__device__ __forceinline__ void emb_bwd_x(const float* __restrict__ dEb, int R, int n, const float* __restrict__ W,
                                          int E, float* __restrict__ dsil, int bx, int b) {
  __shared__ float red[1024];
  const int e = bx * 16 + (threadIdx.x & 15), rg = threadIdx.x >> 4;
  float s = 0.f;
  if (e < E)
    for (int r = rg; r < n; r += 64) s += W[(long long)r * E + e] * dEb[(long long)b * R + r];
  red[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0 && e < E) {
    float t = 0.f;
    for (int q = 0; q < 64; ++q) t += red[threadIdx.x + 16 * q];
    dsil[(long long)b * E + e] += t;
  }
}

// both halves of a ResBlock's emb_layers backward in ONE launch (they read dEb and write
// disjoint outputs): workgroups [0, nwb) the weight / bias gradient, the rest (16 e, b) of dsil
__global__ void __launch_bounds__(1024) emb_bwd_kernel(const float* __restrict__ dEb, int R, int n, int B,
                                                      const float* __restrict__ temb, int E,
                                                      const float* __restrict__ W, float* __restrict__ dw,
                                                      float* __restrict__ db, float* __restrict__ dcb, int acc,
                                                      float* __restrict__ dsil, int nwb, int nxe) {
  const int blk = (int)blockIdx.x;
  if (blk < nwb) {
    emb_bwd_w(dEb, R, n, B, temb, E, dw, db, dcb, acc, blk);
  } else {
    const int x = blk - nwb;
    emb_bwd_x(dEb, R, n, W, E, dsil, x % nxe, x / nxe);
  }
}

// time_embed MLP backward (unet.py:534-539).  TEMB_G workgroups: each recomputes the
// batch's sinusoids, layer-1 pre-activation and dt = dsil * SiLU'(temb) (B x E values, a
// 64-term dot each), then owns a slice of TEMB_R rows of E: dh for its slice (each 256-term
// dot split over 16 lanes, lane sums added in a fixed butterfly order), dw2 / dw1 / db2 / db1
// rows of its slice.  One workgroup ran the whole MLP serially: 130 us per training step.
constexpr int TEMB_R = 16;
__global__ void __launch_bounds__(256) temb_bwd_kernel(const float* __restrict__ t, int B, int mc,
                                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                                      const float* __restrict__ w2,
                                                      const float* __restrict__ temb,
                                                      const float* __restrict__ dsil, float* __restrict__ dw1,
                                                      float* __restrict__ db1, float* __restrict__ dw2,
                                                      float* __restrict__ db2) {
  extern __shared__ float sm[];
  const int E = 4 * mc, half = mc / 2;
  float* sinb = sm;                 // [B][mc]
  float* hid = sinb + B * mc;       // [B][E] pre-activation of layer 1
  float* dt = hid + B * E;          // [B][E] gradient of temb
  float* dh = dt + B * E;           // [B][TEMB_R] gradient of the layer-1 pre-activation, this slice
  const int r0 = blockIdx.x * TEMB_R;
  for (int b = 0; b < B; ++b) {
    const float tv = t[b];
    for (int k = threadIdx.x; k < half; k += blockDim.x) {
      const float fr = expf(__fdiv_rn(__fmul_rn(-9.210340371976184f, (float)k), (float)half));
      const float a = __fmul_rn(tv, fr);
      sinb[b * mc + k] = cosf(a);
      sinb[b * mc + k + half] = sinf(a);
    }
    if ((mc & 1) && threadIdx.x == 0) sinb[b * mc + mc - 1] = 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B * E; i += blockDim.x) {
    const int b = i / E, o = i % E;
    float acc = b1[o];
    for (int k = 0; k < mc; ++k) acc += w1[(long long)o * mc + k] * sinb[b * mc + k];
    hid[i] = acc;
    dt[i] = dsil[i] * dsilu_ref(temb[i]);
  }
  __syncthreads();
  // dh[b][k] = SiLU'(hid[b][k]) sum_o w2[o][k] dt[b][o], k in this slice: 16 lanes per (b, k),
  // lane l the terms o = l, l + 16, ...
  {
    const int l = threadIdx.x & 15, kk = threadIdx.x >> 4;   // 16 (b, k) pairs per pass
    for (int q = kk; q < B * TEMB_R; q += 16) {
      const int b = q / TEMB_R, k = r0 + q % TEMB_R;
      float sacc = 0.f;
      if (k < E)
        for (int o = l; o < E; o += 16) sacc += w2[(long long)o * E + k] * dt[b * E + o];
#pragma unroll
      for (int m = 8; m > 0; m >>= 1) sacc += __shfl_xor(sacc, m, 16);
      if (l == 0 && k < E) dh[q] = sacc * dsilu_ref(hid[b * E + k]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TEMB_R * E; i += blockDim.x) {
    const int o = r0 + i / E, k = i % E;
    if (o >= E) continue;
    float s2 = 0.f;
    for (int b = 0; b < B; ++b) s2 += dt[b * E + o] * silu_ref(hid[b * E + k]);
    dw2[(long long)o * E + k] = s2;
  }
  for (int i = threadIdx.x; i < TEMB_R * mc; i += blockDim.x) {
    const int ol = i / mc, o = r0 + ol, k = i % mc;
    if (o >= E) continue;
    float s1 = 0.f;
    for (int b = 0; b < B; ++b) s1 += dh[b * TEMB_R + ol] * sinb[b * mc + k];
    dw1[(long long)o * mc + k] = s1;
  }
  for (int ol = threadIdx.x; ol < TEMB_R; ol += blockDim.x) {
    const int o = r0 + ol;
    if (o >= E) continue;
    float s2 = 0.f, s1 = 0.f;
    for (int b = 0; b < B; ++b) { s2 += dt[b * E + o]; s1 += dh[b * TEMB_R + ol]; }
    db2[o] = s2;
    db1[o] = s1;
  }
}

template <typename F>
int dispatch_mode(int mode, F&& f) {
  if (mode == 0) return f(std::integral_constant<int, 0>{});
  if (mode == 1) return f(std::integral_constant<int, 1>{});
  return f(std::integral_constant<int, 2>{});
}

// voxel blocks of the reduce pass: one trip of 4 voxels per slot (256 / (C / 8)
// voxel slots per workgroup) where that stays below 512 blocks -- the small
// levels ran 1-8 workgroups looping over 512 voxels each (35-70 us per call at
// 16^3 / 8^3, latency-bound) -- else 512 blocks
// reduce-pass workgroups per batch entry: at most 1024 (R0's 64-channel
// reduce at 2 M voxels: 132 us with 512 = 8 waves per CU, 114 us with 1024;
// 2048 no better, profiles/r03/i_gnb_cap.txt)
long long gn_bwd_blocks(int C, long long V) {
  static const long long cap = [] { const char* e = std::getenv("CWDM_GNB_CAP"); return e ? std::atoll(e) : 1024LL; }();
  const long long slots = std::max(1, 256 / std::max(1, C / 8));
  long long nb = ceil_div(V, 4 * slots);
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  return nb;
}

}  // namespace

int launch_emb_bwd(const float* dEb, int R, int n, int B, const float* temb, int E, const float* W, float* dw,
                   float* db, float* dcb, float* dsil, hipStream_t s, int acc) {
  const int nwb = (int)ceil_div((long long)n * E, 1024), nxe = (int)ceil_div(E, 16);
  hipLaunchKernelGGL(emb_bwd_kernel, dim3((unsigned)(nwb + nxe * B)), dim3(1024), 0, s, dEb, R, n, B, temb, E, W, dw,
                     db, dcb, acc, dsil, nwb, nxe);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

int launch_temb_bwd(const float* t, int B, int mc, const float* w1, const float* b1, const float* w2,
                    const float* temb, const float* dsil, float* dw1, float* db1, float* dw2, float* db2,
                    hipStream_t s) {
  const int E = 4 * mc;
  const size_t sm = (size_t)(B * mc + 2 * B * E + B * TEMB_R) * sizeof(float);
  CWDM_REQUIRE(sm <= 64 * 1024, CWDM_E_SHAPE, "time_embed backward: batch too large for one workgroup");
  hipLaunchKernelGGL(temb_bwd_kernel, dim3((unsigned)ceil_div(E, TEMB_R)), dim3(256), sm, s, t, B, mc, w1, b1, w2,
                     temb, dsil, dw1, db1, dw2, db2);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

int gn_silu_bwd_impl(const void* x0, int c0, const void* x1, int c1, const void* du, int du_mode, const float* ss,
                     const float* mr, const float* gamma, int groups, int64_t B, int64_t d, int64_t h, int64_t w,
                     int dtype, void* dx0, int acc0, void* dx1, int acc1, float* dgamma, float* dbeta, void* ws,
                     int64_t ws_bytes, float* chs, int64_t chs_stride, cwdm_stream_t stream, int acc_affine,
                     const float* pre_part = nullptr, int pre_nblk = 0, const float** coef_out = nullptr);
// Fixed-order slice sums of [B][nblk][W2] partial rows -> [B][slices][W2]
// (the fused GroupNorm-backward partials: one row per dgrad tile, 4096 at
// 128^3, too many for the single-workgroup gn_bwd_finalize).  Workgroup (slice,
// b); thread f sums column f over its rows in order, 8 loads in flight.
__global__ void __launch_bounds__(256) gb_part_reduce_kernel(const float* __restrict__ in, int nblk, int W2, int per,
                                                             float* __restrict__ out) {
  const int sl = blockIdx.x, b = blockIdx.y, S = gridDim.x;
  const int r0 = sl * per, r1 = min(nblk, r0 + per);
  const float* base = in + (long long)b * nblk * W2;
  for (int f = threadIdx.x; f < W2; f += 256) {
    float acc = 0.f;
    int r = r0;
    for (; r + 8 <= r1; r += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = base[(long long)(r + k) * W2 + f];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; r < r1; ++r) acc += base[(long long)r * W2 + f];
    out[((long long)b * S + sl) * W2 + f] = acc;
  }
}

int gb_part_reduce(const float* part, int nblk, int C, int64_t B, int slices, float* out, hipStream_t s) {
  CWDM_REQUIRE(nblk > 0 && slices > 0 && B > 0 && B < 65536, CWDM_E_SHAPE, "gb_part_reduce: bad shape");
  const int per = (int)ceil_div(nblk, slices);
  hipLaunchKernelGGL(gb_part_reduce_kernel, dim3((unsigned)slices, (unsigned)B), dim3(256), 0, s, part, nblk, 2 * C,
                     per, out);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
}  // namespace cwdm

using namespace cwdm;

extern "C" int64_t cwdm_gn_silu_bwd_workspace_bytes(int C, int64_t B, int64_t d, int64_t h, int64_t w) {
  if (C <= 0 || B <= 0 || d <= 0 || h <= 0 || w <= 0) return -1;
  const long long nb = gn_bwd_blocks(C, d * h * w);
  const int64_t part = B * nb * C * 2 * 4;
  // partials, coefficients, then the fused channel sums' per-workgroup partials (<= 1024 per batch entry)
  return (part + 255) / 256 * 256 + (B * (int64_t)C * 4 * 4 + 255) / 256 * 256 + B * 1024LL * C * 4;
}

// cwdm_gn_silu_bwd, plus (chs != nullptr, single source, C / 8 dividing 256)
// the per-channel sums of dx0 added to chs[b * chs_stride + c] (unet_plan.cpp:
// the conv1-output sums of the emb-projection backward).
int cwdm::gn_silu_bwd_impl(const void* x0, int c0, const void* x1, int c1, const void* du, int du_mode,
                           const float* ss, const float* mr, const float* gamma, int groups, int64_t B, int64_t d,
                           int64_t h, int64_t w, int dtype, void* dx0, int acc0, void* dx1, int acc1, float* dgamma,
                           float* dbeta, void* ws, int64_t ws_bytes, float* chs, int64_t chs_stride,
                           cwdm_stream_t stream, int acc_affine, const float* pre_part, int pre_nblk,
                           const float** coef_out) {
  CWDM_REQUIRE(!chs || (c1 == 0 && chs_stride >= c0), CWDM_E_UNSUPPORTED,
               "gn_silu_bwd: fused channel sums need one source");
  CWDM_REQUIRE(x0 && du && ss && mr && gamma && dx0 && dgamma && dbeta && ws, CWDM_E_INVALID,
               "cwdm_gn_silu_bwd: null pointer");
  CWDM_REQUIRE(c1 == 0 || (x1 && dx1), CWDM_E_INVALID, "cwdm_gn_silu_bwd: second source missing");
  const int C = c0 + c1;
  CWDM_REQUIRE(c0 % 8 == 0 && c1 % 8 == 0 && C <= 1024 && C / 8 <= 256, CWDM_E_UNSUPPORTED,
               "cwdm_gn_silu_bwd: channels must be multiples of 8, at most 1024");
  CWDM_REQUIRE(groups > 0 && groups <= 256 && C % groups == 0, CWDM_E_SHAPE, "cwdm_gn_silu_bwd: bad groups");
  CWDM_REQUIRE(du_mode >= 0 && du_mode <= 2, CWDM_E_INVALID, "cwdm_gn_silu_bwd: bad du_mode");
  CWDM_REQUIRE(du_mode != 2 || (d % 2 == 0 && h % 2 == 0 && w % 2 == 0), CWDM_E_SHAPE,
               "cwdm_gn_silu_bwd: pooled grid must be even");
  CWDM_REQUIRE(dtype_compute(dtype), CWDM_E_INVALID, "cwdm_gn_silu_bwd: bad dtype");
  CWDM_REQUIRE(B > 0 && B < 65536 && d > 0 && h > 0 && w > 0, CWDM_E_SHAPE, "cwdm_gn_silu_bwd: empty grid");
  CWDM_REQUIRE(ws_bytes >= cwdm_gn_silu_bwd_workspace_bytes(C, B, d, h, w), CWDM_E_WORKSPACE,
               "cwdm_gn_silu_bwd: workspace too small");
  CWDM_REQUIRE(d * h * w * (C / 8) < (1LL << 31) - 256LL * 1024, CWDM_E_UNSUPPORTED,
               "cwdm_gn_silu_bwd: more than 2^31 channel groups per batch entry");
  const long long V = d * h * w;
  const long long nb = gn_bwd_blocks(C, V);
  const long long vpb = ceil_div(V, nb);
  float* part = reinterpret_cast<float*>(ws);
  float* coef = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(ws) + (B * nb * C * 2 * 4 + 255) / 256 * 256);
  float* chs_part = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(coef) + (B * (int64_t)C * 4 * 4 + 255) / 256 * 256);
  hipStream_t s = (hipStream_t)stream;
  int rc;
  // pre_part: the (sum dz, sum dz xhat) partials already written by the epilogue
  // of the dgrad conv that produced du ([B][pre_nblk][C][2], cwdm::GbwdFuse)
  CWDM_REQUIRE(!pre_part || (du_mode == 0 && pre_nblk > 0), CWDM_E_INVALID, "gn_silu_bwd: bad fused partials");
  if (!pre_part && (rc = dispatch_mode(du_mode, [&](auto M) -> int {
         constexpr int MD = decltype(M)::value;
         dispatch_dtype(dtype, [&](auto tag) -> int {
           using T = decltype(tag);
           hipLaunchKernelGGL((gn_bwd_reduce_kernel<T, MD>), dim3((unsigned)nb, (unsigned)B), dim3(256), 0, s,
                              (const T*)x0, c0, (const T*)x1, c1, (const T*)du, ss, mr, groups, (int)d,
                              (int)h, (int)w, vpb, part);
           return CWDM_OK;
         });
         CWDM_LAUNCHED();
         return CWDM_OK;
       })))
    return rc;
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3((unsigned)groups), dim3(256), 0, s, pre_part ? pre_part : part,
                     pre_part ? pre_nblk : (int)nb, C, (int)B, gamma, mr, groups, V, coef, dgamma, dbeta, acc_affine);
  CWDM_LAUNCHED();
  // coef_out: reduce + finalize only; the caller fuses the apply into a
  // later kernel (cwdm::GapplyFuse) reading coef ([B][C][4]) from the workspace
  if (coef_out) {
    CWDM_REQUIRE(!chs, CWDM_E_INVALID, "gn_silu_bwd: deferred apply with channel sums");
    *coef_out = coef;
    return CWDM_OK;
  }
  // workgroups of (256 / ncg) voxels x ncg channel groups; two voxels per
  // thread (the kernel's UNR; du_mode 1 loops twice instead); with channel
  // sums at most 1024 workgroups per batch entry (one partial row each, summed
  // in workgroup order by chs_reduce_kernel), each looping over its share
  // (at most 1024 workgroups per batch entry in every case: each thread loads its
  // 40 coefficient words once and loops; one voxel pair per thread spent more
  // load instructions on coefficients than on the tensors -- R0 64-channel
  // apply 216 us with one pair per thread vs 160 us capped, same trace)
  const int ncg = C / 8, nvb = 256 / ncg;
  long long nblk = ceil_div(V, 2LL * nvb);
  if (nblk > 1024) nblk = 1024;
  dim3 grid((unsigned)nblk, (unsigned)B);
  const dim3 block((unsigned)(nvb * ncg));
  float* cp = chs ? chs_part : nullptr;
  if ((rc = dispatch_mode(du_mode, [&](auto M) -> int {
         constexpr int MD = decltype(M)::value;
         dispatch_dtype(dtype, [&](auto tag) -> int {
           using T = decltype(tag);
           hipLaunchKernelGGL((gn_bwd_apply_kernel<T, MD>), grid, block, 0, s, (const T*)x0, c0,
                              (const T*)x1, c1, (const T*)du, ss, coef, (int)d, (int)h, (int)w, (T*)dx0,
                              acc0, (T*)dx1, acc1, cp, (long long)chs_stride);
           return CWDM_OK;
         });
         CWDM_LAUNCHED();
         return CWDM_OK;
       })))
    return rc;
  if (chs) {
    hipLaunchKernelGGL(chs_reduce_kernel, dim3((unsigned)ceil_div(C, 64)), dim3(1024), 0, s, chs_part, (int)nblk, C,
                       chs, (long long)chs_stride, nullptr, nullptr, (int)B);
    CWDM_LAUNCHED();
  }
  return CWDM_OK;
}

extern "C" int cwdm_gn_silu_bwd(const void* x0, int c0, const void* x1, int c1, const void* du, int du_mode,
                                const float* ss, const float* mr, const float* gamma, int groups, int64_t B,
                                int64_t d, int64_t h, int64_t w, int dtype, void* dx0, int acc0, void* dx1, int acc1,
                                float* dgamma, float* dbeta, void* ws, int64_t ws_bytes, cwdm_stream_t stream) {
  return gn_silu_bwd_impl(x0, c0, x1, c1, du, du_mode, ss, mr, gamma, groups, B, d, h, w, dtype, dx0, acc0, dx1, acc1,
                          dgamma, dbeta, ws, ws_bytes, nullptr, 0, stream, 0);
}

extern "C" int cwdm_resample_add(void* dst, const void* src, int C, int64_t B, int64_t d, int64_t h, int64_t w,
                                 int mode, int accumulate, int dtype, cwdm_stream_t stream) {
  CWDM_REQUIRE(dst && src, CWDM_E_INVALID, "cwdm_resample_add: null pointer");
  CWDM_REQUIRE(dtype_compute(dtype), CWDM_E_INVALID, "cwdm_resample_add: bad dtype");
  CWDM_REQUIRE(C > 0 && C % 8 == 0, CWDM_E_UNSUPPORTED, "cwdm_resample_add: channels must be a multiple of 8");
  CWDM_REQUIRE(mode >= 0 && mode <= 2, CWDM_E_INVALID, "cwdm_resample_add: bad mode");
  CWDM_REQUIRE(mode != 2 || (d % 2 == 0 && h % 2 == 0 && w % 2 == 0), CWDM_E_SHAPE, "cwdm_resample_add: odd grid");
  CWDM_REQUIRE(B > 0 && B < 65536 && d > 0 && h > 0 && w > 0, CWDM_E_SHAPE, "cwdm_resample_add: empty grid");
  CWDM_REQUIRE(d * h * w * (C / 8) < (1LL << 31) - 256, CWDM_E_UNSUPPORTED,
               "cwdm_resample_add: more than 2^31 channel groups per batch entry");
  const long long V = d * h * w;
  const FastDiv dncg = make_fastdiv((unsigned)(C / 8));
  dim3 grid((unsigned)ceil_div(V * (C / 8), 256), (unsigned)B);
  hipStream_t s = (hipStream_t)stream;
  return dispatch_mode(mode, [&](auto M) -> int {
    constexpr int MD = decltype(M)::value;
    dispatch_dtype(dtype, [&](auto tag) -> int {
      using T = decltype(tag);
      hipLaunchKernelGGL((resample_add_kernel<T, MD>), grid, dim3(256), 0, s, (T*)dst, (const T*)src, C,
                         (int)d, (int)h, (int)w, accumulate, dncg);
      return CWDM_OK;
    });
    CWDM_LAUNCHED();
    return CWDM_OK;
  });
}

namespace {
// voxel blocks: ~8 loads per voxel slot (256 / (C / 8) slots per workgroup),
// at most 512 -- the small levels ran 1-2 workgroups over 2048 voxels each
// (70 us per call at 16^3 x 256 channels, latency-bound)
long long channel_sum_blocks(int64_t V, int C) {
  const long long slots = std::max(1, 256 / std::max(1, (C + 7) / 8));
  long long nb = ceil_div(V, 8 * slots);
  return nb > 512 ? 512 : (nb < 1 ? 1 : nb);
}
}  // namespace

extern "C" int64_t cwdm_channel_sum_workspace_bytes(int64_t B, int64_t V, int C) {
  if (B <= 0 || V <= 0 || C <= 0) return -1;
  return B * channel_sum_blocks(V, C) * C * 4;
}

extern "C" int cwdm_channel_sum(const void* src, int dtype, int64_t B, int64_t V, int C, int cs, float* out_bc,
                                int64_t bc_stride, float* out_c, float* out_c2, void* workspace, int64_t ws_bytes,
                                cwdm_stream_t stream) {
  CWDM_REQUIRE(src, CWDM_E_INVALID, "cwdm_channel_sum: null pointer");
  CWDM_REQUIRE(dtype_compute(dtype), CWDM_E_INVALID, "cwdm_channel_sum: bad dtype");
  CWDM_REQUIRE(C > 0 && cs >= ((C + 7) / 8) * 8 && cs % 8 == 0 && cs <= 2048, CWDM_E_UNSUPPORTED,
               "cwdm_channel_sum: stride must be a multiple of 8 covering C (<= 2048)");
  CWDM_REQUIRE(B > 0 && B < 65536 && V > 0, CWDM_E_SHAPE, "cwdm_channel_sum: empty input");
  CWDM_REQUIRE(workspace && ws_bytes >= cwdm_channel_sum_workspace_bytes(B, V, C), CWDM_E_WORKSPACE,
               "cwdm_channel_sum: workspace (cwdm_channel_sum_workspace_bytes) missing or too small");
  const long long nb = channel_sum_blocks(V, C);
  const long long vpb = ceil_div(V, nb);
  dim3 grid((unsigned)nb, (unsigned)B);
  hipStream_t s = (hipStream_t)stream;
  float* part = reinterpret_cast<float*>(workspace);
  dispatch_dtype(dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL(channel_sum_kernel<T>, grid, dim3(256), 0, s, (const T*)src, (long long)V, C, cs, vpb, part);
    return CWDM_OK;
  });
  CWDM_LAUNCHED();
  hipLaunchKernelGGL(chs_reduce_kernel, dim3((unsigned)ceil_div(C, 64)), dim3(1024), 0, s, part, (int)nb, C, out_bc,
                     (long long)bc_stride, out_c, out_c2, (int)B);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

namespace {
int adamw_launch(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1, double beta2,
                 double eps, double weight_decay, int64_t step, float* maxabs, cwdm_stream_t stream) {
  CWDM_REQUIRE(p && g && m && v, CWDM_E_INVALID, "cwdm_adamw: null pointer");
  CWDM_REQUIRE(n >= 0 && step >= 1, CWDM_E_INVALID, "cwdm_adamw: bad size/step");
  if (maxabs) CWDM_HIP(hipMemsetAsync(maxabs, 0, 2 * sizeof(float), (hipStream_t)stream));
  if (n == 0) return CWDM_OK;
  // scalars as torch computes them (Python doubles, cast to float at the kernel)
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float decay = (float)(1.0 - lr * weight_decay);
  const float neg_step = (float)(-(lr / bc1));
  const float bc2s = (float)std::sqrt(bc2);
  long long blocks = ceil_div(n, 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adamw_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v,
                     (long long)n, decay, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), neg_step, bc2s,
                     (float)eps, reinterpret_cast<unsigned*>(maxabs), nullptr, nullptr, lr, beta1, beta2);
  CWDM_LAUNCHED();
  return CWDM_OK;
}
}  // namespace

extern "C" int cwdm_adamw_device_step(float* p, const float* g, float* m, float* v, int64_t n, double lr,
                                      double beta1, double beta2, double eps, double weight_decay, double* step,
                                      const float* found_inf, cwdm_stream_t stream) {
  CWDM_REQUIRE(p && g && m && v && step, CWDM_E_INVALID, "cwdm_adamw_device_step: null pointer");
  CWDM_REQUIRE(n >= 0, CWDM_E_INVALID, "cwdm_adamw_device_step: bad size");
  hipStream_t s = (hipStream_t)stream;
  if (n > 0) {
    const float decay = (float)(1.0 - lr * weight_decay);
    long long blocks = ceil_div(n, 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(adamw_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, (long long)n, decay,
                       (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), 0.f, 1.f, (float)eps, nullptr, step,
                       found_inf, lr, beta1, beta2);
    CWDM_LAUNCHED();
  }
  hipLaunchKernelGGL(adamw_step_inc, dim3(1), dim3(64), 0, s, step, found_inf);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

extern "C" int cwdm_adamw(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                          double beta2, double eps, double weight_decay, int64_t step, cwdm_stream_t stream) {
  return adamw_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step, nullptr, stream);
}

extern "C" int cwdm_adamw_maxabs(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                                 double beta2, double eps, double weight_decay, int64_t step, float* maxabs,
                                 cwdm_stream_t stream) {
  CWDM_REQUIRE(maxabs, CWDM_E_INVALID, "cwdm_adamw_maxabs: null maxabs");
  return adamw_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step, maxabs, stream);
}
