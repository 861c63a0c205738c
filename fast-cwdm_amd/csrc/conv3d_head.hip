// Output head of the U-Net (unet.py `out`: GroupNorm -> SiLU -> conv3x3x3,
// model_channels -> out_channels = 8): a narrow-output conv with its
// GroupNorm+SiLU fused into the halo staging.
//
// The general kernels tile 32 / 64 output channels per MFMA; with 8 outputs
// that wastes 4-8x of the matrix work and the head ran at ~130 TF/s
// (~0.55 ms of the 128^3 step).  Here the MFMA is v_mfma_f32_16x16x32_bf16 (/ _f16)
// with A = 16 voxels x 32 input channels (from LDS) and B = 32 input channels
// x 16 output channels (8 real + zero rows, held in registers per tap): half
// the lanes of the product are useful instead of an eighth.
//
//   * Tile 32(x) x 4(y) x 4(z) voxels, 4 waves, wave w = output z-plane w:
//     4 lines x 2 x-blocks of 16 voxels = 8 accumulators (f32x4).
//   * Input channels in halves of 32: the 34 x 6 x 6 halo of a half (64 B per
//     voxel, 78 KB, so two workgroups share a CU) is loaded with 16-byte
//     loads, GroupNorm+SiLU applied in registers, zero-padded and written to
//     LDS.  A ds_read_b128 of a wave covers 16 consecutive voxels x 64 B:
//     conflict-free.  For each (dz, dx) the 6 input lines are read once and
//     used by the 3 dy taps (24 MFMAs per 12 reads).
//   * Weights come from the standard packed layout (cwdm_conv3d_pack, NT = 32
//     rows per channel tile; rows >= cout are zero).
//
// SAMP variant (cwdm_unet_forward_step): the sampling step's epilogue runs on
// the accumulators -- the tile's 512 x 8 fp32 outputs (+ bias) go through LDS
// to one thread per voxel, which applies sampler_voxel8 (sampler.hpp; the same
// function as cwdm_sampler_step, so the bits match the unfused step) and
// stores x_{t-1}, the optional pred_xstart and the 16-bit mirror into the next
// step's U-Net input.  The fp32 model output never reaches HBM, and with
// Philox noise neither does the noise tensor.
#include <atomic>
#include <cstdlib>

#include "conv3d_kernels.hpp"
#include "sampler.hpp"

namespace cwdm {

struct HeadParams {
  int B, D, H, W, C, cout;
  int tx, ty, tz;
  const void* x;            // [B][V][C] channels-last, bf16 or fp16
  const float* gn;          // [B][C][2] scale / shift (null: no GroupNorm+SiLU)
  const unsigned char* w;   // packed, NT = 32
  const float* bias; long long bias_bs;
  void* out; int out_f32;   // [B][V][cout]
  cwdm_sampler_args samp;   // SAMP only: the step (out unused)
  int mir_vec;              // SAMP: the mirror's 8 channels are 16-byte vectors
};

namespace {

constexpr int HHX = 34, HHY = 6, HHZ = 6, HHV = HHX * HHY * HHZ;  // 1224 halo voxels
constexpr int HEAD_LDS = HHV * 64;                                 // 78336 B

typedef __bf16 hbf16x8 __attribute__((ext_vector_type(8)));
typedef float hf32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ hf32x4 head_mfma(const u32x4& a, const u32x4& b, hf32x4 acc, bf16_t*) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hbf16x8, a), __builtin_bit_cast(hbf16x8, b), acc,
                                                 0, 0, 0);
}
__device__ __forceinline__ hf32x4 head_mfma(const u32x4& a, const u32x4& b, hf32x4 acc, f16_t*) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0,
                                                0, 0);
}

// T: the 16-bit storage type (bf16 / fp16); SAMP: run the sampler epilogue
// with mirror type MirT (T or fp32)
template <typename T, bool GN, bool SAMP = false, typename MirT = T>
__global__ void __launch_bounds__(256, 2) head_conv_kernel(HeadParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char halo[HEAD_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = lane & 15, kg = lane >> 4;
  const int tiles = p.tx * p.ty * p.tz;
  // XCD-aware: workgroups are dealt round robin to the 8 XCDs; XCD j runs one
  // contiguous run of the x-fastest tile order, so a tile's y / z neighbours
  // (whose halos overlap its own 2.25x) are fetched into the same L2 (the
  // plain order put y neighbours, tx = 4 apart, on different XCDs: 3.5x the
  // input read from HBM)
  const int nb = (int)gridDim.x, xj = (int)(blockIdx.x & 7), q8 = nb >> 3, r8 = nb & 7;
  const int bid = (xj < r8 ? xj * (q8 + 1) : r8 * (q8 + 1) + (xj - r8) * q8) + (int)(blockIdx.x >> 3);
  const int b = bid / tiles, sl = bid - b * tiles;
  const int x0 = (sl % p.tx) * 32, y0 = ((sl / p.tx) % p.ty) * 4, z0 = (sl / (p.tx * p.ty)) * 4;
  const long long V = (long long)p.D * p.H * p.W;
  const int nh = p.C / 32;

  hf32x4 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int xb = 0; xb < 2; ++xb) acc[m][xb] = hf32x4{0.f, 0.f, 0.f, 0.f};

  // fill work: item i = tid + 256 k -> halo voxel i >> 2, quad i & 3 (= tid & 3 for every k);
  // the element offset (voxel * C, within the batch) of each item, -1 outside the volume
  constexpr int NFILL = (HHV * 4 + 255) / 256;  // 20
  const int fq = tid & 3;
  const T* xb = reinterpret_cast<const T*>(p.x) + (long long)b * V * p.C;
  int foff[NFILL];
#pragma unroll
  for (int k = 0; k < NFILL; ++k) {
    const int hv = (tid + 256 * k) >> 2;
    const int hx = hv % HHX, hy = (hv / HHX) % HHY, hz = hv / (HHX * HHY);
    const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
    const bool ok = hv < HHV && ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D;
    foff[k] = ok ? ((oz * p.H + oy) * p.W + ox) * p.C + fq * 8 : -1;
  }
  // this lane's A-operand base: voxel (x = n, line 0, plane wv) of the halo, K group kg
  const int abase = ((wv * HHY) * HHX + n) * 64 + kg * 16;

  for (int h = 0; h < nh; ++h) {
    if (h) __syncthreads();  // the previous half's operand reads are done
    float sc[8], sh[8];
    if constexpr (GN) {
      const float2* g2 = reinterpret_cast<const float2*>(p.gn) + (long long)b * p.C + h * 32 + fq * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 v2 = g2[e];
        sc[e] = v2.x;
        sh[e] = v2.y;
      }
    }
    u32x4 v[NFILL];
#pragma unroll
    for (int k = 0; k < NFILL; ++k) {
      v[k] = u32x4{0u, 0u, 0u, 0u};
      if (foff[k] >= 0) v[k] = *reinterpret_cast<const u32x4*>(xb + foff[k] + h * 32);
    }
#pragma unroll
    for (int k = 0; k < NFILL; ++k) {
      const int i = tid + 256 * k;
      if ((i >> 2) < HHV) {
        u32x4 q = v[k];
        if (GN && foff[k] >= 0) {
          float f[8];
          unpack<T>(v[k], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = silu(f[e] * sc[e] + sh[e]);
          q = pack<T>(f);
        }
        *reinterpret_cast<u32x4*>(halo + i * 16) = q;
      }
    }
    // B operands of this half: tap t, lane (n, kg) = W[co n][ci h 32 + 8 kg .. + 8][t]
    u32x4 wr[27];
    {
      const int chunk = 2 * h + (kg >> 1), q = kg & 1;
      const unsigned char* src = p.w + ((long long)chunk * 27 * 32 + n) * 32 + ((q ^ ((n >> 3) & 1)) << 4);
#pragma unroll
      for (int t = 0; t < 27; ++t) wr[t] = *reinterpret_cast<const u32x4*>(src + (long long)t * 32 * 32);
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 9; ++g) {
      const int dz = g / 3, dx = g % 3;  // 0..2 (offset - 1)
      u32x4 a[6][2];
#pragma unroll
      for (int L = 0; L < 6; ++L)
#pragma unroll
        for (int xb = 0; xb < 2; ++xb)
          a[L][xb] = *reinterpret_cast<const u32x4*>(halo + abase + (((dz * HHY) + L) * HHX + xb * 16 + dx) * 64);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const u32x4 wb = wr[dz * 9 + dy * 3 + dx];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int xb = 0; xb < 2; ++xb) acc[m][xb] = head_mfma(a[m + dy][xb], wb, acc[m][xb], (T*)nullptr);
      }
    }
  }
  // epilogue: lane (n, kg) holds output channel n of voxels x = 16 xb + 4 kg + i
  if constexpr (SAMP) {
    // this thread's 2 voxels (lv = tid, tid + 256 of the tile, x fastest): the
    // x_t (and tensor-noise) loads go out first and fly during the tile exchange
    const cwdm_sampler_args& a = p.samp;
    int64_t t = a.t[b];
    t = t < 0 ? 0 : (t >= a.T ? a.T - 1 : t);
    const int bs = a.per_band ? 8 : 0;
    const float* cf = a.coef + t * (a.per_band ? 64 : 8);
    const bool noisy = a.update != 1 && t != 0;
    int64_t vv[2];
    float xv[2][8], nzv[2][8];
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int lv = tid + 256 * r2;
      vv[r2] = ((int64_t)(z0 + (lv >> 7)) * p.H + y0 + ((lv >> 5) & 3)) * p.W + x0 + (lv & 31);
      const float* xp = a.x_t + b * a.xt_s[0] + vv[r2] * a.xt_s[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[r2][q] = xp[q * a.xt_s[1]];
      if (noisy && a.noise) {
        const float* np = a.noise + b * a.nz_s[0] + vv[r2] * a.nz_s[2];
#pragma unroll
        for (int q = 0; q < 8; ++q) nzv[r2][q] = np[q * a.nz_s[1]];
      }
    }
    __syncthreads();  // every wave's operand reads are done: the halo becomes the output tile
    float* tile = reinterpret_cast<float*>(halo);  // [512 voxels (z, y, x)][8]
    if (n < 8) {
      const float bn = p.bias ? p.bias[(long long)b * p.bias_bs + n] : 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int xb = 0; xb < 2; ++xb)
#pragma unroll
          for (int i = 0; i < 4; ++i) tile[(((wv * 4 + m) * 32) + xb * 16 + 4 * kg + i) * 8 + n] = acc[m][xb][i] + bn;
    }
    const bool philox = noisy && !a.noise && a.noise_philox;
    if (philox) {
#pragma unroll
      for (int r2 = 0; r2 < 2; ++r2) {
        philox_normal4(a.noise_seed, vv[r2], b, t, 0, nzv[r2]);
        philox_normal4(a.noise_seed, vv[r2], b, t, 1, nzv[r2] + 4);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int lv = tid + 256 * r2;
      const int64_t v = vv[r2];
      float m8[8], r[8], pred[8];
      const float4 u0 = *reinterpret_cast<const float4*>(tile + lv * 8);
      const float4 u1 = *reinterpret_cast<const float4*>(tile + lv * 8 + 4);
      m8[0] = u0.x; m8[1] = u0.y; m8[2] = u0.z; m8[3] = u0.w;
      m8[4] = u1.x; m8[5] = u1.y; m8[6] = u1.z; m8[7] = u1.w;
      sampler_voxel8(a, cf, bs, t, m8, xv[r2], noisy && (a.noise || philox), nzv[r2], r, pred);
      float* xo = a.x_prev + b * a.xp_s[0] + v * a.xp_s[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) xo[q * a.xp_s[1]] = r[q];
      if (a.pred_xstart) {
        float* po = a.pred_xstart + b * a.px_s[0] + v * a.px_s[2];
#pragma unroll
        for (int q = 0; q < 8; ++q) po[q * a.px_s[1]] = pred[q];
      }
      if (a.mirror) {
        MirT* o = reinterpret_cast<MirT*>(a.mirror) + b * a.mr_s[0] + v * a.mr_s[2];
        bool done = false;
        if constexpr (sizeof(MirT) == 2) {
          if (p.mir_vec) {
            uint4 q;
            q.x = pack2<MirT>(r[0], r[1]);
            q.y = pack2<MirT>(r[2], r[3]);
            q.z = pack2<MirT>(r[4], r[5]);
            q.w = pack2<MirT>(r[6], r[7]);
            *reinterpret_cast<uint4*>(o) = q;
            done = true;
          }
        }
        if (!done) {
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q * a.mr_s[1]] = Elem<MirT>::from_f(r[q]);
        }
      }
    }
    return;
  }
  if (n < p.cout) {
    const float bn = p.bias ? p.bias[(long long)b * p.bias_bs + n] : 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int xb = 0; xb < 2; ++xb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long long vox =
              (long long)b * V + ((long long)(z0 + wv) * p.H + y0 + m) * p.W + x0 + xb * 16 + 4 * kg + i;
          const float r = acc[m][xb][i] + bn;
          if (p.out_f32) reinterpret_cast<float*>(p.out)[vox * p.cout + n] = r;
          else reinterpret_cast<T*>(p.out)[vox * p.cout + n] = Elem<T>::from_f(r);
        }
  }
}

}  // namespace

extern std::atomic<int> g_conv_path;

bool head_eligible(const cwdm_conv3d_desc* d) {
  if (g_conv_path.load(std::memory_order_relaxed) == 1) return false;
  return dtype_half(d->dtype) && d->a_w && d->cout <= 16 && d->a_c1 == 0 && d->a_c0 % 32 == 0 && d->a_c0 <= 256 &&
         d->a_mode == 0 && !d->b_w && d->res_mode < 0 && !d->stats && !d->out1 && !d->accumulate &&
         d->W % 32 == 0 && d->H % 4 == 0 && d->D % 4 == 0 && d->D * d->H * d->W * d->a_c0 < (1LL << 31);
}

int head_conv_forward(const cwdm_conv3d_desc* d, hipStream_t s) {
  HeadParams p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W; p.C = d->a_c0; p.cout = d->cout;
  p.tx = p.W / 32; p.ty = p.H / 4; p.tz = p.D / 4;
  p.x = d->a0;
  p.gn = d->a_gn;
  p.w = reinterpret_cast<const unsigned char*>(d->a_w);
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.out = d->out; p.out_f32 = d->out_dtype == CWDM_F32;
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d head: grid too large");
  prof_begin(s);
  const dim3 grid((unsigned)nblk);
  if (d->dtype == CWDM_F16) {
    if (p.gn) hipLaunchKernelGGL((head_conv_kernel<f16_t, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<f16_t, false>), grid, dim3(256), 0, s, p);
  } else {
    if (p.gn) hipLaunchKernelGGL((head_conv_kernel<bf16_t, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<bf16_t, false>), grid, dim3(256), 0, s, p);
  }
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * p.C);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

bool head_sampler_eligible(const cwdm_conv3d_desc* d, const cwdm_sampler_args* a) {
  // CWDM_HEAD_SAMPLER=0: the unfused forward + cwdm_sampler_step (A/B switch)
  static const bool on = [] { const char* e = std::getenv("CWDM_HEAD_SAMPLER"); return !(e && e[0] == '0'); }();
  return on && head_eligible(d) && d->a_gn && d->cout == 8 && a->levels <= 1 && a->B == d->B && a->d == d->D && a->h == d->H &&
         a->w == d->W && a->x_t && a->x_prev && a->coef && a->t && a->T > 0 &&
         (!a->mirror || a->mirror_dtype == d->dtype || a->mirror_dtype == CWDM_F32);
}

int head_sampler_forward(const cwdm_conv3d_desc* d, const cwdm_sampler_args* a, hipStream_t s) {
  HeadParams p{};
  p.B = (int)d->B; p.D = (int)d->D; p.H = (int)d->H; p.W = (int)d->W; p.C = d->a_c0; p.cout = d->cout;
  p.tx = p.W / 32; p.ty = p.H / 4; p.tz = p.D / 4;
  p.x = d->a0;
  p.gn = d->a_gn;
  p.w = reinterpret_cast<const unsigned char*>(d->a_w);
  p.bias = d->bias; p.bias_bs = d->bias_bstride;
  p.samp = *a;
  const int mesz = a->mirror ? dtype_size(a->mirror_dtype) : 0;
  p.mir_vec = a->mirror && a->mr_s[1] == 1 && ((uintptr_t)a->mirror % 16) == 0 && (a->mr_s[0] * mesz) % 16 == 0 &&
              (a->mr_s[2] * mesz) % 16 == 0;
  const long long nblk = (long long)p.B * p.tx * p.ty * p.tz;
  CWDM_REQUIRE(nblk < (1LL << 31), CWDM_E_UNSUPPORTED, "conv3d head: grid too large");
  const bool f32m = a->mirror && a->mirror_dtype == CWDM_F32;
  prof_begin(s);
  if (d->dtype == CWDM_F16) {
    if (f32m) hipLaunchKernelGGL((head_conv_kernel<f16_t, true, true, float>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<f16_t, true, true, f16_t>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  } else {
    if (f32m) hipLaunchKernelGGL((head_conv_kernel<bf16_t, true, true, float>), dim3((unsigned)nblk), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((head_conv_kernel<bf16_t, true, true, bf16_t>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  }
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * p.C);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace cwdm
