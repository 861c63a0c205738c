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
#include <atomic>

#include "conv3d_kernels.hpp"

namespace cwdm {

struct HeadParams {
  int B, D, H, W, C, cout;
  int tx, ty, tz;
  const void* x;            // [B][V][C] channels-last, bf16 or fp16
  const float* gn;          // [B][C][2] scale / shift (null: no GroupNorm+SiLU)
  const unsigned char* w;   // packed, NT = 32
  const float* bias; long long bias_bs;
  void* out; int out_f32;   // [B][V][cout]
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

// T: the 16-bit storage type (bf16 / fp16)
template <typename T>
__global__ void __launch_bounds__(256, 2) head_conv_kernel(HeadParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char halo[HEAD_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = lane & 15, kg = lane >> 4;
  const int tiles = p.tx * p.ty * p.tz;
  const int b = blockIdx.x / tiles, sl = blockIdx.x - b * tiles;
  const int x0 = (sl % p.tx) * 32, y0 = ((sl / p.tx) % p.ty) * 4, z0 = (sl / (p.tx * p.ty)) * 4;
  const long long V = (long long)p.D * p.H * p.W;
  const int nh = p.C / 32;
  const int nch = p.C / 16;  // 16-channel chunks of the packed weights

  hf32x4 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int xb = 0; xb < 2; ++xb) acc[m][xb] = hf32x4{0.f, 0.f, 0.f, 0.f};

  // fill work: item i = tid + 256 k -> halo voxel i >> 2, quad i & 3 (= tid & 3 for every k)
  constexpr int NFILL = (HHV * 4 + 255) / 256;  // 20
  const int fq = tid & 3;
  // this lane's A-operand base: voxel (x = n, line 0, plane wv) of the halo, K group kg
  const int abase = ((wv * HHY) * HHX + n) * 64 + kg * 16;

  for (int h = 0; h < nh; ++h) {
    if (h) __syncthreads();  // the previous half's operand reads are done
    float sc[8], sh[8];
    const int cq = h * 32 + fq * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = p.gn ? p.gn[((long long)b * p.C + cq + e) * 2] : 1.f;
      sh[e] = p.gn ? p.gn[((long long)b * p.C + cq + e) * 2 + 1] : 0.f;
    }
    u32x4 v[NFILL];
    bool ok[NFILL];
#pragma unroll
    for (int k = 0; k < NFILL; ++k) {
      const int i = tid + 256 * k;
      const int hv = i >> 2;
      const int hx = hv % HHX, hy = (hv / HHX) % HHY, hz = hv / (HHX * HHY);
      const int ox = x0 + hx - 1, oy = y0 + hy - 1, oz = z0 + hz - 1;
      ok[k] = hv < HHV && ox >= 0 && oy >= 0 && oz >= 0 && ox < p.W && oy < p.H && oz < p.D;
      v[k] = u32x4{0u, 0u, 0u, 0u};
      if (ok[k]) {
        const long long vox = (long long)b * V + ((long long)oz * p.H + oy) * p.W + ox;
        v[k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(p.x) + vox * p.C + cq);
      }
    }
#pragma unroll
    for (int k = 0; k < NFILL; ++k) {
      const int i = tid + 256 * k;
      if ((i >> 2) < HHV) {
        u32x4 q = u32x4{0u, 0u, 0u, 0u};
        if (ok[k]) {
          float f[8];
          unpack<T>(v[k], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = p.gn ? silu(f[e] * sc[e] + sh[e]) : f[e];
          q = pack<T>(f);
        }
        *reinterpret_cast<u32x4*>(halo + (i >> 2) * 64 + fq * 16) = q;
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
    (void)nch;
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
         d->W % 32 == 0 && d->H % 4 == 0 && d->D % 4 == 0;
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
  if (d->dtype == CWDM_F16) hipLaunchKernelGGL(head_conv_kernel<f16_t>, dim3((unsigned)nblk), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(head_conv_kernel<bf16_t>, dim3((unsigned)nblk), dim3(256), 0, s, p);
  prof_end(s, 2.0 * p.B * p.D * p.H * p.W * (double)p.cout * 27.0 * p.C);
  CWDM_LAUNCHED();
  return CWDM_OK;
}

}  // namespace cwdm
