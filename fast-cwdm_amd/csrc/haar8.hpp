// 2x2x2 Haar analysis / synthesis of one block, every product rounded before
// the add (__fmul_rn / __fadd_rn) in the stage order of the reference's
// matrices (DWT: H, W, D; IDWT: D, W, H) -- shared by wavelet.hip and
// wavelet_nd.hip.
#pragma once
#include "common.hpp"

namespace cwdm {

constexpr float kC = 0.70710677f;  // fp32(1/sqrt(2)) -- pywt rec_lo/rec_hi

// Plain operators under contract(off) (HIP's __fmul_rn / __fadd_rn are plain
// operators defined in a header with contraction allowed): no caller -- also
// one compiled with contraction on, e.g. the fused output head -- can fuse a
// product into the following add
__device__ __forceinline__ float mr(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float ad(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float sb(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

// Analysis of a 2x2x2 block v[a][b][e] (a: D parity, b: H, e: W) into the 8
// bands in reference order LLL, LLH, LHL, LHH, HLL, HLH, HHL, HHH.
__device__ __forceinline__ void haar_fwd8(const float v[8], float o[8]) {
  // stage 1: H (index bit 1)
  float s1[8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float x0 = v[a * 4 + 0 * 2 + e], x1 = v[a * 4 + 1 * 2 + e];
      s1[a * 4 + 0 * 2 + e] = ad(mr(kC, x0), mr(kC, x1));  // L_h
      s1[a * 4 + 1 * 2 + e] = sb(mr(kC, x0), mr(kC, x1));  // H_h
    }
  // stage 2: W (bit 0)
  float s2[8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float x0 = s1[a * 4 + b * 2 + 0], x1 = s1[a * 4 + b * 2 + 1];
      s2[a * 4 + b * 2 + 0] = ad(mr(kC, x0), mr(kC, x1));
      s2[a * 4 + b * 2 + 1] = sb(mr(kC, x0), mr(kC, x1));
    }
  // stage 3: D (bit 2); band index = (pD << 2) | (pH << 1) | pW
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float x0 = s2[0 * 4 + b * 2 + e], x1 = s2[1 * 4 + b * 2 + e];
      o[0 * 4 + b * 2 + e] = ad(mr(kC, x0), mr(kC, x1));
      o[1 * 4 + b * 2 + e] = sb(mr(kC, x0), mr(kC, x1));
    }
}

// Synthesis: bands o[pD<<2|pH<<1|pW] -> block v[a<<2|b<<1|e]; D, then W, then H.
__device__ __forceinline__ void haar_inv8(const float o[8], float v[8]) {
  float s2[8];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float lo = o[0 * 4 + b * 2 + e], hi = o[1 * 4 + b * 2 + e];
      s2[0 * 4 + b * 2 + e] = ad(mr(kC, lo), mr(kC, hi));
      s2[1 * 4 + b * 2 + e] = sb(mr(kC, lo), mr(kC, hi));
    }
  float s1[8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float lo = s2[a * 4 + b * 2 + 0], hi = s2[a * 4 + b * 2 + 1];
      s1[a * 4 + b * 2 + 0] = ad(mr(kC, lo), mr(kC, hi));
      s1[a * 4 + b * 2 + 1] = sb(mr(kC, lo), mr(kC, hi));
    }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float lo = s1[a * 4 + 0 * 2 + e], hi = s1[a * 4 + 1 * 2 + e];
      v[a * 4 + 0 * 2 + e] = ad(mr(kC, lo), mr(kC, hi));
      v[a * 4 + 1 * 2 + e] = sb(mr(kC, lo), mr(kC, hi));
    }
}


}  // namespace cwdm
