// Split-bf16 ("x6") helpers shared by the MFMA convolution kernels
// (msp_conv_x6.hip, msp_local.hip): exact three-piece bf16 splits of fp32
// operands and the 16x16x32 bf16 MFMA on packed pieces.
#pragma once
#include "msp_conv_common.h"

namespace msp {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// (a, b) -> packed RNE bf16 pair (v_cvt_pk_bf16_f32), a in the low half
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const floatx2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

__device__ __forceinline__ floatx4 mfma_bf16(const u32x4& a, const u32x4& b, const floatx4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                 0, 0, 0);
}

// 8 consecutive fp32 values -> three bf16x8 pieces, v = p[0] + p[1] + p[2]
__device__ __forceinline__ void split8(const floatx4& a, const floatx4& b, u32x4 (&p)[3]) {
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int s = 0; s < 3; ++s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t h = pk_bf16(v[2 * i], v[2 * i + 1]);
      p[s][i] = h;
      if (s < 2) {
        v[2 * i] -= __uint_as_float(h << 16);
        v[2 * i + 1] -= __uint_as_float(h & 0xffff0000u);
      }
    }
  }
}

// One work item of the per-step weight image (split_weights_kernel, msp_conv_x6.hip): unit g of the image of
// (K, c_out, c_in) weights with NC columns per slice and KS-deep k-slices, zero padded past c_in.  wlay 1: wt is
// [K][c_in][c_out] (the module's layout), else [K][c_out][c_in].
__device__ __forceinline__ void split_weights_unit(const float* __restrict__ wt, int K, int c_out, int c_in, int NC,
                                                   int KS, u32x4* __restrict__ img, int wlay, int64_t g) {
  const int K8 = KS / 8, WU = 3 * K8 * NC;
  const int n_y = c_out / NC, nks = (c_in + KS - 1) / KS;
  if (g >= (int64_t)K * n_y * nks * WU) return;
  const int u = (int)(g % WU);
  const int64_t rest = g / WU;
  const int ks = (int)(rest % nks);
  const int64_t r2 = rest / nks;
  const int cy = (int)(r2 % n_y);
  const int64_t o = r2 / n_y;
  const int p = u / (K8 * NC), rem = u % (K8 * NC), k8 = rem / NC, n = rem % NC;
  const int k = ks * KS + 8 * k8;
  u32x4 pc[3] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
  if (k < c_in) {  // c_in % 16 == 0: a unit is all data or all padding
    if (wlay) {
      const float* src = wt + (o * c_in + k) * c_out + cy * NC + n;
      split8(floatx4{src[0], src[c_out], src[2 * c_out], src[3 * c_out]},
             floatx4{src[4 * c_out], src[5 * c_out], src[6 * c_out], src[7 * c_out]}, pc);
    } else {
      const floatx4* src = reinterpret_cast<const floatx4*>(wt + ((o * c_out) + cy * NC + n) * c_in + k);
      split8(src[0], src[1], pc);
    }
  }
  img[g] = p == 0 ? pc[0] : (p == 1 ? pc[1] : pc[2]);
}

// One work item (thread) of the lane-ordered weight image of conv_x6s (split_weights_lane_kernel, msp_local.hip):
// lane g & 63 of fragment row g >> 6 = (((o * n_y + cy) * nks + ks) * NT + t), its three pieces 64 units apart.
__device__ __forceinline__ void split_weights_lane_unit(const float* __restrict__ wt, int K, int c_out, int c_in,
                                                        int NT, u32x4* __restrict__ img, int wlay, int64_t g) {
  const int n_y = c_out / (16 * NT), nks = (c_in + 31) / 32;
  if (g >= (int64_t)K * n_y * nks * NT * 64) return;
  const int lane = (int)(g & 63), r = lane & 15, q = lane >> 4;
  int64_t rest = g >> 6;
  const int t = (int)(rest % NT);
  rest /= NT;
  const int ks = (int)(rest % nks);
  rest /= nks;
  const int cy = (int)(rest % n_y);
  const int64_t o = rest / n_y;
  const int oc = 16 * (cy * NT + t) + r, k = 32 * ks + 8 * q;
  floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  if (k < c_in) {  // c_in % 16 == 0: an octet is all data or all padding
    if (wlay) {
      const float* src = wt + (o * c_in + k) * c_out + oc;
      a = floatx4{src[0], src[c_out], src[2 * c_out], src[3 * c_out]};
      b = floatx4{src[4 * c_out], src[5 * c_out], src[6 * c_out], src[7 * c_out]};
    } else {
      const floatx4* src = reinterpret_cast<const floatx4*>(wt + (o * c_out + oc) * c_in + k);
      a = src[0];
      b = src[1];
    }
  }
  u32x4* dst = img + ((g >> 6) * 3) * 64 + lane;
  u32x4 pc[3];
  split8(a, b, pc);
#pragma unroll
  for (int p = 0; p < 3; ++p) dst[p * 64] = pc[p];
}

}  // namespace msp
