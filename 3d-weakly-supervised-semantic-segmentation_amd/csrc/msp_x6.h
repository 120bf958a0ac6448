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

}  // namespace msp
