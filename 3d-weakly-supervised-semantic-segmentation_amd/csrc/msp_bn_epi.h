// BatchNormalization statistics from a convolution's epilogue (round 6; include/mi3dsparse.h msp_bn_epilogue,
// DESIGN.md §3.10).
//
// In the UNet's residual blocks every BatchNorm-ReLU sits next to a submanifold convolution
// (models/SparseConvNet.py:63-69: BN -> SubM -> BN -> SubM).  The convolution's epilogue holds each output row in
// registers once, so it can leave the BN's per-channel sums on the way out instead of the BN reading the rows
// again in a statistics pass:
//   forward  (x == nullptr): (sum v, sum v^2) of the convolution's own output rows v -- the input of the BN it
//            feeds (msp_bn_stats' sums, no extra read);
//   backward (x != nullptr): the convolution computes dy, the gradient of the BN output that fed it; with the BN's
//            input rows x and its stats, (sum dz, sum dz * xhat), dz = dy where z > 0 else leak * dy (msp_bn_bwd_stats'
//            sums, per element the same fp32 / fp64 arithmetic; one read of x instead of reading x and dy).
// Sums are fp64, per 128-row tile in a fixed order (lanes by a butterfly, waves in order), into a channel-major
// buffer partial[2][C][P] (P = tiles), which msp_bn_finalize_cm / msp_bn_bwd_apply_cm reduce in tile order:
// deterministic, and the reduction reads each channel's P partials contiguously.
#pragma once
#include "msp_conv_common.h"

namespace msp {

struct BnEpi {
  double* partial;     // nullptr: off
  const float* x;      // backward: the BN's input rows [V][C]; nullptr: forward sums of the output itself
  const float* stats;  // backward: the BN's stats[5][C]
  float leak;
  int C;               // channels of the BN (= the convolution's output channels)
  int64_t P;           // partial slots per (sum, channel): the convolution's 128-row tiles
};

inline BnEpi bn_epi_of(const msp_bn_epilogue* e, int c_out, int64_t n_rows) {
  BnEpi b{nullptr, nullptr, nullptr, 0.f, c_out, (n_rows + 127) / 128};
  if (e != nullptr) {
    b.partial = e->partial;
    b.x = e->x;
    b.stats = e->stats;
    b.leak = e->leak;
  }
  return b;
}

// Per-thread terms of channels c .. c + 3 of output row `row` (value v): s[k] and s[4 + k].
struct BnEpiAcc {
  double s[8];
  float mh[4], ml[4], is[4], sc[4], sh[4];
  __device__ void init(const BnEpi& e, int c) {
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = 0.0;
    if (e.x != nullptr) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mh[k] = e.stats[c + k];
        ml[k] = e.stats[e.C + c + k];
        is[k] = e.stats[2 * e.C + c + k];
        sc[k] = e.stats[3 * e.C + c + k];
        sh[k] = e.stats[4 * e.C + c + k];
      }
    }
  }
  __device__ void add(const BnEpi& e, int64_t row, int c, const floatx4& v) {
    add_x(e, v, e.x != nullptr ? *reinterpret_cast<const floatx4*>(e.x + row * e.C + c) : v);
  }
  // the same with the BN input quad xv already loaded (the kernels prefetch it during their last k-slice)
  __device__ void add_x(const BnEpi& e, const floatx4& v, const floatx4& xv) {
    if (e.x == nullptr) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[k] += v[k];
        s[4 + k] += (double)v[k] * v[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // bn_reduce4_kernel<1>'s term, element for element
        const float xc = (xv[k] - mh[k]) - ml[k];
        const float z = xc * sc[k] + sh[k];
        const float dz = z > 0.f ? v[k] : v[k] * e.leak;
        s[k] += dz;
        s[4 + k] += (double)dz * ((double)xc * is[k]);
      }
    }
  }
  // Sum over the lanes of the wave with the same lane % Q (Q a power of two <= 64), butterfly order.
  template <int Q>
  __device__ void wave_reduce() {
#pragma unroll
    for (int m = Q; m < 64; m <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += __shfl_xor(s[k], m, 64);
  }
};

// Slot p of channel c, sum j (0, 1) in the channel-major buffer.
__device__ __forceinline__ double* bn_epi_slot(const BnEpi& e, int j, int c, int64_t p) {
  return e.partial + ((int64_t)j * e.C + c) * e.P + p;
}

}  // namespace msp
