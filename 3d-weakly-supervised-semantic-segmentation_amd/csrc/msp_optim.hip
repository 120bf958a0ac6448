// The training step's optimizer (the reference's train.py:39, torch.optim.Adam(lr 1e-3)) in one launch over every
// parameter tensor (msp_adam_step, ABI 10).
//
// torch's fused multi-tensor Adam walks the headline UNet's 203 parameter tensors (30.1 M floats) in 12 launches of
// ~50 us per step: ~0.65 ms for 840 MB of algorithmic traffic (read param, grad, exp_avg, exp_avg_sq; write param,
// exp_avg, exp_avg_sq), ~1.3 TB/s.  Here one grid covers all tensors: block b takes a fixed 2048-float chunk of
// tensor i, found by one binary search over the chunks' prefix sums; float4 loads where the tensor allows.  The
// parameter, moment and size table is device memory built once (the tensors do not move); the gradient pointers,
// which a step's autograd allocates afresh, travel in the kernel arguments (<= 256 per launch: a captured graph
// keeps them).  The step count is a device scalar bumped by a one-thread kernel first, so captured steps replay.
//
// Per element, the arithmetic of torch's fused Adam (ADAM_MODE original, amsgrad off, fp32 opmath):
//   g += wd * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g;
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
#include "msp_conv_common.h"

namespace msp {

constexpr int kAdamThreads = 256;
constexpr int kAdamChunk = 2048;  // floats per block: 8 per thread

struct AdamGrads {
  const float* g[MSP_ADAM_MAX_TENSORS];
};

__global__ void adam_count_kernel(float* __restrict__ step) { step[0] += 1.f; }

// omb1 = 1 - beta1, omb2 = 1 - beta2 formed in double on the host (torch takes the betas as doubles: 1 - 0.999 in
// fp32 would be 1.3e-5 off)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1, float omb1, float b2,
                                          float omb2, float wd, float step_size, float bc2_sqrt, float eps) {
  if (wd != 0.f) g += p * wd;
  m = b1 * m + omb1 * g;
  v = b2 * v + omb2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p -= step_size * m / denom;
}

__global__ __launch_bounds__(kAdamThreads) void adam_step_kernel(const msp_adam_tensor* __restrict__ tab,
                                                                 const int64_t* __restrict__ chunk_start, int n,
                                                                 const AdamGrads grads,
                                                                 const float* __restrict__ step, double lr, double b1d,
                                                                 double b2d, float eps, float wd) {
  __shared__ int s_i;
  const int64_t b = blockIdx.x;
  if (threadIdx.x == 0) {
    int lo = 0, hi = n;  // chunk_start[lo] <= b < chunk_start[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (chunk_start[mid] <= b) lo = mid;
      else hi = mid;
    }
    s_i = lo;
  }
  __syncthreads();
  const int i = __builtin_amdgcn_readfirstlane(s_i);
  const float* gp = grads.g[i];
  if (gp == nullptr) return;  // a parameter without a gradient this step: untouched
  const msp_adam_tensor t = tab[i];
  const int64_t e0 = (b - chunk_start[i]) * kAdamChunk;
  const double sd = step[0];  // bias corrections once per block, in double
  const float step_size = (float)(lr / (1.0 - pow(b1d, sd))), bc2_sqrt = (float)sqrt(1.0 - pow(b2d, sd));
  const float b1 = (float)b1d, b2 = (float)b2d, omb1 = (float)(1.0 - b1d), omb2 = (float)(1.0 - b2d);
  const bool vec = (t.n & 3) == 0 && ((((uintptr_t)t.param) | ((uintptr_t)t.exp_avg) | ((uintptr_t)t.exp_avg_sq) |
                                        ((uintptr_t)gp)) & 15) == 0;
  if (vec) {
#pragma unroll
    for (int k = 0; k < kAdamChunk / (4 * kAdamThreads); ++k) {
      const int64_t e = e0 + 4 * (threadIdx.x + kAdamThreads * k);
      if (e >= t.n) break;
      floatx4 p = *reinterpret_cast<const floatx4*>(t.param + e);
      const floatx4 g = *reinterpret_cast<const floatx4*>(gp + e);
      floatx4 m = *reinterpret_cast<const floatx4*>(t.exp_avg + e);
      floatx4 v = *reinterpret_cast<const floatx4*>(t.exp_avg_sq + e);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adam_elem(pj, g[j], mj, vj, b1, omb1, b2, omb2, wd, step_size, bc2_sqrt, eps);
        p[j] = pj;
        m[j] = mj;
        v[j] = vj;
      }
      *reinterpret_cast<floatx4*>(t.param + e) = p;
      *reinterpret_cast<floatx4*>(t.exp_avg + e) = m;
      *reinterpret_cast<floatx4*>(t.exp_avg_sq + e) = v;
    }
  } else {
    for (int k = 0; k < kAdamChunk / kAdamThreads; ++k) {
      const int64_t e = e0 + threadIdx.x + kAdamThreads * k;
      if (e >= t.n) break;
      float p = t.param[e], m = t.exp_avg[e], v = t.exp_avg_sq[e];
      adam_elem(p, gp[e], m, v, b1, omb1, b2, omb2, wd, step_size, bc2_sqrt, eps);
      t.param[e] = p;
      t.exp_avg[e] = m;
      t.exp_avg_sq[e] = v;
    }
  }
}

}  // namespace msp

using namespace msp;

extern "C" {

int64_t msp_adam_chunks(int64_t n) { return n > 0 ? ceil_div(n, kAdamChunk) : 0; }

int msp_adam_step(const msp_adam_tensor* table, const int64_t* chunk_start, const float* const* grads, int n,
                  int64_t n_chunks, float* step, int bump, double lr, double beta1, double beta2, double eps,
                  double weight_decay, msp_stream_t stream) {
  MSP_REQUIRE(n >= 0 && n <= MSP_ADAM_MAX_TENSORS, "msp_adam_step: 0 <= n <= %d tensors per call (got %d)",
              MSP_ADAM_MAX_TENSORS, n);
  MSP_REQUIRE(n_chunks >= 0 && step && (n == 0 || (table && chunk_start && grads)), "msp_adam_step: NULL argument");
  hipStream_t s = as_stream(stream);
  if (bump) adam_count_kernel<<<1, 1, 0, s>>>(step);
  if (n > 0 && n_chunks > 0) {
    AdamGrads g{};
    for (int i = 0; i < n; ++i) g.g[i] = grads[i];
    adam_step_kernel<<<(unsigned)n_chunks, kAdamThreads, 0, s>>>(table, chunk_start, n, g, step, lr, beta1, beta2,
                                                                 (float)eps, (float)weight_decay);
  }
  return check_launch("msp_adam_step");
}

}  // extern "C"
