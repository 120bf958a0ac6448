// Point <-> voxel layers and the parameter-free pooling layers.
//
//   InputLayer(mode=4)  out[v] = mean of the points in voxel v; bwd divides by
//                       the count (Function_test.py:35-44)
//   OutputLayer         out[p] = in[voxel(p)]; bwd sums the points of a voxel
//                       (§8(a) a14)
//   UnPooling(s, s)     out[child] = in[parent]; bwd sums the children (a9)
//   MaxPooling(s, s)    out[parent] = max over children (Function_test.py:83-86)
//
// Every reduction walks a contiguous sorted run (points of a voxel after the
// key sort, children of a parent in Morton order), so no atomics are needed
// and results are bitwise reproducible.
#include "msp_common.h"

namespace msp {

constexpr int kT = 256;

inline unsigned grid_for(int64_t n) {
  int64_t g = (n + kT - 1) / kT;
  if (g > 65535 * 16) g = 65535 * 16;
  return (unsigned)(g < 1 ? 1 : g);
}

// thread per (row, channel) element of the OUTPUT
__global__ __launch_bounds__(kT) void input_avg_fwd_kernel(const float* __restrict__ f, int C,
                                                           const int32_t* __restrict__ perm,
                                                           const int32_t* __restrict__ vs, int64_t V,
                                                           float* __restrict__ out) {
  const int64_t n = V * C;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const int64_t v = e / C;
    const int c = (int)(e % C);
    const int32_t a = vs[v], b = vs[v + 1];
    float s = 0.f;
    for (int32_t j = a; j < b; ++j) s += f[(int64_t)perm[j] * C + c];
    out[e] = s / (float)(b - a);
  }
}

__global__ __launch_bounds__(kT) void input_avg_bwd_kernel(const float* __restrict__ d, int C,
                                                           const int32_t* __restrict__ p2v,
                                                           const int32_t* __restrict__ vs, int64_t np,
                                                           float* __restrict__ df) {
  const int64_t n = np * C;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const int64_t p = e / C;
    const int c = (int)(e % C);
    const int32_t v = p2v[p];
    df[e] = d[(int64_t)v * C + c] / (float)(vs[v + 1] - vs[v]);
  }
}

__global__ __launch_bounds__(kT) void gather_rows_kernel(const float* __restrict__ in, int C,
                                                         const int32_t* __restrict__ idx, int64_t n,
                                                         float* __restrict__ out) {
  const int64_t total = n * C;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const int64_t r = e / C;
    const int c = (int)(e % C);
    out[e] = in[(int64_t)idx[r] * C + c];
  }
}

__global__ __launch_bounds__(kT) void gather_rows4_kernel(const float4* __restrict__ in, int C4,
                                                          const int32_t* __restrict__ idx, int64_t n,
                                                          float4* __restrict__ out) {
  const int64_t total = n * C4;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const int64_t r = e / C4;
    const int c = (int)(e % C4);
    out[e] = in[(int64_t)idx[r] * C4 + c];
  }
}

// out[g] = sum over rows j in [start[g], start[g+1]) of in[perm ? perm[j] : j]
__global__ __launch_bounds__(kT) void segsum_kernel(const float* __restrict__ in, int C,
                                                    const int32_t* __restrict__ perm,
                                                    const int32_t* __restrict__ start, int64_t G,
                                                    float* __restrict__ out) {
  const int64_t n = G * C;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const int64_t g = e / C;
    const int c = (int)(e % C);
    float s = 0.f;
    for (int32_t j = start[g]; j < start[g + 1]; ++j) s += in[(int64_t)(perm ? perm[j] : j) * C + c];
    out[e] = s;
  }
}

__global__ __launch_bounds__(kT) void maxpool_fwd_kernel(const float* __restrict__ in, int C,
                                                         const int32_t* __restrict__ start, int64_t G,
                                                         float* __restrict__ out, int32_t* __restrict__ arg) {
  const int64_t n = G * C;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const int64_t g = e / C;
    const int c = (int)(e % C);
    const int32_t a = start[g], b = start[g + 1];
    float m = in[(int64_t)a * C + c];
    int32_t am = a;
    for (int32_t j = a + 1; j < b; ++j) {
      const float v = in[(int64_t)j * C + c];
      if (v > m) {
        m = v;
        am = j;
      }
    }
    out[e] = m;
    arg[e] = am;
  }
}

__global__ __launch_bounds__(kT) void maxpool_bwd_kernel(const float* __restrict__ d, int C,
                                                         const int32_t* __restrict__ arg, int64_t G,
                                                         float* __restrict__ din) {
  const int64_t n = G * C;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const int c = (int)(e % C);
    din[(int64_t)arg[e] * C + c] = d[e];  // children are disjoint across parents
  }
}

int gather_rows(const float* in, int C, const int32_t* idx, int64_t n, float* out, hipStream_t s) {
  if (n == 0) return MSP_OK;
  if ((C & 3) == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    gather_rows4_kernel<<<grid_for(n * (C / 4)), kT, 0, s>>>(reinterpret_cast<const float4*>(in), C / 4, idx, n,
                                                             reinterpret_cast<float4*>(out));
  } else {
    gather_rows_kernel<<<grid_for(n * C), kT, 0, s>>>(in, C, idx, n, out);
  }
  return check_launch("gather_rows");
}

}  // namespace msp

using namespace msp;

extern "C" {

int msp_input_avg_fwd(const float* feats, int C, const int32_t* perm, const int32_t* vstart, int64_t V,
                      float* out, msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_input_avg_fwd: bad C");
  if (V == 0) return MSP_OK;
  input_avg_fwd_kernel<<<grid_for(V * C), kT, 0, as_stream(stream)>>>(feats, C, perm, vstart, V, out);
  return check_launch("msp_input_avg_fwd");
}

int msp_input_avg_bwd(const float* dout, int C, const int32_t* p2v, const int32_t* vstart, int64_t n_points,
                      float* dfeats, msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_input_avg_bwd: bad C");
  if (n_points == 0) return MSP_OK;
  input_avg_bwd_kernel<<<grid_for(n_points * C), kT, 0, as_stream(stream)>>>(dout, C, p2v, vstart, n_points,
                                                                             dfeats);
  return check_launch("msp_input_avg_bwd");
}

int msp_output_fwd(const float* in, int C, const int32_t* p2v, int64_t n_points, float* out, msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_output_fwd: bad C");
  return gather_rows(in, C, p2v, n_points, out, as_stream(stream));
}

int msp_output_bwd(const float* dout, int C, const int32_t* perm, const int32_t* vstart, int64_t V, float* din,
                   msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_output_bwd: bad C");
  if (V == 0) return MSP_OK;
  segsum_kernel<<<grid_for(V * C), kT, 0, as_stream(stream)>>>(dout, C, perm, vstart, V, din);
  return check_launch("msp_output_bwd");
}

int msp_unpool_fwd(const float* in, int C, const int32_t* parent_of, int64_t n_fine, float* out,
                   msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_unpool_fwd: bad C");
  return gather_rows(in, C, parent_of, n_fine, out, as_stream(stream));
}

int msp_unpool_bwd(const float* dout, int C, const int32_t* child_start, int64_t n_coarse, float* din,
                   msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_unpool_bwd: bad C");
  if (n_coarse == 0) return MSP_OK;
  segsum_kernel<<<grid_for(n_coarse * C), kT, 0, as_stream(stream)>>>(dout, C, nullptr, child_start, n_coarse,
                                                                      din);
  return check_launch("msp_unpool_bwd");
}

int msp_maxpool_fwd(const float* in, int C, const int32_t* child_start, int64_t n_coarse, float* out,
                    int32_t* argmax, msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_maxpool_fwd: bad C");
  if (n_coarse == 0) return MSP_OK;
  maxpool_fwd_kernel<<<grid_for(n_coarse * C), kT, 0, as_stream(stream)>>>(in, C, child_start, n_coarse, out,
                                                                           argmax);
  return check_launch("msp_maxpool_fwd");
}

int msp_maxpool_bwd(const float* dout, int C, const int32_t* argmax, int64_t n_coarse, float* din,
                    msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_maxpool_bwd: bad C");
  if (n_coarse == 0) return MSP_OK;
  maxpool_bwd_kernel<<<grid_for(n_coarse * C), kT, 0, as_stream(stream)>>>(dout, C, argmax, n_coarse, din);
  return check_launch("msp_maxpool_bwd");
}

}  // extern "C"
