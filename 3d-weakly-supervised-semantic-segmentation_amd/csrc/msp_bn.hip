// Batch normalisation + (leaky) ReLU over the active sites of a sparse tensor.
//
// Semantics follow SCN's BatchNormalization with leakiness (SURVEY.md §8(a)
// a10; scn.BatchNormReLU / BatchNormLeakyReLU at models/SparseConvNet.py:69,
// 86,103,116,...): train mode normalises with the batch mean and BIASED
// variance over the V rows, eps inside the sqrt, and updates
//   running_mean = momentum*running_mean + (1-momentum)*mean
//   running_var  = momentum*running_var  + (1-momentum)*var*V/(V-1)
// eval mode uses the running statistics.  y = max(z, 0) + leak*min(z, 0) with
// z = ((x - mean_hi) - mean_lo)*scale + shift, scale = invstd*weight,
// shift = bias.  The fp64 mean is carried as an fp32 hi/lo pair and
// subtracted before scaling: folding it into the shift (or rounding it to
// fp32) moves z by ulp(mean)*invstd, which for low-variance channels far from
// zero is many ulps of z and flips ReLU decisions.
//
// Per-channel statistics live in one float array stats[5][C]:
//   [0] mean_hi  [1] mean_lo  [2] invstd  [3] scale  [4] shift
//
// Reductions accumulate in fp64 per block and are combined in block order,
// so results are deterministic and the 65 stacked BN layers of the headline
// UNet do not drift from an fp64 reference.
#include "msp_common.h"

namespace msp {

constexpr int kT = 256;
#ifndef MSP_BN_MAX_PARTS
#define MSP_BN_MAX_PARTS 1024
#endif
constexpr int64_t kMaxParts = MSP_BN_MAX_PARTS;
#ifndef MSP_BN_UNROLL  // bn_reduce4's rows in flight per thread (experiments: 8)
#define MSP_BN_UNROLL 4
#endif

// Partial-sum blocks: two 4-deep passes of the vector form per block (R = 1024 / C rows per pass, so
// 8 R rows per block, 16..256), at most kMaxParts.  Sized by C so the small levels (C up to 448, a few
// hundred to a few thousand rows) get enough blocks: 256 rows per block there meant 16-64 serial passes
// per thread (20-26 us per reduction, profiles/r01/kernel_stats_r01final2_bench_steps3.csv).
__host__ __device__ inline int64_t bn_parts(int64_t V, int C) {
  int64_t rpb = (C > 0 && C <= 1024) ? 8 * (1024 / C) : 256;
  rpb = rpb > 256 ? 256 : (rpb < 16 ? 16 : rpb);
  const int64_t p = (V + rpb - 1) / rpb;
  return p < 1 ? 1 : (p > kMaxParts ? kMaxParts : p);
}

struct BnStats {
  const float *mh, *ml, *is, *sc, *sh;
  __host__ __device__ BnStats(const float* st, int C)
      : mh(st), ml(st + C), is(st + 2 * C), sc(st + 3 * C), sh(st + 4 * C) {}
  __device__ float centred(float x, int c) const { return (x - mh[c]) - ml[c]; }
  __device__ float z(float x, int c) const { return centred(x, c) * sc[c] + sh[c]; }
};

// MODE 0: (sum x, sum x^2).  MODE 1: (sum dz, sum dz*xhat).
// Vector form (C % 4 == 0, C <= 1024): each thread owns 4 channels (one
// float4 column) and strides over rows with 4 independent loads in flight;
// R = 256 / (C/4) rows are covered per pass and folded in LDS in fixed order.
// MODE 2: residual join fused with the statistics of its output: x = a,
// dy = b, sum = a + b is written to sum_out and reduced as in MODE 0 (same
// partition and order as msp_bn_stats on the sum: identical partials).
// MODE 3: channel join (SCN JoinTable) fused with the statistics of its
// output: x = a [V][ca], dy = b [V][C - ca], the row [a | b] is written to
// sum_out [V][C] and reduced as in MODE 0 (identical partials again).
template <int MODE>
__global__ __launch_bounds__(kT) void bn_reduce4_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        int64_t V, int C, const float* __restrict__ stats,
                                                        float leak, double* __restrict__ partial,
                                                        float* __restrict__ sum_out = nullptr, int ca = 0) {
  __shared__ double red[kT][8];
  const int64_t P = gridDim.x;
  const int64_t per = (V + P - 1) / P;
  const int64_t v0 = blockIdx.x * per, v1 = min(V, v0 + per);
  const int C4 = C >> 2;
  const int R = kT / C4;
  const int t = threadIdx.x, c4 = t % C4, ro = t / C4;
  const BnStats st(stats, C);
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};
  float mh[4], ml[4], is[4], sc[4], sh[4];
  if (MODE == 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * c4 + k;
      mh[k] = st.mh[c];
      ml[k] = st.ml[c];
      is[k] = st.is[c];
      sc[k] = st.sc[c];
      sh[k] = st.sh[c];
    }
  }
  auto term = [&](const float4& xv4, const float4& g4) {
    const float xs[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
    const float gs[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (MODE != 1) {
        s0[k] += xs[k];
        s1[k] += (double)xs[k] * xs[k];
      } else {
        const float xc = (xs[k] - mh[k]) - ml[k];
        const float z = xc * sc[k] + sh[k];
        const float dz = z > 0.f ? gs[k] : gs[k] * leak;
        s0[k] += dz;
        s1[k] += (double)dz * ((double)xc * is[k]);
      }
    }
  };
  if (ro < R) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* g4 = reinterpret_cast<const float4*>(dy);
    float4* s4 = reinterpret_cast<float4*>(sum_out);
    auto join = [&](int64_t e, const float4& a, const float4& b) {  // MODE 2: the residual sum
      const float4 sm = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
      s4[e] = sm;
      return sm;
    };
    // MODE 3: the column's source (a or b) is fixed per thread
    const int ca4 = ca >> 2, cb4 = C4 - ca4;
    const bool from_a = c4 < ca4;
    const float4* src4 = from_a ? x4 : g4;
    const int sc4 = from_a ? ca4 : cb4, soff = from_a ? c4 : c4 - ca4;
    auto cat = [&](int64_t v) {
      const float4 e = src4[v * sc4 + soff];
      s4[v * C4 + c4] = e;
      return e;
    };
    int64_t v = v0 + ro;
    constexpr int U = MSP_BN_UNROLL;  // rows in flight per thread and tensor
    if (MODE == 3) {
      for (; v + (U - 1) * R < v1; v += U * R) {
        float4 e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = src4[(v + u * R) * sc4 + soff];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          s4[(v + u * R) * C4 + c4] = e[u];
          term(e[u], e[u]);
        }
      }
      for (; v < v1; v += R) {
        const float4 e = cat(v);
        term(e, e);
      }
    }
    if (MODE != 3) {
    for (; v + (U - 1) * R < v1; v += U * R) {
      float4 xa[U], ga[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xa[u] = x4[(v + u * R) * C4 + c4];
        if (MODE != 0) ga[u] = g4[(v + u * R) * C4 + c4];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (MODE == 2) {
          const float4 sm = join((v + u * R) * C4 + c4, xa[u], ga[u]);
          term(sm, sm);
        } else {
          term(xa[u], MODE == 1 ? ga[u] : xa[u]);
        }
      }
    }
    for (; v < v1; v += R) {
      if (MODE == 2) {
        const float4 sm = join(v * C4 + c4, x4[v * C4 + c4], g4[v * C4 + c4]);
        term(sm, sm);
      } else {
        term(x4[v * C4 + c4], MODE == 1 ? g4[v * C4 + c4] : x4[v * C4 + c4]);
      }
    }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[t][k] = s0[k];
    red[t][4 + k] = s1[k];
  }
  __syncthreads();
  if (t < C4) {
    double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += red[k * C4 + t][j];
        b[j] += red[k * C4 + t][4 + j];
      }
    double* out0 = partial + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      out0[4 * t + j] = a[j];
      out0[C + 4 * t + j] = b[j];
    }
  }
}

// MODE 0: (sum x, sum x^2).  MODE 1: (sum dz, sum dz*xhat).
template <int MODE>
__global__ __launch_bounds__(kT) void bn_reduce_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                       int64_t V, int C, const float* __restrict__ stats,
                                                       float leak, double* __restrict__ partial) {
  const int64_t P = gridDim.x;
  const int64_t per = (V + P - 1) / P;
  const int64_t v0 = blockIdx.x * per, v1 = min(V, v0 + per);
  const int t = threadIdx.x;
  double* out0 = partial + (int64_t)blockIdx.x * 2 * C;
  double* out1 = out0 + C;
  const BnStats st(stats, C);
  auto term = [&](int64_t v, int c, double& s0, double& s1) {
    const float xv = x[v * C + c];
    if (MODE == 0) {
      s0 += xv;
      s1 += (double)xv * xv;
    } else {
      const float g = dy[v * C + c];
      const float dz = st.z(xv, c) > 0.f ? g : g * leak;
      s0 += dz;
      s1 += (double)dz * ((double)st.centred(xv, c) * st.is[c]);
    }
  };
  if (C <= kT) {
    __shared__ double red0[kT], red1[kT];
    const int R = kT / C;
    const int ro = t / C, c = t % C;
    double s0 = 0.0, s1 = 0.0;
    if (ro < R)
      for (int64_t v = v0 + ro; v < v1; v += R) term(v, c, s0, s1);
    red0[t] = s0;
    red1[t] = s1;
    __syncthreads();
    if (t < C) {
      double a = 0.0, b = 0.0;
      for (int k = 0; k < R; ++k) {
        a += red0[k * C + t];
        b += red1[k * C + t];
      }
      out0[t] = a;
      out1[t] = b;
    }
  } else {
    for (int c = t; c < C; c += kT) {
      double s0 = 0.0, s1 = 0.0;
      for (int64_t v = v0; v < v1; ++v) term(v, c, s0, s1);
      out0[c] = s0;
      out1[c] = s1;
    }
  }
}

// Sum of partial[p][slot][c] over p for one channel per block, fixed order
// (strided per thread, then a tree over the block): deterministic.
__device__ inline void sum_partials(const double* __restrict__ partial, int64_t P, int C, int c, double* out2) {
  __shared__ double red[2][kT];
  double a = 0.0, b = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += kT) {
    a += partial[p * 2 * C + c];
    b += partial[p * 2 * C + C + c];
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int w = kT / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  out2[0] = red[0][0];
  out2[1] = red[1][0];
}

// The same over a channel-major buffer partial[2][C][P] (msp_bn_epilogue): a channel's P slots are contiguous,
// so the block's loads are coalesced however many tiles wrote them.
__device__ inline void sum_partials_cm(const double* __restrict__ partial, int64_t P, int C, int c, double* out2) {
  __shared__ double red[2][kT];
  double a = 0.0, b = 0.0;
  const double* p0 = partial + (int64_t)c * P;
  const double* p1 = partial + ((int64_t)C + c) * P;
  for (int64_t p = threadIdx.x; p < P; p += kT) {
    a += p0[p];
    b += p1[p];
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int w = kT / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  out2[0] = red[0][0];
  out2[1] = red[1][0];
}

// one block per channel
__global__ __launch_bounds__(kT) void bn_finalize_kernel(const double* __restrict__ partial, int64_t P, int C,
                                                         int64_t V, double eps, double momentum, int train,
                                                         float* __restrict__ rmean, float* __restrict__ rvar,
                                                         const float* __restrict__ weight,
                                                         const float* __restrict__ bias, float* __restrict__ stats) {
  const int c = blockIdx.x;
  double sums[2] = {0.0, 0.0};
  if (train) sum_partials(partial, P, C, c, sums);
  if (threadIdx.x != 0) return;
  double mu, var;
  if (train) {
    mu = V > 0 ? sums[0] / (double)V : 0.0;
    var = V > 0 ? sums[1] / (double)V - mu * mu : 0.0;
    if (var < 0.0) var = 0.0;
    const double unb = V > 1 ? var * (double)V / (double)(V - 1) : var;
    rmean[c] = (float)(momentum * rmean[c] + (1.0 - momentum) * mu);
    rvar[c] = (float)(momentum * rvar[c] + (1.0 - momentum) * unb);
  } else {
    mu = rmean[c];
    var = rvar[c];
  }
  const double is = 1.0 / sqrt(var + eps);
  const double w = weight ? weight[c] : 1.0, b = bias ? bias[c] : 0.0;
  const float hi = (float)mu;
  stats[c] = hi;
  stats[C + c] = (float)(mu - (double)hi);
  stats[2 * C + c] = (float)is;
  stats[3 * C + c] = (float)(w * is);
  stats[4 * C + c] = (float)b;
}

__global__ __launch_bounds__(kT) void bn_apply_kernel(const float* __restrict__ x, int64_t n, int C,
                                                      const float* __restrict__ stats, float leak,
                                                      float* __restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  const BnStats st(stats, C);
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) {
    const float z = st.z(x[i], (int)(i % C));
    y[i] = z > 0.f ? z : z * leak;
  }
}

// Vector form (C % 4 == 0, C <= 1024): thread t owns the float4 column
// t % (C/4) for all its rows, so the per-channel constants sit in registers
// and the loop has no index division; rows advance by gridDim * R.
__global__ __launch_bounds__(kT) void bn_apply4_kernel(const float* __restrict__ x, int64_t V, int C,
                                                       const float* __restrict__ stats, float leak,
                                                       float* __restrict__ y) {
  const int C4 = C >> 2, R = kT / C4;
  const int t = threadIdx.x, c4 = t % C4, ro = t / C4;
  if (ro >= R) return;
  const BnStats st(stats, C);
  float mh[4], ml[4], sc[4], sh[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * c4 + k;
    mh[k] = st.mh[c];
    ml[k] = st.ml[c];
    sc[k] = st.sc[c];
    sh[k] = st.sh[c];
  }
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* y4 = reinterpret_cast<float4*>(y);
  const int64_t step = (int64_t)gridDim.x * R;
  auto f = [&](float v, int k) {
    const float z = ((v - mh[k]) - ml[k]) * sc[k] + sh[k];
    return z > 0.f ? z : z * leak;
  };
  for (int64_t v = (int64_t)blockIdx.x * R + ro; v < V; v += step) {
    const float4 a = x4[v * C4 + c4];
    y4[v * C4 + c4] = make_float4(f(a.x, 0), f(a.y, 1), f(a.z, 2), f(a.w, 3));
  }
}

// one block per channel, channel-major partials (msp_bn_finalize_cm)
__global__ __launch_bounds__(kT) void bn_finalize_cm_kernel(const double* __restrict__ partial, int64_t P, int C,
                                                            int64_t V, double eps, double momentum, int train,
                                                            float* __restrict__ rmean, float* __restrict__ rvar,
                                                            const float* __restrict__ weight,
                                                            const float* __restrict__ bias, float* __restrict__ stats) {
  const int c = blockIdx.x;
  double sums[2] = {0.0, 0.0};
  if (train) sum_partials_cm(partial, P, C, c, sums);
  if (threadIdx.x != 0) return;
  double mu, var;
  if (train) {
    mu = V > 0 ? sums[0] / (double)V : 0.0;
    var = V > 0 ? sums[1] / (double)V - mu * mu : 0.0;
    if (var < 0.0) var = 0.0;
    const double unb = V > 1 ? var * (double)V / (double)(V - 1) : var;
    rmean[c] = (float)(momentum * rmean[c] + (1.0 - momentum) * mu);
    rvar[c] = (float)(momentum * rvar[c] + (1.0 - momentum) * unb);
  } else {
    mu = rmean[c];
    var = rvar[c];
  }
  const double is = 1.0 / sqrt(var + eps);
  const double w = weight ? weight[c] : 1.0, b = bias ? bias[c] : 0.0;
  const float hi = (float)mu;
  stats[c] = hi;
  stats[C + c] = (float)(mu - (double)hi);
  stats[2 * C + c] = (float)is;
  stats[3 * C + c] = (float)(w * is);
  stats[4 * C + c] = (float)b;
}

// one block per channel, channel-major partials (msp_bn_bwd_apply_cm)
__global__ __launch_bounds__(kT) void bn_bwd_finalize_cm_kernel(const double* __restrict__ partial, int64_t P, int C,
                                                                float* __restrict__ dweight,
                                                                float* __restrict__ dbias, double* __restrict__ sums) {
  const int c = blockIdx.x;
  double s2[2];
  sum_partials_cm(partial, P, C, c, s2);
  if (threadIdx.x != 0) return;
  sums[c] = s2[0];
  sums[C + c] = s2[1];
  if (dbias) dbias[c] = (float)s2[0];
  if (dweight) dweight[c] = (float)s2[1];
}

// one block per channel
__global__ __launch_bounds__(kT) void bn_bwd_finalize_kernel(const double* __restrict__ partial, int64_t P, int C,
                                                             float* __restrict__ dweight,
                                                             float* __restrict__ dbias, double* __restrict__ sums) {
  const int c = blockIdx.x;
  double s2[2];
  sum_partials(partial, P, C, c, s2);
  if (threadIdx.x != 0) return;
  sums[c] = s2[0];      // sum dz
  sums[C + c] = s2[1];  // sum dz * xhat
  if (dbias) dbias[c] = (float)s2[0];
  if (dweight) dweight[c] = (float)s2[1];
}

// SPLIT (msp_bn_bwd_apply_split, round 6): dx's columns [0, ca) go to dx as [V][ca] and [ca, C) to dxb as
// [V][C - ca] -- the two gradients of a JoinTable that produced x, written here instead of by a split pass.
template <bool SPLIT = false>
__global__ __launch_bounds__(kT) void bn_bwd_apply_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ dy, int64_t n, int C,
                                                          int64_t V, const double* __restrict__ sums,
                                                          const float* __restrict__ stats,
                                                          const float* __restrict__ weight, float leak, int train,
                                                          const float* __restrict__ addend, float* __restrict__ dx,
                                                          int ca = 0, float* __restrict__ dxb = nullptr) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  const double invV = V > 0 ? 1.0 / (double)V : 0.0;
  const BnStats st(stats, C);
  auto store = [&](int64_t i, int c, float d) {
    if constexpr (SPLIT) {
      const int64_t v = i / C;
      if (c < ca) dx[v * ca + c] = d;
      else dxb[v * (C - ca) + (c - ca)] = d;
    } else {
      dx[i] = d;
    }
  };
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % C);
    const float xv = x[i], g = dy[i];
    const float dz = st.z(xv, c) > 0.f ? g : g * leak;
    const float w = weight ? weight[c] : 1.f;
    if (train) {
      const float xh = st.centred(xv, c) * st.is[c];
      const float mdz = (float)(sums[c] * invV), mdzx = (float)(sums[C + c] * invV);
      const float d = w * st.is[c] * (dz - mdz - xh * mdzx);
      store(i, c, addend ? d + addend[i] : d);
    } else {
      const float d = w * st.is[c] * dz;
      store(i, c, addend ? d + addend[i] : d);
    }
  }
}

// Vector form of the above (same column ownership as bn_apply4_kernel).  SPLIT: quad stores when ca % 4 == 0, else
// element stores (a quad may straddle the split); the arithmetic is the same either way.
template <bool SPLIT = false>
__global__ __launch_bounds__(kT) void bn_bwd_apply4_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ dy, int64_t V, int C,
                                                           const double* __restrict__ sums,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ weight, float leak, int train,
                                                           const float* __restrict__ addend, float* __restrict__ dx,
                                                           int ca = 0, float* __restrict__ dxb = nullptr) {
  const int C4 = C >> 2, R = kT / C4;
  const int t = threadIdx.x, c4 = t % C4, ro = t / C4;
  if (ro >= R) return;
  const double invV = V > 0 ? 1.0 / (double)V : 0.0;
  const BnStats st(stats, C);
  float mh[4], ml[4], is[4], sc[4], sh[4], ws[4], mdz[4], mdzx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * c4 + k;
    mh[k] = st.mh[c];
    ml[k] = st.ml[c];
    is[k] = st.is[c];
    sc[k] = st.sc[c];
    sh[k] = st.sh[c];
    ws[k] = (weight ? weight[c] : 1.f) * is[k];
    mdz[k] = train ? (float)(sums[c] * invV) : 0.f;
    mdzx[k] = train ? (float)(sums[C + c] * invV) : 0.f;
  }
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const float4* g4 = reinterpret_cast<const float4*>(dy);
  // the thread's column quad is fixed: SPLIT writes it to the first or the second output, row stride C4o
  const int ca4 = ca >> 2;
  const bool quad = !SPLIT || (ca & 3) == 0;  // block-uniform
  const bool to_b = SPLIT && c4 >= ca4;
  float4* d4 = reinterpret_cast<float4*>(to_b ? dxb : dx);
  const int C4o = SPLIT ? (to_b ? C4 - ca4 : ca4) : C4, c4o = to_b ? c4 - ca4 : c4;
  const int64_t step = (int64_t)gridDim.x * R;
  auto f = [&](float xv, float g, int k) {
    const float xc = (xv - mh[k]) - ml[k];
    const float dz = xc * sc[k] + sh[k] > 0.f ? g : g * leak;
    if (!train) return ws[k] * dz;
    return ws[k] * (dz - mdz[k] - (xc * is[k]) * mdzx[k]);
  };
  for (int64_t v = (int64_t)blockIdx.x * R + ro; v < V; v += step) {
    const float4 a = x4[v * C4 + c4], g = g4[v * C4 + c4];
    float4 d = make_float4(f(a.x, g.x, 0), f(a.y, g.y, 1), f(a.z, g.z, 2), f(a.w, g.w, 3));
    if (addend) {  // uniform: the other consumer's gradient of x (residual fork), one add as autograd's
      const float4 e = reinterpret_cast<const float4*>(addend)[v * C4 + c4];
      d = make_float4(d.x + e.x, d.y + e.y, d.z + e.z, d.w + e.w);
    }
    if (quad) {
      d4[v * C4o + c4o] = d;
    } else {  // SPLIT with ca % 4 != 0
      const float e[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * c4 + k;
        if (c < ca) dx[v * ca + c] = e[k];
        else dxb[v * (C - ca) + (c - ca)] = e[k];
      }
    }
  }
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// blocks for the column-owning vector kernels: R = 256 / (C/4) rows per block pass
inline unsigned rows_grid(int64_t V, int C) {
  const int64_t R = kT / (C / 4);
  int64_t g = (V + R - 1) / R;
  if (g > 4096) g = 4096;
  return (unsigned)(g < 1 ? 1 : g);
}

// [a | b] rows (JoinTable) and the inverse split of a gradient (its backward), element per thread
__global__ __launch_bounds__(kT) void join_cols_kernel(const float* __restrict__ a, int ca,
                                                       const float* __restrict__ b, int cb, int64_t V,
                                                       float* __restrict__ out) {
  const int C = ca + cb;
  const int64_t n = V * C, stride = (int64_t)gridDim.x * kT;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) {
    const int64_t v = i / C;
    const int c = (int)(i - v * C);
    out[i] = c < ca ? a[v * ca + c] : b[v * cb + (c - ca)];
  }
}

__global__ __launch_bounds__(kT) void split_cols_kernel(const float* __restrict__ in, int64_t V, int ca, int cb,
                                                        float* __restrict__ a, float* __restrict__ b) {
  const int C = ca + cb;
  const int64_t n = V * C, stride = (int64_t)gridDim.x * kT;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) {
    const int64_t v = i / C;
    const int c = (int)(i - v * C);
    if (c < ca) {
      if (a) a[v * ca + c] = in[i];
    } else if (b) {
      b[v * cb + (c - ca)] = in[i];
    }
  }
}

__global__ __launch_bounds__(kT) void split_cols4_kernel(const float4* __restrict__ in, int64_t V, int ca4, int cb4,
                                                         float4* __restrict__ a, float4* __restrict__ b) {
  const int C4 = ca4 + cb4;
  const int64_t n = V * C4, stride = (int64_t)gridDim.x * kT;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) {
    const int64_t v = i / C4;
    const int c = (int)(i - v * C4);
    if (c < ca4) {
      if (a) a[v * ca4 + c] = in[i];
    } else if (b) {
      b[v * cb4 + (c - ca4)] = in[i];
    }
  }
}

__global__ __launch_bounds__(kT) void add_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                                 float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) out[i] = a[i] + b[i];
}

inline unsigned ew_grid(int64_t n) {
  int64_t g = (n + kT - 1) / kT;
  if (g > 4096) g = 4096;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace msp

using namespace msp;

extern "C" {

int64_t msp_bn_partials(int64_t V, int C) {
  (void)C;
  return bn_parts(V, C);
}

int msp_bn_stats(const float* x, int64_t V, int C, double* partial, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && C <= 4096 && V >= 0, "msp_bn_stats: bad shape");
  if (C % 4 == 0 && C <= 4 * kT && aligned16(x))
    bn_reduce4_kernel<0><<<(unsigned)bn_parts(V, C), kT, 0, as_stream(stream)>>>(x, nullptr, V, C, nullptr, 0.f,
                                                                              partial);
  else
    bn_reduce_kernel<0><<<(unsigned)bn_parts(V, C), kT, 0, as_stream(stream)>>>(x, nullptr, V, C, nullptr, 0.f,
                                                                             partial);
  return check_launch("msp_bn_stats");
}

int msp_bn_finalize(const double* partial, int64_t V, int C, double eps, double momentum, int train,
                    float* running_mean, float* running_var, const float* weight, const float* bias, float* stats,
                    msp_stream_t stream) {
  MSP_REQUIRE(C > 0, "msp_bn_finalize: bad C");
  bn_finalize_kernel<<<(unsigned)C, kT, 0, as_stream(stream)>>>(
      partial, bn_parts(V, C), C, V, eps, momentum, train, running_mean, running_var, weight, bias, stats);
  return check_launch("msp_bn_finalize");
}

int msp_bn_finalize_cm(const double* partial, int64_t P, int64_t V, int C, double eps, double momentum, int train,
                       float* running_mean, float* running_var, const float* weight, const float* bias, float* stats,
                       msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && P >= 0 && (partial || !train), "msp_bn_finalize_cm: bad shape (C=%d P=%lld)", C,
              (long long)P);
  bn_finalize_cm_kernel<<<(unsigned)C, kT, 0, as_stream(stream)>>>(partial, P, C, V, eps, momentum, train,
                                                                   running_mean, running_var, weight, bias, stats);
  return check_launch("msp_bn_finalize_cm");
}

int msp_bn_apply(const float* x, int64_t V, int C, const float* stats, float leak, float* y, msp_stream_t stream) {
  const int64_t n = V * C;
  if (n == 0) return MSP_OK;
  if (C % 4 == 0 && C <= 4 * kT && aligned16(x) && aligned16(y))
    bn_apply4_kernel<<<rows_grid(V, C), kT, 0, as_stream(stream)>>>(x, V, C, stats, leak, y);
  else
    bn_apply_kernel<<<ew_grid(n), kT, 0, as_stream(stream)>>>(x, n, C, stats, leak, y);
  return check_launch("msp_bn_apply");
}

int msp_bn_bwd_stats(const float* x, const float* dy, int64_t V, int C, const float* stats, float leak,
                     double* partial, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && C <= 4096 && V >= 0, "msp_bn_bwd_stats: bad shape");
  if (C % 4 == 0 && C <= 4 * kT && aligned16(x) && aligned16(dy))
    bn_reduce4_kernel<1><<<(unsigned)bn_parts(V, C), kT, 0, as_stream(stream)>>>(x, dy, V, C, stats, leak, partial);
  else
    bn_reduce_kernel<1><<<(unsigned)bn_parts(V, C), kT, 0, as_stream(stream)>>>(x, dy, V, C, stats, leak, partial);
  return check_launch("msp_bn_bwd_stats");
}

// dx from the per-channel totals `sums` [2][C] (the finalize before it wrote them)
static int bn_bwd_apply_sums(const float* x, const float* dy, int64_t V, int C, const double* sums,
                             const float* stats, const float* weight, float leak, int train, const float* addend,
                             float* dx, hipStream_t s, int ca = 0, float* dxb = nullptr);

int msp_bn_bwd_apply_add(const float* x, const float* dy, int64_t V, int C, const double* partial,
                         const float* stats, const float* weight, float leak, int train, const float* addend,
                         float* dx, float* dweight, float* dbias, msp_stream_t stream) {
  MSP_REQUIRE(addend == nullptr || addend != dx || V * C == 0, "msp_bn_bwd_apply_add: addend must not alias dx");
  hipStream_t s = as_stream(stream);
  // The combined per-channel sums go to the extra 2*C doubles at the tail of
  // the partial buffer (it holds (P + 1) * 2 * C doubles, see the header).
  double* sums = const_cast<double*>(partial) + bn_parts(V, C) * 2 * C;
  bn_bwd_finalize_kernel<<<(unsigned)C, kT, 0, s>>>(partial, bn_parts(V, C), C, dweight, dbias, sums);
  return bn_bwd_apply_sums(x, dy, V, C, sums, stats, weight, leak, train, addend, dx, s);
}

int msp_bn_bwd_apply_cm(const float* x, const float* dy, int64_t V, int C, const double* partial, int64_t P,
                        const float* stats, const float* weight, float leak, int train, const float* addend,
                        float* dx, float* dweight, float* dbias, msp_stream_t stream) {
  MSP_REQUIRE(addend == nullptr || addend != dx || V * C == 0, "msp_bn_bwd_apply_cm: addend must not alias dx");
  MSP_REQUIRE(C > 0 && P >= 0 && partial, "msp_bn_bwd_apply_cm: bad shape (C=%d P=%lld)", C, (long long)P);
  hipStream_t s = as_stream(stream);
  double* sums = const_cast<double*>(partial) + P * 2 * C;  // the [2][C] tail
  bn_bwd_finalize_cm_kernel<<<(unsigned)C, kT, 0, s>>>(partial, P, C, dweight, dbias, sums);
  return bn_bwd_apply_sums(x, dy, V, C, sums, stats, weight, leak, train, addend, dx, s);
}

static int bn_bwd_apply_sums(const float* x, const float* dy, int64_t V, int C, const double* sums,
                             const float* stats, const float* weight, float leak, int train, const float* addend,
                             float* dx, hipStream_t s, int ca, float* dxb) {
  const int64_t n = V * C;
  if (n > 0) {
    const bool vec = C % 4 == 0 && C <= 4 * kT && aligned16(x) && aligned16(dy) && aligned16(dx) &&
                     (addend == nullptr || aligned16(addend));
    if (dxb != nullptr) {  // split output (msp_bn_bwd_apply_split); the vector form whenever the unsplit one runs
      if (vec && (ca % 4 != 0 || aligned16(dxb)))
        bn_bwd_apply4_kernel<true><<<rows_grid(V, C), kT, 0, s>>>(x, dy, V, C, sums, stats, weight, leak, train,
                                                                  addend, dx, ca, dxb);
      else
        bn_bwd_apply_kernel<true><<<ew_grid(n), kT, 0, s>>>(x, dy, n, C, V, sums, stats, weight, leak, train,
                                                             addend, dx, ca, dxb);
    } else if (vec) {
      bn_bwd_apply4_kernel<<<rows_grid(V, C), kT, 0, s>>>(x, dy, V, C, sums, stats, weight, leak, train, addend,
                                                          dx);
    } else {
      bn_bwd_apply_kernel<<<ew_grid(n), kT, 0, s>>>(x, dy, n, C, V, sums, stats, weight, leak, train, addend, dx);
    }
  }
  return check_launch("msp_bn_bwd_apply");
}

int msp_bn_bwd_apply_split(const float* x, const float* dy, int64_t V, int C, const double* partial,
                           const float* stats, const float* weight, float leak, int train, const float* addend,
                           int ca, float* dxa, float* dxb, float* dweight, float* dbias, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && ca > 0 && ca < C && V >= 0, "msp_bn_bwd_apply_split: bad split (C=%d ca=%d)", C, ca);
  MSP_REQUIRE((dxa && dxb) || V == 0, "msp_bn_bwd_apply_split: NULL output");
  MSP_REQUIRE(V == 0 || (dxa != dxb && (const float*)dxa != addend && (const float*)dxb != addend &&
                         (const float*)dxa != x && (const float*)dxb != x),
              "msp_bn_bwd_apply_split: outputs must not alias each other or an input");
  hipStream_t s = as_stream(stream);
  double* sums = const_cast<double*>(partial) + bn_parts(V, C) * 2 * C;
  bn_bwd_finalize_kernel<<<(unsigned)C, kT, 0, s>>>(partial, bn_parts(V, C), C, dweight, dbias, sums);
  return bn_bwd_apply_sums(x, dy, V, C, sums, stats, weight, leak, train, addend, dxa, s, ca, dxb);
}

int msp_bn_bwd_apply(const float* x, const float* dy, int64_t V, int C, const double* partial, const float* stats,
                     const float* weight, float leak, int train, float* dx, float* dweight, float* dbias,
                     msp_stream_t stream) {
  return msp_bn_bwd_apply_add(x, dy, V, C, partial, stats, weight, leak, train, nullptr, dx, dweight, dbias,
                              stream);
}

int msp_join_cols(const float* a, int ca, const float* b, int cb, int64_t V, float* out, double* partial,
                  msp_stream_t stream) {
  const int C = ca + cb;
  MSP_REQUIRE(ca > 0 && cb > 0 && C <= 4096 && V >= 0, "msp_join_cols: bad shape (ca=%d cb=%d)", ca, cb);
  MSP_REQUIRE((out != a && out != b) || V == 0, "msp_join_cols: out must not alias an input");
  hipStream_t s = as_stream(stream);
  if (partial && ca % 4 == 0 && cb % 4 == 0 && C <= 4 * kT && aligned16(a) && aligned16(b) && aligned16(out)) {
    bn_reduce4_kernel<3><<<(unsigned)bn_parts(V, C), kT, 0, s>>>(a, b, V, C, nullptr, 0.f, partial, out, ca);
    return check_launch("msp_join_cols");
  }
  if (V > 0) join_cols_kernel<<<ew_grid(V * C), kT, 0, s>>>(a, ca, b, cb, V, out);
  if (partial) {
    if (C % 4 == 0 && C <= 4 * kT && aligned16(out))
      bn_reduce4_kernel<0><<<(unsigned)bn_parts(V, C), kT, 0, s>>>(out, nullptr, V, C, nullptr, 0.f, partial);
    else
      bn_reduce_kernel<0><<<(unsigned)bn_parts(V, C), kT, 0, s>>>(out, nullptr, V, C, nullptr, 0.f, partial);
  }
  return check_launch("msp_join_cols");
}

int msp_split_cols(const float* in, int64_t V, int ca, int cb, float* a, float* b, msp_stream_t stream) {
  MSP_REQUIRE(ca > 0 && cb > 0 && V >= 0, "msp_split_cols: bad shape (ca=%d cb=%d)", ca, cb);
  if (V == 0 || (!a && !b)) return MSP_OK;
  hipStream_t s = as_stream(stream);
  const int C = ca + cb;
  if (ca % 4 == 0 && cb % 4 == 0 && aligned16(in) && (!a || aligned16(a)) && (!b || aligned16(b)))
    split_cols4_kernel<<<ew_grid(V * (C / 4)), kT, 0, s>>>(reinterpret_cast<const float4*>(in), V, ca / 4, cb / 4,
                                                            reinterpret_cast<float4*>(a), reinterpret_cast<float4*>(b));
  else
    split_cols_kernel<<<ew_grid(V * C), kT, 0, s>>>(in, V, ca, cb, a, b);
  return check_launch("msp_split_cols");
}

int msp_add_bn_stats(const float* a, const float* b, int64_t V, int C, float* sum, double* partial,
                     msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && C <= 4096 && V >= 0, "msp_add_bn_stats: bad shape");
  MSP_REQUIRE((sum != a && sum != b) || V * C == 0, "msp_add_bn_stats: sum must not alias an input");
  hipStream_t s = as_stream(stream);
  if (C % 4 == 0 && C <= 4 * kT && aligned16(a) && aligned16(b) && aligned16(sum)) {
    bn_reduce4_kernel<2><<<(unsigned)bn_parts(V, C), kT, 0, s>>>(a, b, V, C, nullptr, 0.f, partial, sum);
  } else {
    const int64_t n = V * C;
    if (n > 0) add_kernel<<<ew_grid(n), kT, 0, s>>>(a, b, n, sum);
    bn_reduce_kernel<0><<<(unsigned)bn_parts(V, C), kT, 0, s>>>(sum, nullptr, V, C, nullptr, 0.f, partial);
  }
  return check_launch("msp_add_bn_stats");
}

}  // extern "C"
