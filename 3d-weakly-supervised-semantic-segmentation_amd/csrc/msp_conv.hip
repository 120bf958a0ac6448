// Sparse convolution contractions on fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Three kernels cover every convolution pass of SparseConvUNet /
// SparseConvFCNet:
//   conv_tile   output-stationary gather-MFMA over a tile rulebook
//               (submanifold fwd + bwd-data, strided conv fwd, deconv bwd-data)
//   conv_pairs  one contribution per output row over per-offset pair lists
//               (deconv fwd, strided conv bwd-data)
//   conv_wgrad  per-offset x^T dy reductions over pair lists with a
//               deterministic slab reduction (every weight gradient)
//
// The f32-input MFMA computes exact fp32 fmaf chains (no xf32 on gfx950), so
// results match an fp32 CPU reference up to summation order.
//
// MFMA operand maps (16x16x4 f32): lane l supplies A[l&15][l>>4] and
// B[l>>4][l&15]; D[row=(l>>4)*4+j][col=l&15] in register j.  Inside a 16-wide
// channel chunk the 4 k-steps s of lane group q cover channel 4q+s, so each
// lane reads its A row and its B (weight) row as one float4.
#include "msp_common.h"

namespace msp {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ inline floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;

// ---------------------------------------------------------------- conv_tile
// One wave owns one 64-row output tile and 16*NT output channels.  For each
// 16-row chunk of its rulebook (all rows share one filter offset) it gathers
// the 16 input rows, multiplies them by that offset's weights with MFMA and
// adds the 16 x 16NT result into a wave-private LDS accumulator at the chunk's
// row positions (padding rows go to sink row 64).  The tile is stored once.
template <int NT, int ABL = 0>
__global__ __launch_bounds__(kThreads) void conv_tile_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint8_t* __restrict__ chunk_row, int64_t n_rows,
    int64_t n_tiles, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  constexpr int LS = NC + 4;  // LDS row stride (floats)
  constexpr int LR = MSP_TILE_ROWS + 1;
  __shared__ float lds[kWaves][LR * LS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * kWaves + wave;
  if (tile >= n_tiles) return;  // wave-uniform; the kernel has no block barrier
  float* acc_s = lds[wave];
  for (int i = lane; i < LR * LS; i += 64) acc_s[i] = 0.f;

  const int c0 = blockIdx.y * NC;
  const int r = lane & 15, q = lane >> 4;
  const int64_t cb = tile_start[tile], ce = tile_start[tile + 1];
  const int kcn = c_in >> 4;
  floatx4 sink[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) sink[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int64_t c = cb; c < ce; ++c) {
    const int o = chunk_off[c];
    const int ow = flip ? (K - 1 - o) : o;
    const int src = chunk_src[c * MSP_CHUNK + r];
    const uint32_t rows = *reinterpret_cast<const uint32_t*>(chunk_row + c * MSP_CHUNK + 4 * q);
    const float* xs = x + (int64_t)(src < 0 ? 0 : src) * c_in + 4 * q;
    const float* wb = wt + ((int64_t)ow * c_out + c0 + r) * c_in + 4 * q;
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < kcn; ++kc) {
      floatx4 a;
      if (ABL & 1) {
        a = floatx4{(float)kc, 1.f, 2.f, (float)src};
      } else {
        a = *reinterpret_cast<const floatx4*>(xs + kc * 16);
        if (src < 0) a = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      floatx4 b[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (ABL & 2) b[t] = floatx4{(float)ow, (float)t, 0.5f, (float)kc};
        else b[t] = *reinterpret_cast<const floatx4*>(wb + (int64_t)t * 16 * c_in + kc * 16);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[s], b[t][s], acc[t]);
      }
    }
    if (ABL & 4) {
#pragma unroll
      for (int t = 0; t < NT; ++t) sink[t] += acc[t];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (rows >> (8 * j)) & 0xff;
        float* dst = acc_s + row * LS + r;
#pragma unroll
        for (int t = 0; t < NT; ++t) dst[t * 16] += acc[t][j];
      }
    }
  }
  if (ABL & 4) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc_s[lane] += sink[t][0] + sink[t][1] + sink[t][2] + sink[t][3];
  }
  const int64_t row0 = tile * MSP_TILE_ROWS;
  const int nr = (int)((n_rows - row0) < MSP_TILE_ROWS ? (n_rows - row0) : MSP_TILE_ROWS);
  constexpr int V4 = NC / 4;
  for (int i = lane; i < nr * V4; i += 64) {
    const int rr = i / V4, cc = (i % V4) * 4;
    *reinterpret_cast<floatx4*>(out + (row0 + rr) * c_out + c0 + cc) =
        *reinterpret_cast<const floatx4*>(acc_s + rr * LS + cc);
  }
}

// ---------------------------------------------------------------- conv_tile (v4)
// Block-level offset-major form: block = 4 waves = 4 consecutive 64-row
// tiles, one 16*NT output-channel slice.  The block walks the offsets any of
// its tiles needs in (offset, 64-channel slice) steps; each step the weight
// slice W'[o][k0:k0+64][c0:c0+16NT] is staged once in LDS (double-buffered,
// one barrier per step) and every wave applies it to its <= 4 chunks of that
// offset: all gathers of the step are issued before the first MFMA.
template <int NT, int ABL = 0>
__global__ __launch_bounds__(kThreads) void conv_tile4_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint8_t* __restrict__ chunk_row, int64_t n_rows,
    int64_t n_tiles, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  constexpr int LS = NC + 2;
  constexpr int LR = MSP_TILE_ROWS + 1;
  constexpr int BF4 = 16 * NC;  // float4 per 64-channel weight slice, [k/4][n]
  constexpr int SPT = (BF4 + kThreads - 1) / kThreads;
  __shared__ float acc_lds[kWaves][LR * LS];
  __shared__ floatx4 wbuf[2][BF4];
  __shared__ unsigned long long need[2];
  __shared__ int16_t gfirst[kWaves][128];
  __shared__ uint8_t gcount[kWaves][128];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t tile = (int64_t)blockIdx.x * kWaves + wave;
  const bool active = tile < n_tiles;
  const int c0 = blockIdx.y * NC;
  float* acc_s = acc_lds[wave];
  for (int i = lane; i < LR * LS; i += 64) acc_s[i] = 0.f;
  for (int i = lane; i < 128; i += 64) {
    gcount[wave][i] = 0;
    gfirst[wave][i] = 0x7fff;
  }
  if (tid < 2) need[tid] = 0ull;
  __syncthreads();
  const int64_t cb = active ? tile_start[tile] : 0;
  const int64_t ce = active ? tile_start[tile + 1] : 0;
  for (int64_t c = cb + lane; c < ce; c += 64) {
    const int o = chunk_off[c];
    atomicOr(&need[o >> 6], 1ull << (o & 63));
    atomicAdd(reinterpret_cast<unsigned*>(&gcount[wave][0]) + (o >> 2), 1u << (8 * (o & 3)));
  }
  __syncthreads();
  // first chunk of each offset = prefix of the counts (chunks are sorted by offset)
  if (lane == 0) {
    int acc = 0;
    for (int o = 0; o < 128; ++o) {
      gfirst[wave][o] = (int16_t)acc;
      acc += gcount[wave][o];
    }
  }
  __syncthreads();
  unsigned long long it0 = need[0], it1 = need[1];
  const int nks = (c_in + 63) >> 6;
  const int n_steps = (__popcll(it0) + __popcll(it1)) * nks;

  floatx4 stage[SPT];
  auto next_offset = [&](unsigned long long& m0, unsigned long long& m1) {
    int o;
    if (m0) {
      o = __ffsll((long long)m0) - 1;
      m0 &= m0 - 1;
    } else {
      o = 64 + __ffsll((long long)m1) - 1;
      m1 &= m1 - 1;
    }
    return o;
  };
  auto load_slice = [&](int o, int ks) {
    const int ow = flip ? (K - 1 - o) : o;
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int f = tid + kThreads * i;
      const int kq = f & 15, n = f >> 4;
      const int k = ks * 64 + kq * 4;
      stage[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (f < BF4 && k < c_in)
        stage[i] = *reinterpret_cast<const floatx4*>(wt + ((int64_t)ow * c_out + c0 + n) * c_in + k);
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int f = tid + kThreads * i;
      if (f < BF4) wbuf[buf][(f & 15) * NC + (f >> 4)] = stage[i];
    }
  };

  int o_cur = 0, ks = 0;
  if (n_steps > 0) {
    o_cur = next_offset(it0, it1);
    load_slice(o_cur, 0);
    store_slice(0);
  }
  floatx4 acc[4][NT];
  for (int step = 0; step < n_steps; ++step) {
    const int gn = gcount[wave][o_cur];
    const int64_t g0 = cb + gfirst[wave][o_cur];
    if (ks == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();  // wbuf[step & 1] holds this step's slice; the other buffer is free
    const bool more = step + 1 < n_steps;
    int o_nx = o_cur, ks_nx = ks + 1;
    if (more) {
      if (ks_nx == nks) {
        ks_nx = 0;
        o_nx = next_offset(it0, it1);
      }
      load_slice(o_nx, ks_nx);
    }
    const int kcs = min(4, (c_in - ks * 64) >> 4);
    // gathers of all chunks of this step, issued before any MFMA
    int src[4];
    floatx4 a[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) src[j] = (j < gn) ? chunk_src[(g0 + j) * MSP_CHUNK + r] : -1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* xs = x + (int64_t)(src[j] < 0 ? 0 : src[j]) * c_in + ks * 64 + 4 * q;
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        if (ABL & 1)
          a[j][kc] = floatx4{(float)src[j], (float)kc, 1.f, 2.f};
        else
          a[j][kc] = (j < gn && kc < kcs) ? *reinterpret_cast<const floatx4*>(xs + kc * 16)
                                          : floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
    const floatx4* wb = wbuf[step & 1];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      if (kc < kcs) {
        floatx4 b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if (ABL & 2) b[t] = floatx4{(float)t, (float)kc, 0.5f, (float)o_cur};
          else b[t] = wb[(kc * 4 + q) * NC + t * 16 + r];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j < gn) {
            const floatx4 av = src[j] < 0 ? floatx4{0.f, 0.f, 0.f, 0.f} : a[j][kc];
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int t = 0; t < NT; ++t) acc[j][t] = mfma4(av[s], b[t][s], acc[j][t]);
          }
        }
      }
    }
    if (ks == nks - 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < gn) {
          const uint32_t rows = (ABL & 4) ? 0x40404040u : *reinterpret_cast<const uint32_t*>(chunk_row + (g0 + j) * MSP_CHUNK + 4 * q);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* dst = acc_s + ((rows >> (8 * i)) & 0xff) * LS + r;
#pragma unroll
            for (int t = 0; t < NT; ++t) dst[t * 16] += acc[j][t][i];
          }
        }
      }
    }
    if (more && !(ABL & 2)) store_slice((step + 1) & 1);
    o_cur = o_nx;
    ks = ks_nx;
  }
  if (!active) return;
  const int64_t row0 = tile * MSP_TILE_ROWS;
  const int nr = (int)((n_rows - row0) < MSP_TILE_ROWS ? (n_rows - row0) : MSP_TILE_ROWS);
  for (int i = lane; i < nr * NC; i += 64) {
    const int rr = i / NC, cc = i % NC;
    out[(row0 + rr) * c_out + c0 + cc] = acc_s[rr * LS + cc];
  }
}

// Largest o with starts[o] <= v (starts non-decreasing, starts[0] = 0).
__device__ inline int find_offset(const int64_t* __restrict__ starts, int K, int64_t v) {
  int lo = 0, hi = K;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (starts[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------- conv_pairs
template <int NT>
__global__ __launch_bounds__(kThreads) void conv_pairs_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ chunk_start, int64_t n_chunks, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t chunk = (int64_t)blockIdx.x * kWaves + wave;
  if (chunk >= n_chunks) return;
  const int o = find_offset(chunk_start, K, chunk);
  const int64_t p0 = off_start[o] + (chunk - chunk_start[o]) * MSP_CHUNK, p1 = off_start[o + 1];
  const int c0 = blockIdx.y * NC;
  const int r = lane & 15, q = lane >> 4;
  const int64_t p = p0 + r;
  const int src = p < p1 ? pin[p] : -1;
  const float* xs = x + (int64_t)(src < 0 ? 0 : src) * c_in + 4 * q;
  const float* wb = wt + ((int64_t)o * c_out + c0 + r) * c_in + 4 * q;
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int kcn = c_in >> 4;
  for (int kc = 0; kc < kcn; ++kc) {
    floatx4 a = *reinterpret_cast<const floatx4*>(xs + kc * 16);
    if (src < 0) a = floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 b[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) b[t] = *reinterpret_cast<const floatx4*>(wb + (int64_t)t * 16 * c_in + kc * 16);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[s], b[t][s], acc[t]);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t pp = p0 + 4 * q + j;
    if (pp < p1) {
      float* dst = out + (int64_t)pout[pp] * c_out + c0 + r;
#pragma unroll
      for (int t = 0; t < NT; ++t) dst[t * 16] = acc[t][j];
    }
  }
}

// ---------------------------------------------------------------- conv_wgrad
// Block = one slice of <= pairs_per_block pairs of one offset and one
// (16MT x 16NT) tile of dW.  The contraction runs over pairs: MFMA k-step s of
// lane group q takes pair 4q+s of a 16-pair group, so each lane reads its 4
// pairs' indices as one int4, and its operand values X[pair][m0+16i+r],
// dY[pair][n0+16t+r] as scalars (16 lanes = 64 contiguous bytes of a row).
// Software pipeline: the indices of group g+2 and the values of group g+1 are
// in flight while group g's MFMAs run.  The four waves interleave groups; their
// tiles are summed in fixed order and written to the block's slab.
template <int MT, int NT>
struct WgVals {
  float x[4][MT];
  float y[4][NT];
};

template <int MT, int NT>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ block_start, int K, int64_t ppb, float* __restrict__ slab) {
  __shared__ float red[16 * MT * 16 * NT];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t b = blockIdx.x;
  const int o = find_offset(block_start, K, b);
  const int64_t p0 = off_start[o] + (b - block_start[o]) * ppb;
  const int64_t p1 = min(p0 + ppb, off_start[o + 1]);
  const int n_tj = c_out / (16 * NT);
  const int m0 = (blockIdx.y / n_tj) * 16 * MT, n0 = (blockIdx.y % n_tj) * 16 * NT;

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  // groups of this wave: g_k = p0 + 16 * (wave + 4k)
  const int64_t gstride = 16 * kWaves;
  auto load_idx = [&](int64_t g, int32_t (&ii)[4], int32_t (&io)[4]) {
    const int64_t pp = g + 4 * q;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bool ok = pp + s < p1;
      ii[s] = ok ? pin[pp + s] : -1;
      io[s] = ok ? pout[pp + s] : -1;
    }
  };
  auto load_vals = [&](const int32_t (&ii)[4], const int32_t (&io)[4], WgVals<MT, NT>& v) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float* xr = x + (int64_t)(ii[s] < 0 ? 0 : ii[s]) * c_in + m0 + r;
      const float* yr = dy + (int64_t)(io[s] < 0 ? 0 : io[s]) * c_out + n0 + r;
#pragma unroll
      for (int i = 0; i < MT; ++i) v.x[s][i] = ii[s] < 0 ? 0.f : xr[16 * i];
#pragma unroll
      for (int t = 0; t < NT; ++t) v.y[s][t] = io[s] < 0 ? 0.f : yr[16 * t];
    }
  };
  auto compute = [&](const WgVals<MT, NT>& v) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[i][t] = mfma4(v.x[s][i], v.y[s][t], acc[i][t]);
  };

  int64_t g = p0 + 16 * wave;
  if (g < p1) {
    int32_t ia[4], oa[4], ib[4], ob[4];
    WgVals<MT, NT> va, vb;
    load_idx(g, ia, oa);
    load_vals(ia, oa, va);
    load_idx(g + gstride, ib, ob);
    for (;;) {
      // even: compute va (group g); values of g+stride -> vb; indices of g+2*stride -> ia
      const bool n1 = g + gstride < p1;
      if (n1) {
        load_vals(ib, ob, vb);
        load_idx(g + 2 * gstride, ia, oa);
      }
      compute(va);
      g += gstride;
      if (!n1) break;
      const bool n2 = g + gstride < p1;
      if (n2) {
        load_vals(ia, oa, va);
        load_idx(g + 2 * gstride, ib, ob);
      }
      compute(vb);
      g += gstride;
      if (!n2) break;
    }
  }
  // deterministic cross-wave sum: wave 0 stores, waves 1..3 add in order
  constexpr int RN = 16 * NT;
  for (int w = 0; w < kWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float* d = red + (i * 16 + 4 * q + j) * RN + t * 16 + r;
            *d = (w == 0) ? acc[i][t][j] : (*d + acc[i][t][j]);
          }
    }
    __syncthreads();
  }
  float* sb = slab + b * (int64_t)c_in * c_out;
  for (int e = threadIdx.x; e < 16 * MT * RN; e += kThreads) {
    const int i = e / RN, j = e % RN;
    sb[(int64_t)(m0 + i) * c_out + n0 + j] = red[e];
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab,
                                                           const int64_t* __restrict__ block_start,
                                                           int64_t cc, float* __restrict__ dw) {
  const int o = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= cc) return;
  const int64_t b0 = block_start[o], b1 = block_start[o + 1];
  float s = 0.f;
  for (int64_t b = b0; b < b1; ++b) s += slab[b * cc + e];
  dw[(int64_t)o * cc + e] = s;
}

inline int pick_tile(int n16) {
  if (n16 % 4 == 0) return 4;
  if (n16 % 3 == 0) return 3;
  if (n16 % 2 == 0) return 2;
  return 1;
}

}  // namespace msp

using namespace msp;

extern "C" {

int msp_conv_tile(const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                  const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                  const uint8_t* chunk_row, int64_t n_rows, float* out, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_tile: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= 128, "msp_conv_tile: K must be in [1, 128] (got %d)", K);
  const int64_t n_tiles = ceil_div(n_rows, MSP_TILE_ROWS);
  if (n_tiles == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  if (c_in >= 64 && (c_out / 16) % 2 == 0) {
    // block offset-major form: weights staged once per block and offset
    dim3 grid((unsigned)ceil_div(n_tiles, kWaves), (unsigned)(c_out / 32));
    conv_tile4_kernel<2><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                                   chunk_src, chunk_row, n_rows, n_tiles, out);
  } else {
    // narrow inputs (level 0 of m=32, m=16 nets): per-wave form, no barriers
    const int NT = (c_out / 16) % 2 == 0 ? 2 : 1;
    dim3 grid((unsigned)ceil_div(n_tiles, kWaves), (unsigned)(c_out / (16 * NT)));
    if (NT == 2)
      conv_tile_kernel<2><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                                    chunk_src, chunk_row, n_rows, n_tiles, out);
    else
      conv_tile_kernel<1><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                                    chunk_src, chunk_row, n_rows, n_tiles, out);
  }
  return check_launch("msp_conv_tile");
}

// Experiment hook (not part of the public ABI; scripts/kbench_conv.py): the
// two conv_tile forms with parts of their data movement replaced by constants
// to find the limiter.  abl 0-7: per-wave form (bits: 1 no gathers, 2 no
// weight loads, 4 no LDS accumulation); abl 16-23: block offset-major form
// (same bits).  nt forces NT.
int msp_debug_conv_tile(int abl, int nt, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                        const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                        const uint8_t* chunk_row, int64_t n_rows, float* out, msp_stream_t stream) {
  const int64_t n_tiles = ceil_div(n_rows, MSP_TILE_ROWS);
  if (n_tiles == 0) return MSP_OK;
  const int NT = nt > 0 ? nt : pick_tile(c_out / 16);
  MSP_REQUIRE((c_out / 16) % NT == 0, "bad nt");
  dim3 grid((unsigned)ceil_div(n_tiles, kWaves), (unsigned)(c_out / (16 * NT)));
  hipStream_t s = as_stream(stream);
#define L(N, A)                                                                                            \
  if (NT == N && abl == A)                                                                                 \
    conv_tile_kernel<N, A><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,   \
                                                     chunk_src, chunk_row, n_rows, n_tiles, out);
#define LN(N) L(N, 0) L(N, 1) L(N, 2) L(N, 3) L(N, 4) L(N, 5) L(N, 6) L(N, 7)
  LN(1) LN(2) LN(4)
#define L4(N, A)                                                                                           \
  if (NT == N && abl == 16 + A)                                                                            \
    conv_tile4_kernel<N, A><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,  \
                                                      chunk_src, chunk_row, n_rows, n_tiles, out);
  L4(2, 0) L4(2, 1) L4(2, 2) L4(2, 3) L4(2, 4) L4(2, 7)
#undef L4

#undef LN
#undef L
  return check_launch("msp_debug_conv_tile");
}

int msp_conv_pairs(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* pair_in,
                   const int32_t* pair_out, const int64_t* off_start, const int64_t* chunk_start,
                   int64_t n_chunks, float* out, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_pairs: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  if (n_chunks == 0) return MSP_OK;
  const int NT = pick_tile(c_out / 16);
  dim3 grid((unsigned)ceil_div(n_chunks, kWaves), (unsigned)(c_out / (16 * NT)));
  hipStream_t s = as_stream(stream);
#define LAUNCH(N)                                                                                       \
  case N:                                                                                               \
    conv_pairs_kernel<N><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, c_out, pair_in, pair_out, off_start, \
                                                   chunk_start, n_chunks, out);                        \
    break;
  switch (NT) { LAUNCH(1) LAUNCH(2) LAUNCH(3) LAUNCH(4) }
#undef LAUNCH
  return check_launch("msp_conv_pairs");
}

int msp_conv_wgrad(const float* x, int c_in, const float* dy, int c_out, const int32_t* pair_in,
                   const int32_t* pair_out, const int64_t* off_start, const int64_t* block_start, int K,
                   int64_t pairs_per_block, int64_t n_blocks, float* slab, float* dw, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_wgrad: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(pairs_per_block > 0 && pairs_per_block % 16 == 0, "msp_conv_wgrad: pairs_per_block % 16");
  hipStream_t s = as_stream(stream);
  // dW tiles of at most 32 x 32 per block: the register pipeline holds two
  // groups of operand values plus the accumulators (94 VGPRs at 2 x 2)
  auto pick = [](int n16) { return n16 % 2 == 0 ? 2 : (n16 % 3 == 0 ? 3 : 1); };
  const int MT = pick(c_in / 16), NT = pick(c_out / 16);
  if (n_blocks > 0) {
    dim3 grid((unsigned)n_blocks, (unsigned)((c_in / (16 * MT)) * (c_out / (16 * NT))));
#define LAUNCH(A, B)                                                                                  \
  if (MT == A && NT == B)                                                                             \
    conv_wgrad_kernel<A, B><<<grid, kThreads, 0, s>>>(x, c_in, dy, c_out, pair_in, pair_out, off_start, \
                                                      block_start, K, pairs_per_block, slab);
#define LAUNCH_ROW(A) LAUNCH(A, 1) LAUNCH(A, 2) LAUNCH(A, 3)
    LAUNCH_ROW(1) LAUNCH_ROW(2) LAUNCH_ROW(3)
#undef LAUNCH_ROW
#undef LAUNCH
  }
  const int64_t cc = (int64_t)c_in * c_out;
  dim3 g2((unsigned)ceil_div(cc, 256), (unsigned)K);
  wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, block_start, cc, dw);
  return check_launch("msp_conv_wgrad");
}

}  // extern "C"
