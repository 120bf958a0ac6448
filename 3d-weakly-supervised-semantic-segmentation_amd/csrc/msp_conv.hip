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
template <int NT>
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
      const int row = (rows >> (8 * j)) & 0xff;
      float* dst = acc_s + row * LS + r;
#pragma unroll
      for (int t = 0; t < NT; ++t) dst[t * 16] += acc[t][j];
    }
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
// (16MT x 16NT) tile of dW.  Each wave stages 16 gathered x rows and dy rows
// into its own LDS region (float4 loads) and accumulates x^T dy with MFMA;
// the four waves are then summed in fixed order and the partial tile is
// written to the block's slab.
template <int MT>
constexpr int wg_stride() { return 16 * MT + ((MT % 2 == 0) ? 16 : 0); }

template <int MT, int NT>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ block_start, int K, int64_t ppb, float* __restrict__ slab) {
  constexpr int XS = wg_stride<MT>(), YS = wg_stride<NT>();
  __shared__ float xs_s[kWaves][16 * XS];
  __shared__ float ys_s[kWaves][16 * YS];
  __shared__ float red[16 * MT * 16 * NT];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t b = blockIdx.x;
  const int o = find_offset(block_start, K, b);
  const int64_t p0 = off_start[o] + (b - block_start[o]) * ppb;
  const int64_t p1 = min(p0 + ppb, off_start[o + 1]);
  const int n_tj = c_out / (16 * NT);
  const int m0 = (blockIdx.y / n_tj) * 16 * MT, n0 = (blockIdx.y % n_tj) * 16 * NT;
  float* xw = xs_s[wave];
  float* yw = ys_s[wave];

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int64_t g = p0 + 16 * wave; g < p1; g += 16 * kWaves) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int f = lane + 64 * i;
      const int row = f / (4 * MT), col = (f % (4 * MT)) * 4;
      const int64_t pp = g + row;
      floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
      if (pp < p1) v = *reinterpret_cast<const floatx4*>(x + (int64_t)pin[pp] * c_in + m0 + col);
      *reinterpret_cast<floatx4*>(xw + row * XS + col) = v;
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int f = lane + 64 * i;
      const int row = f / (4 * NT), col = (f % (4 * NT)) * 4;
      const int64_t pp = g + row;
      floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
      if (pp < p1) v = *reinterpret_cast<const floatx4*>(dy + (int64_t)pout[pp] * c_out + n0 + col);
      *reinterpret_cast<floatx4*>(yw + row * YS + col) = v;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float a[MT], bb[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = xw[(4 * s + q) * XS + i * 16 + r];
#pragma unroll
      for (int t = 0; t < NT; ++t) bb[t] = yw[(4 * s + q) * YS + t * 16 + r];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[i][t] = mfma4(a[i], bb[t], acc[i][t]);
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
  MSP_REQUIRE(K >= 1 && K <= 255, "msp_conv_tile: bad K %d", K);
  const int64_t n_tiles = ceil_div(n_rows, MSP_TILE_ROWS);
  if (n_tiles == 0) return MSP_OK;
  const int NT = pick_tile(c_out / 16);
  dim3 grid((unsigned)ceil_div(n_tiles, kWaves), (unsigned)(c_out / (16 * NT)));
  hipStream_t s = as_stream(stream);
#define LAUNCH(N)                                                                                       \
  case N:                                                                                               \
    conv_tile_kernel<N><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off, \
                                                  chunk_src, chunk_row, n_rows, n_tiles, out);         \
    break;
  switch (NT) { LAUNCH(1) LAUNCH(2) LAUNCH(3) LAUNCH(4) }
#undef LAUNCH
  return check_launch("msp_conv_tile");
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
  const int MT = pick_tile(c_in / 16), NT = pick_tile(c_out / 16);
  if (n_blocks > 0) {
    dim3 grid((unsigned)n_blocks, (unsigned)((c_in / (16 * MT)) * (c_out / (16 * NT))));
#define LAUNCH(A, B)                                                                                  \
  if (MT == A && NT == B)                                                                             \
    conv_wgrad_kernel<A, B><<<grid, kThreads, 0, s>>>(x, c_in, dy, c_out, pair_in, pair_out, off_start, \
                                                      block_start, K, pairs_per_block, slab);
#define LAUNCH_ROW(A) LAUNCH(A, 1) LAUNCH(A, 2) LAUNCH(A, 3) LAUNCH(A, 4)
    LAUNCH_ROW(1) LAUNCH_ROW(2) LAUNCH_ROW(3) LAUNCH_ROW(4)
#undef LAUNCH_ROW
#undef LAUNCH
  }
  const int64_t cc = (int64_t)c_in * c_out;
  dim3 g2((unsigned)ceil_div(cc, 256), (unsigned)K);
  wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, block_start, cc, dw);
  return check_launch("msp_conv_wgrad");
}

}  // extern "C"
