// Sparse convolution entry points of msp_conv_tile / msp_conv_pairs / msp_conv_wgrad.
//
//   msp_conv_tile   output-stationary convolution over a 128-row tile rulebook (submanifold levels the tile-local
//                   form does not take, strided conv fwd, deconv bwd-data): the split-bf16 MFMA kernels of
//                   msp_conv_x6.hip (per-wave tiles conv_x6r for narrow outputs, shared tiles conv_x6d otherwise)
//   msp_conv_pairs  one contribution per output row over per-offset pair lists (deconv fwd, strided conv
//                   bwd-data): f32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 fmaf chains) below
//   msp_conv_wgrad  per-offset x^T dy reductions over the pair lists (wgrad_x6_kernel, msp_conv_x6.hip) and
//                   the deterministic piece reduction below
//
// MFMA operand maps (16x16x4 f32): lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; D[row=(l>>4)*4+j][col=l&15]
// in register j.  Inside a 16-wide channel chunk the 4 k-steps s of lane group q cover channel 4q+s, so each
// lane reads its A row and its B (weight) row as one float4.
#include "msp_conv_common.h"

namespace msp {

__device__ inline floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}


// ---------------------------------------------------------------- conv_pairs
// offset o with starts[o] <= v < starts[o + 1] (starts ascending, K + 1 entries)
__device__ inline int find_offset(const int64_t* __restrict__ starts, int K, int64_t v) {
  int lo = 0, hi = K;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (starts[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

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

// dw[o][e] = sum over pieces j of slab[j][o][e]: block = 64 elements x 4
// contiguous piece segments; the segment sums are added in segment order
// (fixed order, deterministic).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, int64_t n_pieces,
                                                           int K, int64_t cc, float* __restrict__ dw) {
  __shared__ float part[4][64];
  const int o = blockIdx.y;
  const int el = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + el;
  const int64_t j0 = n_pieces * seg / 4, j1 = n_pieces * (seg + 1) / 4;
  float s = 0.f;
  if (e < cc) {
    const float* p = slab + (int64_t)o * cc + e;
    const int64_t stride = (int64_t)K * cc;
    int64_t j = j0;
    for (; j + 8 <= j1; j += 8) {  // eight loads in flight, added in piece order (same sum as one at a time)
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = p[(j + k) * stride];
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; j < j1; ++j) s += p[j * stride];
  }
  part[seg][el] = s;
  __syncthreads();
  if (seg == 0 && e < cc) dw[(int64_t)o * cc + e] = ((part[0][el] + part[1][el]) + part[2][el]) + part[3][el];
}

// ---------------------------------------------------------------- narrow inputs
// The first SubmanifoldConvolution of every encoder takes the 3 colour channels (models/SparseConvNet.py:62).
// Padded to 16 channels it ran the per-wave MFMA tile at the cost of a 32-channel layer (0.3 ms at level 0 of
// the headline batch, ~6 TF/s algorithmic) and its weight gradient the pair lists at 0.29 ms.  With CIN <= 4
// the whole contraction is 27 CIN fmaf per output element: one thread per (row, output channel), the
// neighbour indices and gathered inputs (broadcast over the COUT threads of a row) all in flight, weights in
// LDS; exact fp32 products accumulated in offset-then-channel order.
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_narrow_in_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                             int K, const int32_t* __restrict__ nbr, int64_t n,
                                                             float* __restrict__ out) {
  constexpr int RPB = 256 / COUT, KM = 27;
  __shared__ float w_s[KM * CIN * COUT];
  for (int i = threadIdx.x; i < K * CIN * COUT; i += 256) w_s[i] = wt[i];
  __syncthreads();
  const int c = threadIdx.x % COUT, rs = threadIdx.x / COUT;
  for (int64_t row = (int64_t)blockIdx.x * RPB + rs; row < n; row += (int64_t)gridDim.x * RPB) {
    int32_t nb[KM];
#pragma unroll
    for (int o = 0; o < KM; ++o) nb[o] = o < K ? nbr[o * n + row] : -1;
    float xv[KM][CIN];
#pragma unroll
    for (int o = 0; o < KM; ++o)
#pragma unroll
      for (int k = 0; k < CIN; ++k) xv[o][k] = x[(int64_t)(nb[o] < 0 ? 0 : nb[o]) * CIN + k];
    float acc = 0.f;
#pragma unroll
    for (int o = 0; o < KM; ++o)
#pragma unroll
      for (int k = 0; k < CIN; ++k)
        if (nb[o] >= 0) acc = fmaf(xv[o][k], w_s[(o * CIN + k) * COUT + c], acc);
    out[row * COUT + c] = acc;
  }
}

// dW[o][k][c] = sum over rows i with a neighbour at offset o of x[nbr(i, o)][k] dy[i][c]: block = a contiguous
// row range, thread = (row group g, output channel c) with the 27 CIN sums in registers; the row groups' sums
// are added in group order in LDS and the block's partial goes to slab[block] (wgrad_reduce_kernel adds the
// blocks in order: deterministic).
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void wgrad_narrow_in_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ dy, int K,
                                                              const int32_t* __restrict__ nbr, int64_t n,
                                                              int64_t n_parts, float* __restrict__ slab) {
  constexpr int G = 256 / COUT, KM = 27;
  __shared__ float red[KM * CIN * COUT];
  const int c = threadIdx.x % COUT, g = threadIdx.x / COUT;
  const int64_t r0 = n * blockIdx.x / n_parts, r1 = n * (blockIdx.x + 1) / n_parts;
  float acc[KM][CIN];
#pragma unroll
  for (int o = 0; o < KM; ++o)
#pragma unroll
    for (int k = 0; k < CIN; ++k) acc[o][k] = 0.f;
  for (int64_t row = r0 + g; row < r1; row += G) {
    const float d = dy[row * COUT + c];
#pragma unroll
    for (int o = 0; o < KM; ++o) {
      const int32_t nb = o < K ? nbr[o * n + row] : -1;
#pragma unroll
      for (int k = 0; k < CIN; ++k) {
        const float xv = x[(int64_t)(nb < 0 ? 0 : nb) * CIN + k];
        if (nb >= 0) acc[o][k] = fmaf(xv, d, acc[o][k]);
      }
    }
  }
  for (int gg = 0; gg < G; ++gg) {
    if (g == gg)
#pragma unroll
      for (int o = 0; o < KM; ++o)
#pragma unroll
        for (int k = 0; k < CIN; ++k) {
          float& e = red[(o * CIN + k) * COUT + c];
          e = gg == 0 ? acc[o][k] : e + acc[o][k];
        }
    __syncthreads();
  }
  float* sb = slab + (int64_t)blockIdx.x * K * CIN * COUT;
  for (int i = threadIdx.x; i < K * CIN * COUT; i += 256) sb[i] = red[i];
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

int msp_conv_tile_rows(int64_t n_rows, int c_in, int c_out) {
  (void)n_rows;
  (void)c_in;
  (void)c_out;
  // 128-row tiles everywhere: per-wave tiles for narrow outputs, shared tiles (with the offset split on small
  // grids) otherwise
  return 128;
}

int msp_conv_tile_form(int64_t n_rows, int c_in, int c_out, int tile_rows) {
  if (n_rows <= 0 || c_in <= 0 || c_out <= 0 || tile_rows != 128) return 0;
  return (c_out <= 32 && c_in <= 64) ? 1 : 2;
}

size_t msp_conv_tile_workspace_size(int64_t n_rows, int K, int c_in, int c_out, int tile_rows) {
  if (tile_rows != 128 || n_rows <= 0 || c_out <= 0 || K <= 0) return 0;
  if (c_out <= 32 && c_in <= 64) return x6p_ws_bytes(K, c_in, c_out);
  return x6_ws_bytes(n_rows, K, c_in, c_out, plan_x6(n_rows, c_out));
}

int msp_conv_tile(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                  const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                  const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                  msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_tile: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= 128, "msp_conv_tile: K must be in [1, 128] (got %d)", K);
  MSP_REQUIRE(tile_rows == 128, "msp_conv_tile: tile_rows must be 128 (got %d)", tile_rows);
  MSP_REQUIRE(flip >= 0 && flip <= 3, "msp_conv_tile: flip must be 0..3 (got %d)", flip);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  if (c_out <= 32 && c_in <= 64) {
    // narrow outputs: per-wave 128-row tiles, no barriers (msp_conv_x6.hip)
    const size_t need = x6p_ws_bytes(K, c_in, c_out);
    MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_tile: workspace too small (%zu < %zu)", ws_bytes, need);
    const int rc = launch_x6r(x, c_in, wt, K, flip, c_out, tile_start, chunk_off, chunk_src, chunk_row, n_rows, out,
                              ws, s);
    return rc ? rc : check_launch("msp_conv_tile");
  }
  // shared 128-row tiles on bf16 MFMA with exact operand splits (msp_conv_x6.hip)
  const PlanX6 p = plan_x6(n_rows, c_out);
  const size_t need = x6_ws_bytes(n_rows, K, c_in, c_out, p);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_tile: workspace too small (%zu < %zu)", ws_bytes, need);
  const int rc = launch_x6(p, x, c_in, wt, K, flip, c_out, tile_start, chunk_off, chunk_src, chunk_row, n_rows, out,
                           ws, s);
  return rc ? rc : check_launch("msp_conv_tile");
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

int msp_conv_narrow_in_ok(int K, int c_in, int c_out) {
  return (K >= 1 && K <= 27 && c_in >= 1 && c_in <= 4 && (c_out == 16 || c_out == 32 || c_out == 64)) ? 1 : 0;
}

int msp_conv_narrow_in(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* nbr,
                       int64_t n_rows, float* out, msp_stream_t stream) {
  MSP_REQUIRE(msp_conv_narrow_in_ok(K, c_in, c_out), "msp_conv_narrow_in: needs K <= 27, c_in <= 4, c_out in "
              "{16, 32, 64} (K=%d c_in=%d c_out=%d)", K, c_in, c_out);
  MSP_REQUIRE(n_rows >= 0, "msp_conv_narrow_in: n_rows must be >= 0");
  if (n_rows == 0) return MSP_OK;
  MSP_REQUIRE(x && wt && nbr && out, "msp_conv_narrow_in: null pointer");
  hipStream_t s = as_stream(stream);
  const int64_t rpb = 256 / c_out;
  int64_t grid = ceil_div(n_rows, rpb);
  if (grid > 8192) grid = 8192;
#define NL(CI, CO)                                                                                                   \
  if (c_in == CI && c_out == CO) conv_narrow_in_kernel<CI, CO><<<(unsigned)grid, 256, 0, s>>>(x, wt, K, nbr, n_rows, out);
  NL(1, 16) NL(1, 32) NL(1, 64) NL(2, 16) NL(2, 32) NL(2, 64) NL(3, 16) NL(3, 32) NL(3, 64) NL(4, 16) NL(4, 32)
  NL(4, 64)
#undef NL
  return check_launch("msp_conv_narrow_in");
}

int64_t msp_conv_wgrad_narrow_parts(int64_t n_rows, int K, int c_in, int c_out) {
  (void)K;
  (void)c_in;
  (void)c_out;
  const int64_t p = ceil_div(n_rows > 0 ? n_rows : 1, 2048);
  return p < 1 ? 1 : (p > 512 ? 512 : p);
}

int msp_conv_wgrad_narrow_in(const float* x, int c_in, const float* dy, int c_out, const int32_t* nbr, int K,
                             int64_t n_rows, int64_t n_parts, float* slab, float* dw, msp_stream_t stream) {
  MSP_REQUIRE(msp_conv_narrow_in_ok(K, c_in, c_out), "msp_conv_wgrad_narrow_in: needs K <= 27, c_in <= 4, c_out "
              "in {16, 32, 64} (K=%d c_in=%d c_out=%d)", K, c_in, c_out);
  MSP_REQUIRE(n_rows >= 0 && n_parts >= 1, "msp_conv_wgrad_narrow_in: n_rows=%lld n_parts=%lld",
              (long long)n_rows, (long long)n_parts);
  MSP_REQUIRE(x && dy && nbr && slab && dw, "msp_conv_wgrad_narrow_in: null pointer");
  hipStream_t s = as_stream(stream);
#define WL(CI, CO)                                                                                     \
  if (c_in == CI && c_out == CO)                                                                       \
    wgrad_narrow_in_kernel<CI, CO><<<(unsigned)n_parts, 256, 0, s>>>(x, dy, K, nbr, n_rows, n_parts, slab);
  WL(1, 16) WL(1, 32) WL(1, 64) WL(2, 16) WL(2, 32) WL(2, 64) WL(3, 16) WL(3, 32) WL(3, 64) WL(4, 16) WL(4, 32)
  WL(4, 64)
#undef WL
  const int64_t cc = (int64_t)c_in * c_out;
  dim3 g2((unsigned)ceil_div(cc, 64), (unsigned)K);
  wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, n_parts, K, cc, dw);
  return check_launch("msp_conv_wgrad_narrow_in");
}

int64_t msp_wgrad_pieces(int64_t total_pairs, int K, int c_in, int c_out) {
  // about 4096 blocks per launch (pieces x offsets x dW tiles), at least 256 pairs per piece; one-offset
  // contractions (network-in-network weight gradients) at most 768 pieces (fewer partial tiles to reduce)
  if (K < 1 || c_in < 16 || c_out < 16) return 1;
  int wa, wb;
  wgrad_x6_tile(c_in, c_out, wa, wb);
  const int64_t n_ty = (int64_t)(c_in / (16 * wa)) * (c_out / (16 * wb));
  int64_t n = total_pairs / ((int64_t)K * 256);
  const int64_t by_grid = 4096 / ((int64_t)K * n_ty);
  if (n > by_grid) n = by_grid;
  if (K == 1 && n > 768) n = 768;
  return n < 1 ? 1 : n;
}

int msp_conv_wgrad(const float* x, int c_in, const float* dy, int c_out, const int32_t* pair_in,
                   const int32_t* pair_out, const int64_t* off_start, int K, int64_t n_pieces, float* slab,
                   float* dw, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_wgrad: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && n_pieces >= 1, "msp_conv_wgrad: K=%d n_pieces=%lld", K, (long long)n_pieces);
  hipStream_t s = as_stream(stream);
  const int64_t cc = (int64_t)c_in * c_out;
  dim3 g2((unsigned)ceil_div(cc, 64), (unsigned)K);
  // bf16 MFMA on exact operand splits (msp_conv_x6.hip)
  MSP_REQUIRE(launch_wgrad_x6(x, c_in, dy, c_out, pair_in, pair_out, off_start, K, n_pieces, slab, s) == MSP_OK,
              "msp_conv_wgrad: no x6 kernel for c_in=%d c_out=%d", c_in, c_out);
  wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, n_pieces, K, cc, dw);
  return check_launch("msp_conv_wgrad");
}

}  // extern "C"
