// Helpers shared by the convolution kernels (msp_conv.hip, msp_conv_x6.hip).
#pragma once
#include "msp_common.h"

namespace msp {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;

// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8), each
// with its own L2.  Neighbouring tiles gather the same input rows, so give
// every XCD a contiguous range of logical blocks (bijective for any count).
__device__ inline int64_t xcd_linear(int64_t bid, int64_t nb) {
  const int64_t q = nb >> 3, rem = nb & 7, x = bid & 7;
  return (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + (bid >> 3);
}

// LDS tile accumulator [rows][NC] with the 16-byte column groups XOR-
// swizzled by row: 16 distinct consecutive rows at one column group land on
// 16 distinct bank quads (ds_read/write_b128 are served per 16 lanes).
template <int NC>
__device__ inline int acc_pos(int row, int g) {
  constexpr int G = NC / 4;
  if constexpr ((G & (G - 1)) == 0) {
    constexpr int RP = NC >= 64 ? 1 : 64 / NC;
    return row * NC + 4 * (g ^ ((row / RP) & (G - 1)));
  } else {
    return row * NC + 4 * ((g + row) % G);
  }
}

// W consecutive floats (W = 4: one 16-byte load, 2: 8-byte, else scalar)
template <int W>
__device__ inline void load_vec(const float* p, float (&v)[W]) {
  if (W == 4) {
    const floatx4 t = *reinterpret_cast<const floatx4*>(p);
#pragma unroll
    for (int i = 0; i < W; ++i) v[i] = t[i];
  } else if (W == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x;
    v[W - 1] = t.y;
  } else {
#pragma unroll
    for (int i = 0; i < W; ++i) v[i] = p[i];
  }
}

// out[i] = sum over splits sp = 0, 1, ... (in order) of part[sp][i]
static __global__ __launch_bounds__(256) void split_reduce_kernel(const floatx4* __restrict__ part, int n_split,
                                                                  int64_t n4, floatx4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  floatx4 s = part[i];
  for (int k = 1; k < n_split; ++k) s += part[(int64_t)k * n4 + i];
  out[i] = s;
}

// Shared-tile convolution on bf16 MFMA with exact three-piece operand splits
// (msp_conv_x6.hip), used by msp_conv_tile for 128-row tiles: nt 16-column groups per block, nb weight
// buffers, split = blocks per tile on small grids (partials reduced in split order).
struct PlanX6 {
  int nt, n_y, split, nb;
};
PlanX6 plan_x6(int64_t n_rows, int c_out);
size_t x6_ws_bytes(int64_t n_rows, int K, int c_in, int c_out, const PlanX6& p);
int launch_x6(const PlanX6& p, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
              const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
              const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, hipStream_t s);

// Per-wave split-bf16 form for narrow outputs (c_out <= 32, c_in <= 64), 128-row tiles.
int launch_x6r(const float* x, int c_in, const float* wt, int K, int flip, int c_out, const int64_t* tile_start,
               const uint8_t* chunk_off, const int32_t* chunk_src, const uint16_t* chunk_row, int64_t n_rows,
               float* out, void* ws, hipStream_t s, const msp_bn_epilogue* epi = nullptr);
size_t x6p_ws_bytes(int K, int c_in, int c_out);

// Dense row-group split-bf16 form over the neighbour map (submanifold convs).
int launch_x6g(const float* x, int c_in, const float* wt, int K, int flip, int c_out, const int32_t* nbr,
               const int32_t* perm, int64_t n_rows, float* out, void* ws, hipStream_t s);
size_t x6g_ws_bytes(int K, int c_in, int c_out);

// bf16-split weight gradient (msp_conv_x6.hip), used by msp_conv_wgrad.
int launch_wgrad_x6(const float* x, int c_in, const float* dy, int c_out, const int32_t* pair_in,
                    const int32_t* pair_out, const int64_t* off_start, int K, int64_t n_pieces, float* slab,
                    hipStream_t s);
void wgrad_x6_tile(int c_in, int c_out, int& wa, int& wb);

}  // namespace msp
