// Sparse convolution contractions on fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Three kernels cover every convolution pass of SparseConvUNet /
// SparseConvFCNet:
//   conv_tile   output-stationary gather-MFMA over a tile rulebook
//               (submanifold fwd + bwd-data, strided conv fwd, deconv bwd-data)
//   conv_pairs  one contribution per output row over per-offset pair lists
//               (deconv fwd, strided conv bwd-data)
//   conv_wgrad  per-offset x^T dy reductions over row-band pieces of the
//               pair lists with a deterministic slab reduction (every
//               weight gradient)
//
// The f32-input MFMA computes exact fp32 fmaf chains (no xf32 on gfx950), so
// results match an fp32 CPU reference up to summation order.
//
// MFMA operand maps (16x16x4 f32): lane l supplies A[l&15][l>>4] and
// B[l>>4][l&15]; D[row=(l>>4)*4+j][col=l&15] in register j.  Inside a 16-wide
// channel chunk the 4 k-steps s of lane group q cover channel 4q+s, so each
// lane reads its A row and its B (weight) row as one float4.
#include "msp_conv_common.h"

namespace msp {

__device__ inline floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- conv_tile
// Both forms run the MFMA transposed, D = W^T X^T: lane (r, q) then holds
// output channels 16t + 4q .. +3 of chunk row r, so a chunk is added into the
// LDS tile accumulator with one 16-byte read-modify-write per lane and t;
// padding lanes (row 64) skip it.  Logical block l covers tile group l / n_y and channel slice
// l % n_y: the slices of a tile group run back to back on one XCD.
//
// Per-wave form: one wave owns one 64-row output tile and 16*NT output
// channels; for each 16-row chunk (all rows share one filter offset) it
// gathers the 16 input rows and the weight fragment straight into registers.
template <int NT, int ABL = 0>
__global__ __launch_bounds__(kThreads) void conv_tile_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows,
    int64_t n_tiles, int n_y, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  __shared__ floatx4 lds4[kWaves][MSP_TILE_ROWS * NC / 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t tile = (lb / n_y) * kWaves + wave;
  if (tile >= n_tiles) return;  // wave-uniform; the kernel has no block barrier
  float* acc_s = reinterpret_cast<float*>(lds4[wave]);
  for (int i = lane; i < MSP_TILE_ROWS * NC / 4; i += 64) lds4[wave][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int c0 = (int)(lb % n_y) * NC;
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
    const int row = chunk_row[c * MSP_CHUNK + r];
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
        for (int t = 0; t < NT; ++t) acc[t] = mfma4(b[t][s], a[s], acc[t]);
      }
    }
    if (ABL & 4) {
#pragma unroll
      for (int t = 0; t < NT; ++t) sink[t] += acc[t];
    } else if (row < MSP_TILE_ROWS) {
#pragma unroll
      for (int t = 0; t < NT; ++t) *reinterpret_cast<floatx4*>(acc_s + acc_pos<NC>(row, 4 * t + q)) += acc[t];
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
    const int rr = i / V4, g = i % V4;
    *reinterpret_cast<floatx4*>(out + (row0 + rr) * c_out + c0 + 4 * g) =
        *reinterpret_cast<const floatx4*>(acc_s + acc_pos<NC>(rr, g));
  }
}

// Pipelined per-wave form for c_in = 16*KC <= 64: chunk indices are loaded
// two chunks ahead, input rows and weight fragments one chunk ahead, so a
// wave always has the next chunk's loads in flight while it runs MFMAs.
template <int NT, int KC, int TR = MSP_TILE_ROWS>
__global__ __launch_bounds__(kThreads) void conv_tilep_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows,
    int64_t n_tiles, int n_y, float* __restrict__ out) {
  constexpr int NC = 16 * NT, C_IN = 16 * KC;
  __shared__ floatx4 lds4[kWaves][TR * NC / 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t tile = (lb / n_y) * kWaves + wave;
  if (tile >= n_tiles) return;  // wave-uniform; the kernel has no block barrier
  float* acc_s = reinterpret_cast<float*>(lds4[wave]);
  for (int i = lane; i < TR * NC / 4; i += 64) lds4[wave][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int c0 = (int)(lb % n_y) * NC;
  const int r = lane & 15, q = lane >> 4;
  const int64_t cb = tile_start[tile], ce = tile_start[tile + 1];

  struct St {
    int o, src, row;
  };
  // Branch-free loads: chunk positions past the tile's last chunk are clamped
  // to it (loads stay in range, the work is skipped by a uniform branch), so
  // the compiler's wait counts stay exact and a prefetch is never waited for
  // before it is consumed (conditional loads made it drain every load at the
  // MFMAs).
  const int64_t clast = ce > cb ? ce - 1 : cb;
  auto ld_idx = [&](int64_t c, St& d) {
    const int64_t cc = c < clast ? c : clast;
    d.o = chunk_off[cc];
    d.src = chunk_src[cc * MSP_CHUNK + r];
    d.row = chunk_row[cc * MSP_CHUNK + r];
  };
  auto ld_val = [&](const St& d, floatx4 (&av)[KC], floatx4 (&bv)[NT][KC]) {
    // padding slots hold a present row (see the header); their result column
    // is never stored
    const float* xs = x + (int64_t)d.src * C_IN + 4 * q;
    const int ow = flip ? (K - 1 - d.o) : d.o;
    const float* wb = wt + ((int64_t)ow * c_out + c0 + r) * C_IN + 4 * q;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      av[kc] = *reinterpret_cast<const floatx4*>(xs + kc * 16);
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[t][kc] = *reinterpret_cast<const floatx4*>(wb + t * 16 * C_IN + kc * 16);
    }
  };
  auto run = [&](const floatx4 (&av)[KC], const floatx4 (&bv)[NT][KC], int row, bool live) {
    if (live) {
      floatx4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma4(bv[t][kc][s], av[kc][s], acc[t]);
      if (row < TR) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          *reinterpret_cast<floatx4*>(acc_s + acc_pos<NC>(row, 4 * t + q)) += acc[t];
      }
    }
    // mark the set read on every path (see conv_tile7_kernel)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      asm volatile("" ::"v"(av[kc]));
#pragma unroll
      for (int t = 0; t < NT; ++t) asm volatile("" ::"v"(bv[t][kc]));
    }
  };
  // D register sets used in turn (no copies of loaded values): chunk c+k
  // computes from set k while the other sets' loads (chunks up to c+k+D-1)
  // are in flight; a chunk's indices are loaded D chunks before its values.
  // Trip count a multiple of D; chunk positions past the end compute nothing.
  constexpr int D = 2;  // 4 was measured: no gain at level 0 (35.8 vs 36.4 TF/s)
  St J[D];
  int rowR[D];
  floatx4 S_a[D][KC], S_b[D][NT][KC];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    ld_idx(cb + k, J[k]);
    rowR[k] = J[k].row;
    ld_val(J[k], S_a[k], S_b[k]);
  }
#pragma unroll
  for (int k = 0; k < D; ++k) ld_idx(cb + D + k, J[k]);
  for (int64_t c = cb; c < ce; c += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      run(S_a[k], S_b[k], rowR[k], c + k < ce);
      ld_val(J[k], S_a[k], S_b[k]);  // chunk c+k+D
      rowR[k] = J[k].row;
      ld_idx(c + k + 2 * D, J[k]);
    }
  }
  const int64_t row0 = tile * TR;
  const int nr = (int)((n_rows - row0) < TR ? (n_rows - row0) : TR);
  constexpr int V4 = NC / 4;
  for (int i = lane; i < nr * V4; i += 64) {
    const int rr = i / V4, g = i % V4;
    *reinterpret_cast<floatx4*>(out + (row0 + rr) * c_out + c0 + 4 * g) =
        *reinterpret_cast<const floatx4*>(acc_s + acc_pos<NC>(rr, g));
  }
}

// ---------------------------------------------------------------- conv_tile (block form)
// Block-level offset-major form: block = 4 waves = 4 consecutive 64-row
// tiles, one 16*NT output-channel slice.  The block walks the offsets any of
// its tiles needs in (offset, 64-channel slice) steps; each step the weight
// slice W'[o][k0:k0+64][c0:c0+16NT] is staged once in LDS (double-buffered,
// one barrier per step) and every wave applies it to its <= 4 chunks of that
// offset: all gathers of the step are issued before the first MFMA.
template <int NT, int ABL = 0, bool PF = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(3))) void conv_tile4_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows,
    int64_t n_tiles, int n_y, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  constexpr int BF4 = 16 * NC;  // float4 per 64-channel weight slice, [k/4][n]
  constexpr int SPT = (BF4 + kThreads - 1) / kThreads;
  __shared__ floatx4 acc_lds4[kWaves][MSP_TILE_ROWS * NC / 4];
  __shared__ floatx4 wbuf[2][BF4];
  __shared__ unsigned long long need[2];
  __shared__ int16_t gfirst[kWaves][128];
  __shared__ uint8_t gcount[kWaves][128];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t tile = (lb / n_y) * kWaves + wave;
  const bool active = tile < n_tiles;
  const int c0 = (int)(lb % n_y) * NC;
  float* acc_s = reinterpret_cast<float*>(acc_lds4[wave]);
  for (int i = lane; i < MSP_TILE_ROWS * NC / 4; i += 64) acc_lds4[wave][i] = floatx4{0.f, 0.f, 0.f, 0.f};
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
  // wave-uniform offset masks in scalar registers
  auto uniform64 = [](unsigned long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
  };
  unsigned long long it0 = uniform64(need[0]), it1 = uniform64(need[1]);
  const int nks = (c_in + 63) >> 6;
  const int n_steps = (__popcll(it0) + __popcll(it1)) * nks;

  floatx4 stage[SPT];
  auto next_offset = [&](unsigned long long& m0, unsigned long long& m1) {
    // branch-free (a data-dependent choice between the two references made
    // the compiler keep them in scratch)
    const bool lo = m0 != 0ull;
    const unsigned long long mm = lo ? m0 : m1;
    const int o = (lo ? 0 : 64) + __ffsll((long long)mm) - 1;
    const unsigned long long nm = mm & (mm - 1);
    m0 = lo ? nm : m0;
    m1 = lo ? m1 : nm;
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
      if (f < BF4) wbuf[buf][(f & 15) * NC + ((f >> 4) ^ (f & 15))] = stage[i];  // n ^ kq: conflict-free
    }
  };

  // Chunk indices of a step are loaded one step ahead; with PF the input rows
  // are gathered one step ahead too, so the only exposed latency per step is
  // the barrier.
  struct Idx {
    int src[4], row[4], gn;
  };
  auto load_idx = [&](int o, Idx& d) {
    d.gn = __builtin_amdgcn_readfirstlane(gcount[wave][o]);
    const int64_t g0 = cb + __builtin_amdgcn_readfirstlane(gfirst[wave][o]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d.src[j] = (j < d.gn) ? chunk_src[(g0 + j) * MSP_CHUNK + r] : -1;
      d.row[j] = (j < d.gn) ? (int)chunk_row[(g0 + j) * MSP_CHUNK + r] : MSP_TILE_ROWS;
    }
  };
  auto gather = [&](const Idx& d, int kslice, floatx4 (&av)[4][4]) {
    const int kcs = min(4, (c_in - kslice * 64) >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // padding slots hold a present row (see the header); their result
      // column is never stored
      const float* xs = x + (int64_t)d.src[j] * c_in + kslice * 64 + 4 * q;
      if (j < d.gn) {
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
          if (ABL & 1)
            av[j][kc] = floatx4{(float)d.src[j], (float)kc, 1.f, 2.f};
          else if (kc < kcs)
            av[j][kc] = *reinterpret_cast<const floatx4*>(xs + kc * 16);
        }
      }
    }
  };

  int o_cur = 0, ks = 0;
  Idx ic;
  floatx4 a[4][4];
  if (n_steps > 0) {
    o_cur = next_offset(it0, it1);
    load_slice(o_cur, 0);
    store_slice(0);
    load_idx(o_cur, ic);
    if (PF) gather(ic, 0, a);
  }
  floatx4 acc[4][NT];
  floatx4 sink[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) sink[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int step = 0; step < n_steps; ++step) {
    const int gn = ic.gn;
    if (ks == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (!(ABL & 8)) __syncthreads();  // wbuf[step & 1] holds this step's slice; the other buffer is free
    const bool more = step + 1 < n_steps;
    int o_nx = o_cur, ks_nx = ks + 1;
    if (more && ks_nx == nks) {
      ks_nx = 0;
      o_nx = next_offset(it0, it1);
    }
    if (more) load_slice(o_nx, ks_nx);
    Idx in = ic;
    if (more && ks_nx == 0) load_idx(o_nx, in);
    floatx4 an[4][4];
    if (PF) {
      if (more) gather(in, ks_nx, an);
    } else {
      gather(ic, ks, a);
    }
    const int kcs = min(4, (c_in - ks * 64) >> 4);
    const floatx4* wb = wbuf[step & 1];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      if (kc < kcs) {
        floatx4 b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if (ABL & 2) b[t] = floatx4{(float)t, (float)kc, 0.5f, (float)o_cur};
          else b[t] = wb[(kc * 4 + q) * NC + ((t * 16 + r) ^ (kc * 4 + q))];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j < gn) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int t = 0; t < NT; ++t) acc[j][t] = mfma4(b[t][s], a[j][kc][s], acc[j][t]);
          }
        }
      }
    }
    if ((ABL & 4) && ks == nks - 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < gn)
#pragma unroll
          for (int t = 0; t < NT; ++t) sink[t] += acc[j][t];
    } else if (ks == nks - 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < gn) {
          const int row = ic.row[j];
          if (row < MSP_TILE_ROWS) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
              *reinterpret_cast<floatx4*>(acc_s + acc_pos<NC>(row, 4 * t + q)) += acc[j][t];
          }
        }
      }
    }
    if (more && !(ABL & 2)) store_slice((step + 1) & 1);
    o_cur = o_nx;
    ks = ks_nx;
    ic = in;
    if (PF) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) a[j][kc] = an[j][kc];
    }
  }
  if (ABL & 4) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc_s[lane] += sink[t][0] + sink[t][1] + sink[t][2] + sink[t][3];
  }
  if (!active) return;
  const int64_t row0 = tile * MSP_TILE_ROWS;
  const int nr = (int)((n_rows - row0) < MSP_TILE_ROWS ? (n_rows - row0) : MSP_TILE_ROWS);
  constexpr int V4 = NC / 4;
  for (int i = lane; i < nr * V4; i += 64) {
    const int rr = i / V4, g = i % V4;
    *reinterpret_cast<floatx4*>(out + (row0 + rr) * c_out + c0 + 4 * g) =
        *reinterpret_cast<const floatx4*>(acc_s + acc_pos<NC>(rr, g));
  }
}

// ---------------------------------------------------------------- conv_tile (shared tile, software pipelined)
// Block = 4 waves sharing ONE output tile of TR rows and one 16*NT
// output-channel slice, accumulated in LDS.  The block walks the offsets the
// tile needs in (offset, 64-channel k-slice) steps; the weight slice is
// staged in LDS once per step (double-buffered, one barrier per step) and the
// offset's chunks are dealt round-robin to the waves (wave w takes chunks w,
// w+4, ...).  Chunks of one offset cover distinct rows, so the waves' LDS
// read-modify-writes of a step never collide, and the per-step barrier
// orders steps.  Compared with per-wave 64-row tiles the larger tile packs
// the chunks denser (fewer padding rows) and the waves of a step carry
// equal work.  The kernel is written so that no load is ever
// waited for before it is consumed: every load is unconditional (indices and
// channel offsets are clamped into range; the work they would feed is
// skipped by uniform branches), loaded registers are never copied, and the
// register sets of consecutive steps alternate by unrolling the step loop
// by two.  Per step s, in issue order:
//   barrier | src(s+2) | weights(s+1) | gathers(s+1) | MFMAs(s) | LDS
//   read-modify-write(s) | rows(s+2) | weights(s+1) -> LDS
// so the gathers of a step have a whole step of MFMAs to land, and the
// index loads two.
template <int NT, int TR, int ABL = 0>
__global__ __launch_bounds__(kThreads) void conv_tile7_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows,
    int n_y, int n_split, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  constexpr int BF4 = 16 * NC;  // float4 per 64-channel weight slice, [k/4][n]
  constexpr int SPT = (BF4 + kThreads - 1) / kThreads;
  constexpr int MJ = TR / (16 * kWaves);  // chunk slots per wave and step
  __shared__ floatx4 acc4[TR * NC / 4];
  __shared__ floatx4 wbuf[2][BF4];
  __shared__ unsigned long long need[2];
  __shared__ int gfirst[128];
  __shared__ int gcount[128];
  __shared__ uint8_t olist[128];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  // logical block = (tile, channel slice, split): the splits of a tile are
  // adjacent (one XCD).  With n_split > 1 split sp takes the sp-th share of
  // the tile's offsets and writes its partial sums to out + sp*n_rows*c_out
  // (summed in split order by split_reduce_kernel).
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int sp = (int)(lb % n_split);
  const int64_t rest = lb / n_split;
  const int64_t tile = rest / n_y;
  const int c0 = (int)(rest % n_y) * NC;
  float* dst = out + (int64_t)sp * n_rows * c_out;
  float* acc_s = reinterpret_cast<float*>(acc4);
  for (int i = tid; i < TR * NC / 4; i += kThreads) acc4[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (tid < 128) gcount[tid] = 0;
  if (tid < 2) need[tid] = 0ull;
  __syncthreads();
  const int64_t cb = tile_start[tile], ce = tile_start[tile + 1];
  for (int64_t c = cb + tid; c < ce; c += kThreads) {
    const int o = chunk_off[c];
    if (c == cb || chunk_off[c - 1] != o) {  // chunks are sorted by offset
      gfirst[o] = (int)(c - cb);
      atomicOr(&need[o >> 6], 1ull << (o & 63));
    }
    atomicAdd(&gcount[o], 1);
  }
  __syncthreads();
  if (tid < 128) {  // olist[i] = i-th needed offset (ascending)
    const unsigned long long m0 = need[0], m1 = need[1];
    const bool has = tid < 64 ? ((m0 >> tid) & 1ull) : ((m1 >> (tid - 64)) & 1ull);
    const int below = tid < 64 ? __popcll(m0 & ((1ull << tid) - 1ull))
                               : __popcll(m0) + __popcll(m1 & ((1ull << (tid - 64)) - 1ull));
    if (has) olist[below] = (uint8_t)tid;
  }
  // (readfirstlane returns int: go through unsigned so bit 31 does not sign-extend)
  auto uniform64 = [](unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
  };
  const int n_off_all = __popcll(uniform64(need[0])) + __popcll(uniform64(need[1]));
  const int oi0 = sp * n_off_all / n_split;
  const int n_off = (sp + 1) * n_off_all / n_split - oi0;
  __syncthreads();
  const int nks = (c_in + 63) >> 6;
  const int n_steps = n_off * nks;
  if (n_steps == 0) {
    // no rules: the tile's rows are zero
    const int64_t row0 = tile * TR;
    const int nr = (int)((n_rows - row0) < TR ? (n_rows - row0) : TR);
    for (int i = tid; i < nr * NC / 4; i += kThreads)
      *reinterpret_cast<floatx4*>(dst + (row0 + i / (NC / 4)) * c_out + c0 + 4 * (i % (NC / 4))) =
          floatx4{0.f, 0.f, 0.f, 0.f};
    return;
  }

  // Step descriptor, all scalar: offset index oi into olist, k-slice ks,
  // offset o, first chunk l0, chunk count cnt and this wave's chunk count gn.
  // Built incrementally (one LDS read per step); past the last step it
  // repeats the last one so its loads stay in range.
  struct Step {
    int oi, ks, o, l0, cnt, gn;
  };
  auto fill = [&](Step& d) {
    const bool live = d.oi < n_off;
    const int oc = live ? d.oi : n_off - 1;
    d.o = __builtin_amdgcn_readfirstlane(olist[oi0 + oc]);
    d.cnt = __builtin_amdgcn_readfirstlane(gcount[d.o]);
    d.l0 = __builtin_amdgcn_readfirstlane(gfirst[d.o]);
    const int gn = (d.cnt - wave + kWaves - 1) / kWaves;
    d.gn = !live || gn < 0 ? 0 : (gn > MJ ? MJ : gn);  // steps past the end do nothing
  };
  auto advance = [&](const Step& d) {
    Step e;
    e.ks = d.ks + 1;
    e.oi = d.oi;
    if (e.ks == nks) {
      e.ks = 0;
      e.oi = d.oi + 1;
    }
    fill(e);
    return e;
  };
  // chunk slot j of this wave; slots past the offset's chunks read its first chunk
  auto chunk_elem = [&](const Step& d, int j) {
    const int l = wave + kWaves * j;
    return (cb + d.l0 + (l < d.cnt ? l : 0)) * MSP_CHUNK + r;
  };
  struct Src {
    int32_t v[MJ];
  };
  struct Row {
    int v[MJ];
  };
  struct Val {
    floatx4 a[MJ][4];
  };
  floatx4 stage[SPT];
  auto ld_src = [&](const Step& sd, Src& d) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) d.v[j] = chunk_src[chunk_elem(sd, j)];
  };
  auto ld_row = [&](const Step& sd, Row& d) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) d.v[j] = chunk_row[chunk_elem(sd, j)];
  };
  auto ld_w = [&](const Step& sd) {
    const int ow = flip ? (K - 1 - sd.o) : sd.o;
    const float* wo = wt + ((int64_t)ow * c_out + c0) * c_in;
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int f = (tid + kThreads * i) < BF4 ? tid + kThreads * i : BF4 - 1;
      const int kq = f & 15, n = f >> 4;
      const int k = min(sd.ks * 64 + kq * 4, c_in - 4);
      stage[i] = *reinterpret_cast<const floatx4*>(wo + n * c_in + k);
    }
  };
  auto st_w = [&](int buf) {
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int f = tid + kThreads * i;
      if (f < BF4) wbuf[buf][(f & 15) * NC + ((f >> 4) ^ (f & 15))] = stage[i];
    }
  };
  // 32-bit byte offsets from the uniform base (x < 4 GiB): saddr + voffset loads
  const char* xb = reinterpret_cast<const char*>(x);
  const uint32_t row_bytes = (uint32_t)c_in * 4u;
  auto gather = [&](const Step& sd, const Src& sv, Val& v) {
    const int kb = sd.ks * 64;
    const bool full = kb + 64 <= c_in;  // uniform
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const uint32_t ro = (uint32_t)sv.v[j] * row_bytes + 16u * q;
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        const int k = full ? kb + kc * 16 : min(kb + kc * 16, c_in - 16);
        if (ABL & 2)
          v.a[j][kc] = floatx4{(float)sv.v[j], (float)kc, 1.f, 2.f};
        else
          v.a[j][kc] = *reinterpret_cast<const floatx4*>(xb + (ro + 4u * (uint32_t)k));
      }
    }
  };
  floatx4 acc[MJ][NT];
  auto mma = [&](const Step& sd, int buf, const Val& v) {
    if (sd.ks == 0) {
#pragma unroll
      for (int j = 0; j < MJ; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    const int kcs = min(4, (c_in - sd.ks * 64) >> 4);
    const floatx4* wb = wbuf[buf];
    auto ld_b = [&](int kc, floatx4 (&b)[NT]) {
#pragma unroll
      for (int t = 0; t < NT; ++t) b[t] = wb[(kc * 4 + q) * NC + ((t * 16 + r) ^ (kc * 4 + q))];
    };
    auto mm = [&](int kc, const floatx4 (&b)[NT]) {
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        if (j < sd.gn) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[j][t] = mfma4(b[t][s], v.a[j][kc][s], acc[j][t]);
        }
      }
    };
    {
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        if (kc < kcs) {
          floatx4 b[NT];
          ld_b(kc, b);
          mm(kc, b);
        }
      }
    }
  };
  // Mark loaded registers as read on every path (slots a step skipped by a
  // uniform branch included), so the compiler never finds a load into them
  // still in flight when it reuses them later and does not insert a wait for
  // every younger load there.  Placed where these loads are complete anyway.
  auto consume_val = [&](const Val& v) {
#pragma unroll
    for (int j = 0; j < MJ; ++j)
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) asm volatile("" ::"v"(v.a[j][kc]));
  };
  auto consume_row = [&](const Row& rw) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) asm volatile("" ::"v"(rw.v[j]));
  };
  auto rmw = [&](const Step& sd, const Row& rw) {
    if (sd.ks != nks - 1) return;
    if (ABL & 4) {  // ablation: no LDS accumulation (sum into one slot)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        if (j < sd.gn)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc_s[lane] += acc[j][t][0] + acc[j][t][1] + acc[j][t][2] + acc[j][t][3];
      return;
    }
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (j < sd.gn && rw.v[j] < TR) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          *reinterpret_cast<floatx4*>(acc_s + acc_pos<NC>(rw.v[j], 4 * t + q)) += acc[j][t];
      }
    }
  };

  Step d0;
  d0.oi = 0;
  d0.ks = 0;
  fill(d0);
  Step d1 = advance(d0);
  Src s0, s1;
  Row r0, r1;
  Val v0, v1;
  ld_src(d0, s0);
  ld_src(d1, s1);
  ld_w(d0);
  ld_row(d0, r0);
  ld_row(d1, r1);
  gather(d0, s0, v0);
  st_w(0);
  // one step: dc = this step, dn = the next one; returns the step after dn
  auto body = [&](int st, const Step& dc, const Step& dn, Src& s_cur, Src& s_nxt, Row& r_cur, Val& v_cur,
                  Val& v_nxt) {
    const Step d2 = advance(dn);
    if (!(ABL & 1)) __syncthreads();  // wbuf[st & 1] holds this step's slice; all step st-1 LDS updates are done
    ld_src(d2, s_cur);
    ld_w(dn);
    gather(dn, s_nxt, v_nxt);
    mma(dc, st & 1, v_cur);
    consume_val(v_cur);
    rmw(dc, r_cur);
    consume_row(r_cur);
    ld_row(d2, r_cur);
    st_w((st + 1) & 1);
    return d2;
  };
  // even trip count: a step past the end loads in range and computes nothing
  for (int st = 0; st < n_steps; st += 2) {
    const Step d2 = body(st, d0, d1, s0, s1, r0, v0, v1);
    const Step d3 = body(st + 1, d1, d2, s1, s0, r1, v1, v0);
    d0 = d2;
    d1 = d3;
  }
  __syncthreads();
  const int64_t row0 = tile * TR;
  const int nr = (int)((n_rows - row0) < TR ? (n_rows - row0) : TR);
  constexpr int V4 = NC / 4;
  for (int i = tid; i < nr * V4; i += kThreads) {
    const int rr = i / V4, g = i % V4;
    *reinterpret_cast<floatx4*>(dst + (row0 + rr) * c_out + c0 + 4 * g) =
        *reinterpret_cast<const floatx4*>(acc_s + acc_pos<NC>(rr, g));
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
// Weight gradient.  Block = piece j of offset o's pair list (see
// msp_conv_wgrad in the header) and one (16WA x 16WB) tile of dW; MFMA k-step = 4 pairs, one per
// lane group q.  Lane r loads WA consecutive input channels
// m0 + WA*r .. and WB consecutive output channels n0 + WB*r .. of its pair
// (16 lanes read whole 64-wide row slices), and the WA x WB MFMAs of a k-step
// take component (sa, sb): accumulator (sa, sb) holds
//   dW[m0 + WA*(4q + j) + sa][n0 + WB*r + sb]   (register j of lane (r, q)).
// Indices run two 16-pair super-steps ahead, values one.  Waves take
// super-steps round-robin;
// their tiles are summed in fixed order into the block's slab (deterministic).

template <int WA, int WB>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(WA * WB > 9 ? 2 : 3))) void conv_wgrad4_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    int K, int64_t n_pieces, int n_ty, float* __restrict__ slab) {
  constexpr int TM = 16 * WA, TN = 16 * WB;
  __shared__ float red[TM * TN];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  // logical block = ((piece j * K) + offset o) * n_ty + channel tile: the K
  // pieces of one row band and their channel tiles are adjacent on one XCD
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t b = lb / n_ty;  // slab index j * K + o
  const int ty = (int)(lb % n_ty);
  const int n_tj = c_out / TN;
  const int m0 = (ty / n_tj) * TM, n0 = (ty % n_tj) * TN;
  const int o = (int)(b % K);
  const int64_t j = b / K;
  const int64_t os = off_start[o], cnt = off_start[o + 1] - os;
  const int64_t p0 = os + cnt * j / n_pieces;
  const int64_t p1 = os + cnt * (j + 1) / n_pieces;

  floatx4 acc[WA][WB];
#pragma unroll
  for (int i = 0; i < WA; ++i)
#pragma unroll
    for (int t = 0; t < WB; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  // super-step = 16 pairs: lane group q takes pairs g + 4q .. g + 4q + 3 as
  // its four k-steps.  Loads are branch-free and nothing is computed from a
  // loaded value until it is consumed (a select right after a load would make
  // the wave wait for every younger load too): positions past the piece are
  // clamped to its last pair and masked out when the MFMA operands are formed.
  struct Ix {
    int32_t i[4], o[4];
    bool ok[4];
  };
  struct Vals {
    float a[4][WA], b[4][WB];
    bool ok[4];
  };
  auto ld_idx = [&](int64_t g, Ix& d) {
    const int64_t pp = g + 4 * q;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t pc = min(pp + k, p1 - 1);
      d.ok[k] = pp + k < p1;
      d.i[k] = pin[pc];
      d.o[k] = pout[pc];
    }
  };
  auto ld_val = [&](const Ix& d, Vals& v) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      load_vec<WA>(x + (int64_t)d.i[k] * c_in + m0 + WA * r, v.a[k]);
      load_vec<WB>(dy + (int64_t)d.o[k] * c_out + n0 + WB * r, v.b[k]);
      v.ok[k] = d.ok[k];
    }
  };
  auto compute = [&](const Vals& v) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < WA; ++i) {
        const float av = v.ok[k] ? v.a[k][i] : 0.f;
#pragma unroll
        for (int t = 0; t < WB; ++t) acc[i][t] = mfma4(av, v.b[k][t], acc[i][t]);
      }
  };

  // D register sets used in turn (no copies of loaded values): super-step
  // g+k computes from set k while the loads of the next D-1 super-steps are
  // in flight; indices are loaded D super-steps before their values.  Loads
  // are never conditional (positions past the piece are clamped and masked
  // by `ok`), so the compiler's wait counts stay exact.  Small dW tiles do
  // little MFMA work per super-step and get the deeper pipeline.
  constexpr int D = (WA * WB <= 4) ? 4 : 2;  // measured: 6 (L0) and 3 (L2) are slower
  constexpr int64_t kStride = 16 * kWaves;
  const int64_t g0 = p0 + 16 * wave;
  if (g0 < p1) {  // wave-uniform
    Ix X[D];
    Vals V[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      ld_idx(g0 + k * kStride, X[k]);
      ld_val(X[k], V[k]);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) ld_idx(g0 + (D + k) * kStride, X[k]);
    for (int64_t g = g0; g < p1; g += D * kStride) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        if (g + k * kStride < p1) compute(V[k]);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {  // mark the set read on every path
#pragma unroll
          for (int i = 0; i < WA; ++i) asm volatile("" ::"v"(V[k].a[kk][i]));
#pragma unroll
          for (int t = 0; t < WB; ++t) asm volatile("" ::"v"(V[k].b[kk][t]));
        }
        ld_val(X[k], V[k]);
        ld_idx(g + (2 * D + k) * kStride, X[k]);
      }
    }
  }
  // deterministic cross-wave sum: wave 0 stores, waves 1..3 add in order
  for (int w = 0; w < kWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < WA; ++i)
#pragma unroll
        for (int t = 0; t < WB; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float* d = red + (WA * (4 * q + j) + i) * TN + WB * r + t;
            *d = (w == 0) ? acc[i][t][j] : (*d + acc[i][t][j]);
          }
    }
    __syncthreads();
  }
  float* sb = slab + b * (int64_t)c_in * c_out;
  for (int e = threadIdx.x; e < TM * TN; e += kThreads) {
    const int i = e / TN, j = e % TN;
    sb[(int64_t)(m0 + i) * c_out + n0 + j] = red[e];
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

inline int pick_tile(int n16) {
  if (n16 % 4 == 0) return 4;
  if (n16 % 3 == 0) return 3;
  if (n16 % 2 == 0) return 2;
  return 1;
}

}  // namespace msp

using namespace msp;

extern "C" {

namespace {

int launch_tile7(int nt, int tile_rows, int split, const float* x, int c_in, const float* wt, int K, int flip,
                 int c_out, const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                 const uint16_t* chunk_row, int64_t n_rows, float* out, float* part, hipStream_t s) {
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  const int n_y = c_out / (16 * nt);
  const unsigned grid = (unsigned)(n_tiles * n_y * split);
  float* dst = split > 1 ? part : out;
  bool launched = false;
#define L7(N, T)                                                                                              \
  if (!launched && nt == N && tile_rows == T) {                                                               \
    conv_tile7_kernel<N, T><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,     \
                                                      chunk_src, chunk_row, n_rows, n_y, split, dst);         \
    launched = true;                                                                                          \
  }
  L7(1, 128) L7(2, 128) L7(3, 128) L7(4, 128) L7(2, 256) L7(4, 256)
#undef L7
  if (!launched) {
    set_error("msp_conv_tile: no shared-tile kernel for nt=%d tile_rows=%d", nt, tile_rows);
    return MSP_EINVAL;
  }
  if (split > 1) {
    const int64_t n4 = n_rows * c_out / 4;
    split_reduce_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, s>>>(reinterpret_cast<const floatx4*>(part), split,
                                                                    n4, reinterpret_cast<floatx4*>(out));
  }
  return MSP_OK;
}

}  // namespace

int msp_conv_tile_rows(int64_t n_rows, int c_in, int c_out) {
  (void)n_rows;
  (void)c_in;
  (void)c_out;
  // 128-row tiles everywhere: per-wave pipelined tiles for narrow outputs,
  // shared tiles (with the offset split on small grids) otherwise
  return 128;
}

int msp_conv_tile_form(int64_t n_rows, int c_in, int c_out, int tile_rows) {
  if (n_rows <= 0 || c_in <= 0 || c_out <= 0) return 0;
  if (tile_rows != 128) return 3;
  return (c_out <= 32 && c_in <= 64) ? 1 : 2;
}

size_t msp_conv_tile_workspace_size(int64_t n_rows, int K, int c_in, int c_out, int tile_rows) {
  if (tile_rows != 128 || n_rows <= 0 || c_out <= 0 || K <= 0) return 0;
  if (c_out <= 32 && c_in <= 64) return x6p_ws_bytes(K, c_in, c_out);
  return x6_ws_bytes(n_rows, K, c_in, c_out, plan_x6(n_rows, c_out, 0, 0));
}

int msp_conv_tile(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                  const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                  const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                  msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_tile: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= 128, "msp_conv_tile: K must be in [1, 128] (got %d)", K);
  MSP_REQUIRE(tile_rows == 64 || tile_rows == 128 || tile_rows == 256,
              "msp_conv_tile: tile_rows must be 64, 128 or 256 (got %d)", tile_rows);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  MSP_REQUIRE(flip >= 0 && flip <= 3, "msp_conv_tile: flip must be 0..3 (got %d)", flip);
  MSP_REQUIRE(tile_rows == 128 || !(flip & 2),
              "msp_conv_tile: the [K][c_in][c_out] weight layout (flip bit 1) needs 128-row tiles");
  if (tile_rows == 64) {
    const int64_t n_tb = ceil_div(n_tiles, kWaves);
    const int NT = (c_out / 16) % 2 == 0 ? 2 : 1;
    const int n_y = c_out / (16 * NT);
    const unsigned grid = (unsigned)(n_tb * n_y);
    if (c_in >= 64 && NT == 2) {
      // block offset-major form over 4 per-wave tiles
      conv_tile4_kernel<2><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                                     chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
    } else if (c_in <= 64) {
#define LP(N, C)                                                                                              \
  if (NT == N && c_in == 16 * C)                                                                              \
    conv_tilep_kernel<N, C, 64><<<grid, kThreads, 0, s>>>(x, wt, K, flip, c_out, tile_start, chunk_off,      \
                                                          chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
      LP(1, 1) LP(1, 2) LP(1, 3) LP(1, 4) LP(2, 1) LP(2, 2) LP(2, 3) LP(2, 4)
#undef LP
    } else {
      conv_tile_kernel<1><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                                    chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
    }
    return check_launch("msp_conv_tile");
  }
  if (tile_rows == 256) {
    MSP_REQUIRE((c_out / 16) % 2 == 0, "msp_conv_tile: 256-row tiles need an even number of 16-channel groups");
    const int rc = launch_tile7((c_out / 16) % 4 == 0 ? 4 : 2, 256, 1, x, c_in, wt, K, flip, c_out, tile_start,
                                chunk_off, chunk_src, chunk_row, n_rows, out, nullptr, s);
    return rc ? rc : check_launch("msp_conv_tile");
  }
  if (c_out <= 32 && c_in <= 64) {
    // narrow outputs: per-wave 128-row tiles, no barriers (msp_conv_x6.hip)
    const size_t need = x6p_ws_bytes(K, c_in, c_out);
    MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_tile: workspace too small (%zu < %zu)", ws_bytes, need);
    // weights kept per offset run, chunk values three deep (scripts/kbench_x6.py,
    // profiles/r01/kbench_x6r_r01u.log)
    const int rc = launch_x6p(x, c_in, wt, K, flip, c_out, 128, tile_start, chunk_off, chunk_src, chunk_row,
                              n_rows, out, ws, s, 0, 3, 1);
    return rc ? rc : check_launch("msp_conv_tile");
  }
  // shared 128-row tiles on bf16 MFMA with exact operand splits (msp_conv_x6.hip)
  const PlanX6 p = plan_x6(n_rows, c_out, 0, 0);
  const size_t need = x6_ws_bytes(n_rows, K, c_in, c_out, p);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_tile: workspace too small (%zu < %zu)", ws_bytes, need);
  const int rc = launch_x6(p, x, c_in, wt, K, flip, c_out, tile_start, chunk_off, chunk_src, chunk_row, n_rows, out,
                           ws, s);
  return rc ? rc : check_launch("msp_conv_tile");
}

// Experiment hook (not part of the public ABI; scripts/kbench_conv.py): the
// conv_tile forms with parts of their data movement replaced by constants
// to find the limiter (64-row tiles).  abl 0-7: per-wave form (bits: 1 no
// gathers, 2 no weight loads, 4 no LDS accumulation); abl 16-23: block
// offset-major form (same bits, + 8: no per-step barrier -- wrong results,
// timing only); 32: block form with gathers one step ahead; 48: pipelined
// per-wave form (any tile_rows <= 128); 80 + s (s = 1..8): shared-tile form
// with an s-way offset split (ws = s*n_rows*c_out floats); 68-74:
// shared-tile ablations (bits of abl-67: 1 no barrier, 2 no gathers, 4 no
// LDS accumulation; tile_rows 128, nt 4).  nt forces NT.
int msp_debug_conv_tile(int abl, int nt, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                        int tile_rows, const int64_t* tile_start, const uint8_t* chunk_off,
                        const int32_t* chunk_src, const uint16_t* chunk_row, int64_t n_rows, float* out, float* ws,
                        msp_stream_t stream) {
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  const int NT = nt > 0 ? nt : pick_tile(c_out / 16);
  MSP_REQUIRE((c_out / 16) % NT == 0, "bad nt");
  const int n_y = c_out / (16 * NT);
  const unsigned grid = (unsigned)(ceil_div(n_tiles, kWaves) * n_y);
  hipStream_t s = as_stream(stream);
  if (abl > 80 && abl <= 88) {
    const int rc = launch_tile7(NT, tile_rows, abl - 80, x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                chunk_src, chunk_row, n_rows, out, ws, s);
    return rc ? rc : check_launch("msp_debug_conv_tile");
  }
  if (abl >= 68 && abl <= 74 && tile_rows == 128 && NT == 4) {
    const unsigned g7 = (unsigned)(ceil_div(n_rows, 128) * (c_out / 64));
#define A7(A)                                                                                                 \
  if (abl - 67 == A)                                                                                          \
    conv_tile7_kernel<4, 128, A><<<g7, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,  \
                                                         chunk_src, chunk_row, n_rows, c_out / 64, 1, out);
    A7(1) A7(2) A7(3) A7(4) A7(5) A7(6) A7(7)
#undef A7
    return check_launch("msp_debug_conv_tile");
  }
  if (abl == 48) {
    const int KC = c_in / 16;
    MSP_REQUIRE(c_in % 16 == 0 && KC <= 4 && tile_rows <= 128, "tilep: c_in / tile_rows");
#define LP(N, C, T)                                                                                         \
  if (NT == N && KC == C && tile_rows == T)                                                                 \
    conv_tilep_kernel<N, C, T><<<grid, kThreads, 0, s>>>(x, wt, K, flip, c_out, tile_start, chunk_off,      \
                                                         chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
    LP(1, 2, 64) LP(2, 2, 64) LP(2, 4, 64) LP(1, 2, 128) LP(2, 2, 128) LP(2, 4, 128)
#undef LP
    return check_launch("msp_debug_conv_tile");
  }
  MSP_REQUIRE(tile_rows == 64, "debug variants %d need 64-row tiles", abl);
#define L(N, A)                                                                                            \
  if (NT == N && abl == A)                                                                                 \
    conv_tile_kernel<N, A><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,   \
                                                     chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
#define LN(N) L(N, 0) L(N, 1) L(N, 2) L(N, 3) L(N, 4) L(N, 5) L(N, 6) L(N, 7)
  LN(1) LN(2) LN(4)
#define L4(N, A)                                                                                           \
  if (NT == N && abl == 16 + A)                                                                            \
    conv_tile4_kernel<N, A><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,  \
                                                      chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
  L4(2, 0) L4(2, 1) L4(2, 2) L4(2, 3) L4(2, 4) L4(2, 7) L4(2, 8) L4(2, 15)
#undef L4
  if (NT == 2 && abl == 32)
    conv_tile4_kernel<2, 0, true><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, flip, c_out, tile_start, chunk_off,
                                                            chunk_src, chunk_row, n_rows, n_tiles, n_y, out);
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

// Experiment hook (not part of the public ABI): 1 = weight gradients on the
// f32-MFMA kernel (conv_wgrad4_kernel) instead of the x6 one; the piece count
// stays the x6 plan's (callers size the slab from msp_wgrad_pieces).
static int g_wgrad_f32 = 0;
int msp_debug_wgrad_f32(int on) {
  g_wgrad_f32 = on;
  return MSP_OK;
}

// Experiment hook (not part of the public ABI): target block count of a
// weight-gradient launch (msp_wgrad_pieces); 0 = the default.
static int64_t g_wgrad_blocks = 0;
int msp_debug_wgrad_blocks(int64_t target) {
  g_wgrad_blocks = target;
  return MSP_OK;
}

int64_t msp_wgrad_pieces(int64_t total_pairs, int K, int c_in, int c_out) {
  // about 4096 blocks per launch (pieces x offsets x dW tiles), at least 256
  // pairs per piece; one-offset contractions (network-in-network weight
  // gradients) at most 768 pieces (fewer partial tiles to reduce)
  if (K < 1 || c_in < 16 || c_out < 16) return 1;
  int wa, wb;
  wgrad_x6_tile(c_in, c_out, wa, wb);
  const int64_t n_ty = (int64_t)(c_in / (16 * wa)) * (c_out / (16 * wb));
  int64_t n = total_pairs / ((int64_t)K * 256);
  const int64_t by_grid = (g_wgrad_blocks > 0 ? g_wgrad_blocks : 4096) / ((int64_t)K * n_ty);
  if (n > by_grid) n = by_grid;
  if (K == 1 && n > 768) n = 768;
  return n < 1 ? 1 : n;
}

// The banded form is correct (tests/test_gpu_ops.py::test_conv_wgrad_band) but
// measured 1.8-2.2x slower than the pair-list form (profiles/r01/
// kbench_wgrad_band_r01zz.log): 8-11 % of the pairs have their input row
// outside a 256-row band's +-64-row halo in key order (Morton neighbours
// jump), nearly every 32-pair step then waits on one un-prefetched global
// load.  Off unless msp_debug_wgrad_band(1).
static int g_wgrad_band_on = 0;
int msp_debug_wgrad_band(int on) {
  g_wgrad_band_on = on;
  return MSP_OK;
}

int msp_wgrad_band_ok(int64_t n_rows, int K, int c_in, int c_out) {
  if (!g_wgrad_band_on) return 0;
  return n_rows > 0 && K >= 1 && K <= 32 && c_in % 32 == 0 && c_out % 32 == 0 && c_in > 0 && c_out > 0 ? 1 : 0;
}

int64_t msp_wgrad_band_groups(int64_t n_rows, int c_in, int c_out) {
  if (n_rows <= 0 || c_in < 32 || c_out < 32) return 1;
  int S;
  return wgrad_band_groups(n_rows, c_in, c_out, S);
}

int64_t msp_wgrad_band_seg_len(int64_t n_rows, int K) {
  return (int64_t)K * (wgrad_band_n_sub(n_rows > 0 ? n_rows : 1) + 1);
}

int msp_wgrad_band_segments(const int32_t* pair_out, const int64_t* off_start, int K, int64_t n_rows, int64_t* seg,
                            msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && n_rows >= 0, "msp_wgrad_band_segments: bad arguments");
  if (n_rows == 0) return MSP_OK;
  launch_wgrad_band_seg(pair_out, off_start, K, n_rows, seg, as_stream(stream));
  return check_launch("msp_wgrad_band_segments");
}

int msp_conv_wgrad_band(const float* x, int c_in, const float* dy, int c_out, const int32_t* pair_in,
                        const int32_t* pair_out, const int64_t* seg, int K, int64_t n_rows, float* slab, float* dw,
                        msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= 32 && c_in % 32 == 0 && c_out % 32 == 0 && c_in > 0 && c_out > 0,
              "msp_conv_wgrad_band: needs K <= 32 and channels in multiples of 32 (K=%d c_in=%d c_out=%d)", K, c_in,
              c_out);
  hipStream_t s = as_stream(stream);
  const int64_t cc = (int64_t)c_in * c_out;
  if (n_rows <= 0) {
    MSP_HIP(hipMemsetAsync(dw, 0, (size_t)K * cc * sizeof(float), s), "msp_conv_wgrad_band");
    return MSP_OK;
  }
  int S;
  const int64_t n_groups = wgrad_band_groups(n_rows, c_in, c_out, S);
  MSP_REQUIRE(launch_wgrad_band(x, c_in, dy, c_out, pair_in, pair_out, seg, K, n_rows, n_groups, S, slab, s) ==
                  MSP_OK,
              "msp_conv_wgrad_band: no kernel for K=%d", K);
  dim3 g2((unsigned)ceil_div(cc, 64), (unsigned)K);
  wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, n_groups, K, cc, dw);
  return check_launch("msp_conv_wgrad_band");
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
  if (!g_wgrad_f32) {  // bf16 MFMA on exact operand splits (msp_conv_x6.hip)
    MSP_REQUIRE(launch_wgrad_x6(x, c_in, dy, c_out, pair_in, pair_out, off_start, K, n_pieces, slab, s) == MSP_OK,
                "msp_conv_wgrad: no x6 kernel for c_in=%d c_out=%d", c_in, c_out);
    wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, n_pieces, K, cc, dw);
    return check_launch("msp_conv_wgrad");
  }
  // f32-MFMA form (msp_debug_wgrad_f32): dW tiles of up to 64 x 64 per
  // block, the largest divisor <= 4 of the 16-channel group counts
  auto pick = [](int n16) { return n16 % 4 == 0 ? 4 : (n16 % 3 == 0 ? 3 : (n16 % 2 == 0 ? 2 : 1)); };
  const int WA = pick(c_in / 16), WB = pick(c_out / 16);
  const int n_ty = (c_in / (16 * WA)) * (c_out / (16 * WB));
  const unsigned grid = (unsigned)(n_pieces * K * n_ty);
#define LAUNCH(A, B)                                                                                         \
  if (WA == A && WB == B)                                                                                    \
    conv_wgrad4_kernel<A, B><<<grid, kThreads, 0, s>>>(x, c_in, dy, c_out, pair_in, pair_out, off_start, K, \
                                                       n_pieces, n_ty, slab);
#define LAUNCH_ROW(A) LAUNCH(A, 1) LAUNCH(A, 2) LAUNCH(A, 3) LAUNCH(A, 4)
  LAUNCH_ROW(1) LAUNCH_ROW(2) LAUNCH_ROW(3) LAUNCH_ROW(4)
#undef LAUNCH_ROW
#undef LAUNCH
  wgrad_reduce_kernel<<<g2, 256, 0, s>>>(slab, n_pieces, K, cc, dw);
  return check_launch("msp_conv_wgrad");
}

}  // extern "C"
