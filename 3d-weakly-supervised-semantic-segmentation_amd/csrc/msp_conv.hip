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

// Runs of chunks (MSP_PAIRS_RUN): one wave takes `run` consecutive chunks.  The chunks are offset-major, so a run
// stays in one offset except where it crosses into the next; the offset's weight block (c_in / 16 <= KMAX k-steps
// of NT 16-column groups) is loaded into registers once per run and reloaded only at such a crossing, instead of
// once per 16 pairs (conv_pairs_kernel reads 2x the bytes of the x rows it multiplies in weights at level 0).
// The next chunk's pair indices are loaded while the current chunk's x rows are in flight.  Per chunk the
// arithmetic is conv_pairs_kernel's, in the same order: the outputs are bit-identical.
template <int NT, int KMAX>
__global__ __launch_bounds__(kThreads) void conv_pairs_run_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ chunk_start, int64_t n_chunks, int run, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t ch0 = ((int64_t)blockIdx.x * kWaves + wave) * run;
  if (ch0 >= n_chunks) return;
  const int64_t ch1 = ch0 + run < n_chunks ? ch0 + run : n_chunks;
  const int c0 = blockIdx.y * NC;
  const int r = lane & 15, q = lane >> 4;
  const int kcn = c_in >> 4;
  // offset walk of the index loads (wave-uniform; empty offsets have equal chunk starts)
  int oi = find_offset(chunk_start, K, ch0);
  int64_t oi_first = chunk_start[oi], oi_end = chunk_start[oi + 1], pb = off_start[oi], pe = off_start[oi + 1];
  auto indices = [&](int64_t ch, int& src, int (&dst)[4], int& o_of) {
    if (ch >= oi_end) {
      do {
        ++oi;
        oi_end = chunk_start[oi + 1];
      } while (ch >= oi_end);
      oi_first = chunk_start[oi];
      pb = off_start[oi];
      pe = off_start[oi + 1];
    }
    const int64_t p0 = pb + (ch - oi_first) * MSP_CHUNK;
    src = p0 + r < pe ? pin[p0 + r] : -1;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = p0 + 4 * q + j < pe ? pout[p0 + 4 * q + j] : -1;
    o_of = oi;
  };
  floatx4 b[KMAX][NT];
  int ow = -1;  // the offset whose weights are in b
  int src, dst[4], o;
  indices(ch0, src, dst, o);
  for (int64_t ch = ch0; ch < ch1; ++ch) {
    if (o != ow) {
      ow = o;
      const float* wb = wt + ((int64_t)o * c_out + c0 + r) * c_in + 4 * q;
#pragma unroll
      for (int kc = 0; kc < KMAX; ++kc)
        if (kc < kcn) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
            b[kc][t] = *reinterpret_cast<const floatx4*>(wb + (int64_t)t * 16 * c_in + kc * 16);
        }
    }
    const float* xs = x + (int64_t)(src < 0 ? 0 : src) * c_in + 4 * q;
    floatx4 a[KMAX];
#pragma unroll
    for (int kc = 0; kc < KMAX; ++kc)
      if (kc < kcn) {
        a[kc] = *reinterpret_cast<const floatx4*>(xs + kc * 16);
        if (src < 0) a[kc] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    int dcur[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) dcur[j] = dst[j];
    if (ch + 1 < ch1) indices(ch + 1, src, dst, o);
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KMAX; ++kc)
      if (kc < kcn) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[kc][s], b[kc][t][s], acc[t]);
        }
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (dcur[j] >= 0) {
        float* d = out + (int64_t)dcur[j] * c_out + c0 + r;
#pragma unroll
        for (int t = 0; t < NT; ++t) d[t * 16] = acc[t][j];
      }
    }
  }
}

// MSP_PAIRS_DEPTH 2: conv_pairs_run_kernel with the next chunk's x rows loaded as well (and the indices two chunks
// ahead) while the current chunk's MFMAs and stores run.
template <int NT, int KMAX>
__global__ __launch_bounds__(kThreads) void conv_pairs_pipe_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ wt, int K, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ chunk_start, int64_t n_chunks, int run, float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t ch0 = ((int64_t)blockIdx.x * kWaves + wave) * run;
  if (ch0 >= n_chunks) return;
  const int64_t ch1 = ch0 + run < n_chunks ? ch0 + run : n_chunks;
  const int c0 = blockIdx.y * NC;
  const int r = lane & 15, q = lane >> 4;
  const int kcn = c_in >> 4;
  int oi = find_offset(chunk_start, K, ch0);
  int64_t oi_first = chunk_start[oi], oi_end = chunk_start[oi + 1], pb = off_start[oi], pe = off_start[oi + 1];
  auto indices = [&](int64_t ch, int& src, int (&dst)[4], int& o_of) {
    if (ch >= oi_end) {
      do {
        ++oi;
        oi_end = chunk_start[oi + 1];
      } while (ch >= oi_end);
      oi_first = chunk_start[oi];
      pb = off_start[oi];
      pe = off_start[oi + 1];
    }
    const int64_t p0 = pb + (ch - oi_first) * MSP_CHUNK;
    src = p0 + r < pe ? pin[p0 + r] : -1;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = p0 + 4 * q + j < pe ? pout[p0 + 4 * q + j] : -1;
    o_of = oi;
  };
  auto load_x = [&](int src, floatx4 (&a)[KMAX]) {
    const float* xs = x + (int64_t)(src < 0 ? 0 : src) * c_in + 4 * q;
#pragma unroll
    for (int kc = 0; kc < KMAX; ++kc)
      if (kc < kcn) a[kc] = *reinterpret_cast<const floatx4*>(xs + kc * 16);
  };
  floatx4 b[KMAX][NT];
  int ow = -1;
  // chunk ch: a / s_c / d_c / o_c; chunk ch + 1: indices s_n / d_n / o_n (its x rows are loaded in the body)
  int s_c, d_c[4], o_c, s_n = -1, d_n[4] = {-1, -1, -1, -1}, o_n = 0;
  floatx4 a[KMAX];
  indices(ch0, s_c, d_c, o_c);
  load_x(s_c, a);
  if (ch0 + 1 < ch1) indices(ch0 + 1, s_n, d_n, o_n);
  for (int64_t ch = ch0; ch < ch1; ++ch) {
    if (o_c != ow) {
      ow = o_c;
      const float* wb = wt + ((int64_t)o_c * c_out + c0 + r) * c_in + 4 * q;
#pragma unroll
      for (int kc = 0; kc < KMAX; ++kc)
        if (kc < kcn) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
            b[kc][t] = *reinterpret_cast<const floatx4*>(wb + (int64_t)t * 16 * c_in + kc * 16);
        }
    }
    const bool more = ch + 1 < ch1;
    floatx4 an[KMAX];
    if (more) load_x(s_n, an);
    int s2 = -1, d2[4] = {-1, -1, -1, -1}, o2 = o_n;
    if (ch + 2 < ch1) indices(ch + 2, s2, d2, o2);
    if (s_c < 0) {
#pragma unroll
      for (int kc = 0; kc < KMAX; ++kc) a[kc] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KMAX; ++kc)
      if (kc < kcn) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[kc][s], b[kc][t][s], acc[t]);
        }
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (d_c[j] >= 0) {
        float* d = out + (int64_t)d_c[j] * c_out + c0 + r;
#pragma unroll
        for (int t = 0; t < NT; ++t) d[t * 16] = acc[t][j];
      }
    }
    if (more) {
#pragma unroll
      for (int kc = 0; kc < KMAX; ++kc) a[kc] = an[kc];
      s_c = s_n;
      o_c = o_n;
#pragma unroll
      for (int j = 0; j < 4; ++j) d_c[j] = d_n[j];
      s_n = s2;
      o_n = o2;
#pragma unroll
      for (int j = 0; j < 4; ++j) d_n[j] = d2[j];
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
// the headline batch, ~6 TF/s algorithmic) and its weight gradient the pair lists at 0.29 ms.
//
// Forward: one lane per output row.  The lane gathers its 27 neighbour indices (coalesced over the wave's 64
// rows) and their CIN-channel input rows (one dwordx3 per neighbour for CIN = 3), and accumulates all COUT
// outputs in registers from weights held in SGPRs (uniform scalar loads: every lane needs the same weight),
// so the contraction is 27 CIN COUT v_fma_f32 with a scalar operand per row and nothing else; exact fp32
// products, offsets then channels in order.
template <int CIN>
struct RowIn {
  float v[CIN];
};

template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_narrow_in_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                             int K, const int32_t* __restrict__ nbr, int64_t n,
                                                             float* __restrict__ out) {
  const RowIn<CIN>* xr = reinterpret_cast<const RowIn<CIN>*>(x);
  auto ld = [&](int32_t i) {  // the neighbour's input row (zero where absent)
    RowIn<CIN> v = xr[i < 0 ? 0 : i];
#pragma unroll
    for (int k = 0; k < CIN; ++k) v.v[k] = i < 0 ? 0.f : v.v[k];
    return v;
  };
  for (int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x; row < n; row += (int64_t)gridDim.x * 256) {
    float acc[COUT];
#pragma unroll
    for (int c = 0; c < COUT; ++c) acc[c] = 0.f;
    // offsets in a rolled loop (the weights of one offset, CIN COUT of them, are its scalar operands): indices
    // two offsets ahead, input rows one ahead
    int32_t i1 = K > 1 ? nbr[n + row] : -1;
    RowIn<CIN> v0 = ld(nbr[row]);
    for (int o = 0; o < K; ++o) {
      const int32_t i2 = o + 2 < K ? nbr[(o + 2) * n + row] : -1;
      const RowIn<CIN> v1 = ld(i1);
      const float* w = wt + o * CIN * COUT;
#pragma unroll
      for (int k = 0; k < CIN; ++k)
#pragma unroll
        for (int c = 0; c < COUT; ++c) acc[c] = fmaf(v0.v[k], w[k * COUT + c], acc[c]);
      v0 = v1;
      i1 = i2;
    }
    floatx4* dst = reinterpret_cast<floatx4*>(out + row * COUT);
#pragma unroll
    for (int c = 0; c < COUT / 4; ++c) dst[c] = floatx4{acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]};
  }
}

// Weight gradient: dW^T[c][(o, k)] = sum over rows i of dy[i][c] X[i][(o, k)], X[i][(o, k)] = x[nbr(o, i)][k]
// (0 where absent) -- a dense [COUT x rows] x [rows x 27 CIN] product with the rows as the contraction, on
// v_mfma_f32_16x16x4_f32 (k = 4 rows).  Per 16-row batch a wave gathers X into its LDS tile (4 lanes per row,
// 7 offsets each; columns past 27 CIN stay zero), its dy fragments for the batch's 4 k-steps are loaded from
// global memory alongside (16 lanes read 64 contiguous bytes of one row); the block's 4 waves take batches
// round-robin over a contiguous row range and their tiles are added in wave order into the block's slab
// (wgrad_reduce_kernel adds the blocks in order: deterministic).
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void wgrad_narrow_in_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ dy, int K,
                                                              const int32_t* __restrict__ nbr, int64_t n,
                                                              int64_t n_parts, float* __restrict__ slab) {
  constexpr int KM = 27, KC = KM * CIN, NU = (KC + 15) / 16, NCOL = 16 * NU, MT = COUT / 16, BR = 16;
  constexpr int OQ = (KM + 3) / 4;  // offsets per gathering lane
  __shared__ float xl[4][BR][NCOL + 1];  // +1: the rows a ds_write_b32 spans land on distinct banks
  __shared__ float red[KC * COUT];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const RowIn<CIN>* xr = reinterpret_cast<const RowIn<CIN>*>(x);
  for (int i = lane; i < BR * (NCOL + 1); i += 64) (&xl[wave][0][0])[i] = 0.f;
  const int64_t r0 = n * blockIdx.x / n_parts, r1 = n * (blockIdx.x + 1) / n_parts;
  floatx4 acc[MT][NU];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[t][u] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int gr = lane & 15, oq = lane >> 4;  // gather: row of the batch, offset quarter
  for (int64_t b0 = r0 + (int64_t)BR * wave; b0 < r1; b0 += 4 * BR) {
    const int64_t grow = b0 + gr;
    int32_t nb[OQ];
#pragma unroll
    for (int j = 0; j < OQ; ++j) {
      const int o = oq * OQ + j;
      nb[j] = (o < K && o < KM && grow < r1) ? nbr[o * n + grow] : -1;
    }
    float a[BR / 4][MT];  // dy fragments of the batch's k-steps, in flight with the gather
#pragma unroll
    for (int j = 0; j < BR / 4; ++j) {
      const int64_t row = b0 + 4 * j + q;
#pragma unroll
      for (int t = 0; t < MT; ++t) a[j][t] = row < r1 ? dy[row * COUT + 16 * t + r] : 0.f;
    }
    RowIn<CIN> v[OQ];
#pragma unroll
    for (int j = 0; j < OQ; ++j) v[j] = xr[nb[j] < 0 ? 0 : nb[j]];
#pragma unroll
    for (int j = 0; j < OQ; ++j) {
      const int o = oq * OQ + j;
      if (o < KM)
#pragma unroll
        for (int k = 0; k < CIN; ++k) xl[wave][gr][o * CIN + k] = nb[j] < 0 ? 0.f : v[j].v[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < BR / 4; ++j) {
      float bv[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) bv[u] = xl[wave][4 * j + q][16 * u + r];
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int u = 0; u < NU; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][t], bv[u], acc[t][u], 0, 0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the tile's reads are done before the next batch's gather overwrites it
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // lane (r, q) register jj of tile (t, u): dW[(o, k) = 16 u + r][c = 16 t + 4 q + jj]; waves added in order
  for (int w = 0; w < 4; ++w) {
    if (wave == w)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int ok = 16 * u + r;
          if (ok < KC)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              float& e = red[ok * COUT + 16 * t + 4 * q + jj];
              e = w == 0 ? acc[t][u][jj] : e + acc[t][u][jj];
            }
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

// Per-wave tiles (x6r) for narrow outputs, and since round 5 for level 0's 32 -> 64 too (two 32-column passes
// over the gathers, n_y = 2) instead of the shared tiles (x6d: mfma_busy 0.15 there, 0.83 ms per call): 49.73-49.81
// vs 50.07-50.11 ms/step (profiles/r05/ab_r05am_x6r_wide.log).  MSP_X6R_WIDE 0: the round-4 choice.
#ifndef MSP_X6R_WIDE
#define MSP_X6R_WIDE 1
#endif
static bool use_x6r(int64_t n_rows, int c_in, int c_out) {
  return (c_out <= 32 && c_in <= 64) || (MSP_X6R_WIDE && c_out == 64 && c_in <= 32 && n_rows >= 100000);
}

int msp_conv_tile_form(int64_t n_rows, int c_in, int c_out, int tile_rows) {
  if (n_rows <= 0 || c_in <= 0 || c_out <= 0 || tile_rows != 128) return 0;
  return use_x6r(n_rows, c_in, c_out) ? 1 : 2;
}

size_t msp_conv_tile_workspace_size(int64_t n_rows, int K, int c_in, int c_out, int tile_rows) {
  if (tile_rows != 128 || n_rows <= 0 || c_out <= 0 || K <= 0) return 0;
  if (use_x6r(n_rows, c_in, c_out)) return x6p_ws_bytes(K, c_in, c_out);
  return x6_ws_bytes(n_rows, K, c_in, c_out, plan_x6(n_rows, c_out));
}

int msp_conv_tile(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                  const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                  const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                  msp_stream_t stream) {
  return msp_conv_tile_bn(x, c_in, wt, K, flip, c_out, tile_rows, tile_start, chunk_off, chunk_src, chunk_row,
                          n_rows, out, ws, ws_bytes, nullptr, stream);
}

int64_t msp_conv_bn_parts(int64_t n_rows) { return n_rows > 0 ? ceil_div(n_rows, 128) : 0; }

int msp_conv_tile_bn(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                     const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                     const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                     const msp_bn_epilogue* epi, msp_stream_t stream) {
  MSP_REQUIRE(epi == nullptr || (epi->partial != nullptr && (epi->x == nullptr || epi->stats != nullptr)),
              "msp_conv_tile_bn: epilogue without a partial buffer (or a backward one without stats)");
  MSP_REQUIRE(epi == nullptr || n_rows <= 0 || msp_conv_tile_form(n_rows, c_in, c_out, tile_rows) == 1,
              "msp_conv_tile_bn: the BatchNorm epilogue needs the per-wave form (msp_conv_tile_form 1)");
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_tile: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= 128, "msp_conv_tile: K must be in [1, 128] (got %d)", K);
  MSP_REQUIRE(tile_rows == 128, "msp_conv_tile: tile_rows must be 128 (got %d)", tile_rows);
  MSP_REQUIRE(flip >= 0 && flip <= 7, "msp_conv_tile: flip must be 0..7 (got %d)", flip);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  if (use_x6r(n_rows, c_in, c_out)) {
    // narrow outputs: per-wave 128-row tiles, no barriers (msp_conv_x6.hip)
    const size_t need = x6p_ws_bytes(K, c_in, c_out);
    MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_tile: workspace too small (%zu < %zu)", ws_bytes, need);
    const int rc = launch_x6r(x, c_in, wt, K, flip, c_out, tile_start, chunk_off, chunk_src, chunk_row, n_rows, out,
                              ws, s, epi);
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

// Runs of chunks with the weights in registers where c_in <= 64; MSP_PAIRS_RUN 0: one chunk per wave, weights
// re-read per chunk (the round-4 form).  Level 0 of the headline batch (64 -> 32, 1.30 M pairs): 148.8 us in the
// one-chunk form, 137.6 with runs (MSP_PAIRS_DEPTH 1: indices one chunk ahead), 123.5 with the x rows one chunk
// ahead as well (MSP_PAIRS_DEPTH 2); 4096 waves instead of 8192: 133.1 (profiles/r05/kb_pairs_r05b.log).  Without
// any prefetch the runs were slower than the one-chunk form (163 vs 150 us).
#ifndef MSP_PAIRS_RUN
#define MSP_PAIRS_RUN 1
#endif
#ifndef MSP_PAIRS_WAVES
#define MSP_PAIRS_WAVES 8192
#endif
#ifndef MSP_PAIRS_DEPTH
#define MSP_PAIRS_DEPTH 2
#endif

int msp_conv_pairs(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* pair_in,
                   const int32_t* pair_out, const int64_t* off_start, const int64_t* chunk_start,
                   int64_t n_chunks, float* out, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_pairs: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  if (n_chunks == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  const int kcn = c_in / 16, n16 = c_out / 16;
  if (MSP_PAIRS_RUN && kcn <= 4) {
    // weights in registers (c_in <= 64); wider inputs keep the one-chunk form, which measured faster there (the
    // weight registers cost occupancy and narrower column groups re-read x: profiles/r05/kb_pairs_r05*.log)
    const int NT = pick_tile(n16), ny = n16 / NT;
    // about MSP_PAIRS_WAVES waves over the grid: runs long enough to amortise the weights, enough waves to fill
    // the chip
    int64_t run = n_chunks * ny / MSP_PAIRS_WAVES;
    run = run < 1 ? 1 : run > 16 ? 16 : run;
    const int64_t waves = ceil_div(n_chunks, run);
    dim3 grid((unsigned)ceil_div(waves, kWaves), (unsigned)ny);
#define LAUNCH_RUN(N)                                                                                          \
  if (MSP_PAIRS_DEPTH == 2)                                                                                    \
    conv_pairs_pipe_kernel<N, 4><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, c_out, pair_in, pair_out, off_start, \
                                                           chunk_start, n_chunks, (int)run, out);              \
  else                                                                                                         \
    conv_pairs_run_kernel<N, 4><<<grid, kThreads, 0, s>>>(x, c_in, wt, K, c_out, pair_in, pair_out, off_start,  \
                                                          chunk_start, n_chunks, (int)run, out)
    switch (NT) {
      case 1: LAUNCH_RUN(1); break;
      case 2: LAUNCH_RUN(2); break;
      case 3: LAUNCH_RUN(3); break;
      default: LAUNCH_RUN(4); break;
    }
#undef LAUNCH_RUN
    return check_launch("msp_conv_pairs");
  }
  const int NT = pick_tile(n16);
  dim3 grid((unsigned)ceil_div(n_chunks, kWaves), (unsigned)(c_out / (16 * NT)));
#define LAUNCH(N)                                                                                     \
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
  int64_t grid = ceil_div(n_rows, 256);
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
  // blocks of at least 4 batches of 16 rows per wave, at most 1024 (4 per CU: 36 KiB of LDS each)
  const int64_t p = ceil_div(n_rows > 0 ? n_rows : 1, 256);
  return p < 1 ? 1 : (p > 1024 ? 1024 : p);
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
