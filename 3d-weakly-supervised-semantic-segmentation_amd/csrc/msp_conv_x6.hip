// Shared-tile gather convolution on bf16 MFMA with exact three-piece operand
// splits ("x6" form of msp_conv_tile).
//
// gfx950 has no xf32 MFMA: its f32-input MFMA runs at the fp32 vector rate,
// 1/16 of v_mfma_f32_16x16x32_bf16.  Every fp32 operand v is written exactly
// as v = v0 + v1 + v2 with bf16 pieces (v0 = RNE(v), v1 = RNE(v - v0),
// v2 = v - v0 - v1: each residual is exact in fp32 and the last one has at
// most 7 significant bits, so it is exact in bf16).  The product w*x is then
// the sum of the nine piece products, each exact in the fp32 accumulator; the
// six with i + j <= 2 are computed (w0x0 w0x1 w1x0 w0x2 w1x1 w2x0) and the
// three dropped ones are bounded by |w1 x2| + |w2 x1| + |w2 x2| <~ 2^-23 |wx|
// (|v1| <= 2^-8 |v|, |v2| <= 2^-16 |v|): about one fp32 rounding of the product.  Six bf16 MFMAs (16 cycles
// each) replace eight f32 MFMAs of 32 cycles per 32-deep k-step: 2.7x fewer
// matrix-core cycles at fp32-class accuracy (tests/test_gpu_ops.py checks the
// error against an fp64 reference next to the f32-MFMA path's).
//
// Weights are split once per call by split_weights_kernel into the exact
// LDS images of the steps, [K][c_out / NC][k-slices][3][KS/8][NC] 16-byte
// units of 8 k (XOR swizzle applied, zero padded past c_in), so a step's
// staging is a straight coalesced copy; the gathered input rows are split in
// registers (4.5 VALU per value: v_cvt_pk_bf16_f32, shift/and back to fp32,
// v_pk_add_f32).
//
// Structure as conv_tile7 (msp_conv.hip): block = 4 waves sharing one
// 128-row output tile accumulated in LDS, steps over (offset, KS-deep k-slice)
// with the weight slice staged in LDS (double buffered, one barrier per step),
// chunks dealt round-robin to the waves, software pipelined with alternating
// register sets and branch-free clamped loads.
//
// MFMA operand maps (16x16x32 bf16, run transposed: D = W^T X^T): lane
// (r = l & 15, q = l >> 4) supplies A = W^T[out 16t + r][k 8q .. 8q+7] and
// B = X^T[k 8q .. 8q+7][chunk row r]; D[out 16t + 4q + j][chunk row r] lands in
// register j, the accumulator layout of the f32 kernels.
#include "msp_x6.h"
#include "msp_bn_epi.h"

#include <cstdlib>

namespace msp {

// wt [K][c_out][c_in] fp32 -> the per-step LDS images of conv_x6d_kernel:
// unit u = (p * K8 + k8) * NC + n of image (o, cy, ks) holds piece p of
// wt[o][cy * NC + n][ks * KS + 8 k8 .. + 7] (zero past c_in).  Unswizzled:
// the staging copy is linear, and the fragment reads (lane (r, q) reads unit
// row k8 = 4kk + q, column 16t + r) put the 16 lanes of each ds_read_b128 lane
// group ({0-3,12-15,20-27}, ... -- MI355X_MICROARCH.md LDS table) on 16
// distinct bank quads (r of q covers 0-3 and 12-15, r of q+1 covers 4-11).
// One thread per unit.
// wlay 1: wt given as [K][c_in][c_out] (the module's own layout; no transposed copy).
__global__ __launch_bounds__(256) void split_weights_kernel(const float* __restrict__ wt, int K, int c_out, int c_in,
                                                            int NC, int KS, u32x4* __restrict__ img, int wlay = 0) {
  split_weights_unit(wt, K, c_out, c_in, NC, KS, img, wlay, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// D-deep pipelined form.  A step is one (offset, KS-deep k-slice); with the
// bf16 MFMAs a step is short (a wave averages about one chunk per offset of
// a 128-row tile), so one step of lead time does not hide L2 latency.  D
// register slots rotate: slot k = s % D holds the gathered rows, tile rows
// and chunk sources of step s + D, s + D and s + 2D once step s has used it,
// and the weight staging registers of step s + 1 + D.  Per step, in order:
//   barrier | MFMAs(s) | LDS RMW(s) | weights(s+1) regs -> LDS |
//   weights(s+1+D) load | rows + gathers(s+D) | sources(s+2D)
// so every load has D steps to land.  Step descriptors come from a packed
// per-offset table in LDS (one read per step, for step s + 2D).
// ABL (timing experiments only, wrong results): bit 1 no barrier, 2 no
// gathers, 4 no LDS accumulation, 8 no weight staging, 16 no split, 32 no MFMA.
// NB = weight slice buffers: 2 (one barrier per step) or 1 (a second barrier
// before the slice is overwritten; 12 KiB less LDS -> 3 blocks per CU).
template <int NT, int KS, int D, int TR, int ABL = 0, int NB = 2>
__global__ __launch_bounds__(kThreads) void conv_x6d_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows, int n_y,
    int n_split, float* __restrict__ out) {
  static_assert(D >= 2, "the weight slot of step s+1 must differ from step s's");
  constexpr int NC = 16 * NT;
  constexpr int K8 = KS / 8;
  constexpr int NKK = KS / 32;
  constexpr int WU = 3 * K8 * NC;
  constexpr int SPT = (WU + kThreads - 1) / kThreads;
  constexpr int MJ = TR / (16 * kWaves);
  __shared__ floatx4 acc4[TR * NC / 4];
  __shared__ u32x4 wbuf[NB][WU];
  __shared__ unsigned long long need[2];
  __shared__ int gfirst[128];
  __shared__ int gcount[128];
  __shared__ int dtab[128];

  // wave id through readfirstlane: the compiler then knows it is uniform and
  // branches on per-wave chunk counts become scalar branches
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
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
    if (c == cb || chunk_off[c - 1] != o) {
      gfirst[o] = (int)(c - cb);
      atomicOr(&need[o >> 6], 1ull << (o & 63));
    }
    atomicAdd(&gcount[o], 1);
  }
  __syncthreads();
  if (tid < 128) {  // dtab[i] = i-th needed offset o | first chunk << 8 | chunk count << 20
    const unsigned long long m0 = need[0], m1 = need[1];
    const bool has = tid < 64 ? ((m0 >> tid) & 1ull) : ((m1 >> (tid - 64)) & 1ull);
    const int below = tid < 64 ? __popcll(m0 & ((1ull << tid) - 1ull))
                               : __popcll(m0) + __popcll(m1 & ((1ull << (tid - 64)) - 1ull));
    if (has) dtab[below] = tid | (gfirst[tid] << 8) | (gcount[tid] << 20);
  }
  auto uniform64 = [](unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
  };
  const int n_off_all = __popcll(uniform64(need[0])) + __popcll(uniform64(need[1]));
  const int oi0 = sp * n_off_all / n_split;
  const int n_off = (sp + 1) * n_off_all / n_split - oi0;
  __syncthreads();
  const int nks = (c_in + KS - 1) / KS;
  const int n_steps = n_off * nks;
  if (n_steps == 0) {
    const int64_t row0 = tile * TR;
    const int nr = (int)((n_rows - row0) < TR ? (n_rows - row0) : TR);
    for (int i = tid; i < nr * NC / 4; i += kThreads)
      *reinterpret_cast<floatx4*>(dst + (row0 + i / (NC / 4)) * c_out + c0 + 4 * (i % (NC / 4))) =
          floatx4{0.f, 0.f, 0.f, 0.f};
    return;
  }

  struct Step {
    int ks, o, l0, cnt, gn;
  };
  // frontier (oi, ks) of the next descriptor to make; past the last step
  // the last offset repeats (loads stay in range) with gn = 0
  int foi = 0, fks = 0;
  auto next_desc = [&]() {
    Step d;
    const bool live = foi < n_off;
    const int pkd = __builtin_amdgcn_readfirstlane(dtab[oi0 + (live ? foi : n_off - 1)]);
    d.o = pkd & 255;
    d.l0 = (pkd >> 8) & 4095;
    d.cnt = pkd >> 20;
    d.ks = fks;
    const int gn = (d.cnt - wave + kWaves - 1) / kWaves;
    d.gn = !live || gn < 0 ? 0 : (gn > MJ ? MJ : gn);
    if (++fks == nks) {
      fks = 0;
      ++foi;
    }
    return d;
  };
  // chunk arrays of this tile: uniform base, per-step uniform chunk index
  const int32_t* csrc_t = chunk_src + cb * MSP_CHUNK;
  const uint16_t* crow_t = chunk_row + cb * MSP_CHUNK;
  auto chunk_idx = [&](const Step& d, int j) {  // uniform
    const int l = wave + kWaves * j;
    return (d.l0 + (l < d.cnt ? l : 0)) * MSP_CHUNK;
  };
  struct Src {
    int32_t v[MJ];
  };
  struct Row {
    int v[MJ];
  };
  struct Val {
    floatx4 a[MJ][NKK][2];
  };
  struct WSt {
    u32x4 u[SPT];
  };
  auto ld_src = [&](const Step& sd, Src& d) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) d.v[j] = (csrc_t + chunk_idx(sd, j))[r];
  };
  auto ld_row = [&](const Step& sd, Row& d) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) d.v[j] = (crow_t + chunk_idx(sd, j))[r];
  };
  // weight staging: a step's slice is one contiguous image (split_weights_
  // kernel), copied unit for unit (coalesced loads, linear LDS stores)
  const int n_y_w = c_out / NC;
  const u32x4* wimg_c = wimg + (int64_t)(c0 / NC) * nks * WU;
  auto ld_w = [&](const Step& sd, WSt& w) {
    const int ow = flip ? (K - 1 - sd.o) : sd.o;
    const u32x4* wb = wimg_c + ((int64_t)ow * n_y_w * nks + sd.ks) * WU;
#pragma unroll
    for (int i = 0; i < SPT; ++i) w.u[i] = wb[(tid + kThreads * i) < WU ? tid + kThreads * i : WU - 1];
  };
  auto st_w = [&](const WSt& w, int buf) {
#pragma unroll
    for (int i = 0; i < SPT; ++i)
      if (tid + kThreads * i < WU) wbuf[buf][tid + kThreads * i] = w.u[i];
  };
  const char* xb = reinterpret_cast<const char*>(x);
  const uint32_t row_bytes = (uint32_t)c_in * 4u;
  auto gather = [&](const Step& sd, const Src& sv, Val& v) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const uint32_t ro = (uint32_t)sv.v[j] * row_bytes;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const int k = min(sd.ks * KS + kk * 32 + 8 * q, c_in - 8);
        const floatx4* pv = reinterpret_cast<const floatx4*>(xb + (ro + 4u * (uint32_t)k));
        if (ABL & 2) {
          v.a[j][kk][0] = floatx4{(float)sv.v[j], (float)k, 1.f, 2.f};
          v.a[j][kk][1] = floatx4{(float)k, (float)sv.v[j], 3.f, 4.f};
        } else {
          v.a[j][kk][0] = pv[0];
          v.a[j][kk][1] = pv[1];
        }
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
    const u32x4* wb = wbuf[buf];
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if (sd.ks * KS + kk * 32 < c_in) {
        u32x4 xp[MJ][3];
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          if (j < sd.gn) {
            if (ABL & 16) {
#pragma unroll
              for (int pp = 0; pp < 3; ++pp)
                xp[j][pp] = u32x4{__float_as_uint(v.a[j][kk][0][pp]), __float_as_uint(v.a[j][kk][0][pp + 1]),
                                  __float_as_uint(v.a[j][kk][1][pp]), __float_as_uint(v.a[j][kk][1][pp + 1])};
            } else {
              split8(v.a[j][kk][0], v.a[j][kk][1], xp[j]);
            }
          }
        const int k8 = kk * 4 + q;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int un = 16 * t + r;
          const u32x4 w0 = wb[(0 * K8 + k8) * NC + un];
          const u32x4 w1 = wb[(1 * K8 + k8) * NC + un];
          const u32x4 w2 = wb[(2 * K8 + k8) * NC + un];
#pragma unroll
          for (int j = 0; j < MJ; ++j) {
            if (j < sd.gn && (ABL & 32)) {
              acc[j][t] += __builtin_bit_cast(floatx4, w0 ^ w1 ^ w2 ^ xp[j][0] ^ xp[j][1] ^ xp[j][2]);
            } else if (j < sd.gn) {
              floatx4 a = acc[j][t];
              a = mfma_bf16(w2, xp[j][0], a);
              a = mfma_bf16(w1, xp[j][1], a);
              a = mfma_bf16(w0, xp[j][2], a);
              a = mfma_bf16(w1, xp[j][0], a);
              a = mfma_bf16(w0, xp[j][1], a);
              acc[j][t] = mfma_bf16(w0, xp[j][0], a);
            }
          }
        }
      }
    }
  };
  auto consume_val = [&](const Val& v) {
#pragma unroll
    for (int j = 0; j < MJ; ++j)
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) asm volatile("" ::"v"(v.a[j][kk][0]), "v"(v.a[j][kk][1]));
  };
  auto consume_row = [&](const Row& rw) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) asm volatile("" ::"v"(rw.v[j]));
  };
  auto rmw = [&](const Step& sd, const Row& rw) {
    if (sd.ks != nks - 1) return;
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (j < sd.gn && rw.v[j] < TR) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          *reinterpret_cast<floatx4*>(acc_s + acc_pos<NC>(rw.v[j], 4 * t + q)) += acc[j][t];
      }
    }
  };

  Step Vd[D], Sd[D];
  Src S[D];
  Row R[D];
  Val V[D];
  WSt Wr[D];
#pragma unroll
  for (int k = 0; k < D; ++k) Vd[k] = next_desc();  // steps 0 .. D-1
#pragma unroll
  for (int k = 0; k < D; ++k) ld_src(Vd[k], S[k]);
#pragma unroll
  for (int k = 0; k < D; ++k) Sd[k] = next_desc();  // steps D .. 2D-1
  ld_w(Vd[0], Wr[0]);
#pragma unroll
  for (int k = 0; k < D; ++k) {
    ld_row(Vd[k], R[k]);
    gather(Vd[k], S[k], V[k]);
  }
#pragma unroll
  for (int k = 0; k < D; ++k) ld_src(Sd[k], S[k]);
#pragma unroll
  for (int t = 1; t < D; ++t) ld_w(Vd[t], Wr[t]);  // steps 1 .. D-1
  st_w(Wr[0], 0);
  ld_w(Sd[0], Wr[0]);  // step D
  for (int base = 0; base < n_steps; base += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int s = base + k;
      const int k1 = (k + 1) % D;
      if (!(ABL & 1)) __syncthreads();  // wbuf[s & 1] holds step s's slice; step s-1's LDS updates are done
      mma(Vd[k], (s & 1) % NB, V[k]);
      consume_val(V[k]);
      if (!(ABL & 4)) {
        rmw(Vd[k], R[k]);
      } else if (Vd[k].gn > 0) {
        floatx4 z = acc[0][0];
#pragma unroll
        for (int j = 0; j < MJ; ++j)
#pragma unroll
          for (int t = 0; t < NT; ++t) z += acc[j][t];
        acc4[lane] += z;
      }
      consume_row(R[k]);
      if (!(ABL & 8)) {
        if (NB == 1) __syncthreads();  // every wave is done with step s's slice
        st_w(Wr[k1], ((s + 1) & 1) % NB);  // step s+1's slice (loaded D steps ago)
        ld_w(Sd[k1], Wr[k1]);       // step s+1+D
      }
      Vd[k] = Sd[k];
      ld_row(Vd[k], R[k]);  // step s+D
      gather(Vd[k], S[k], V[k]);
      Sd[k] = next_desc();  // step s+2D
      ld_src(Sd[k], S[k]);
    }
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


// ---------------------------------------------------------------- per-wave tiles
// Narrow outputs (c_out <= 32, c_in <= 64: level 0 of m=32 nets): one wave owns one 128-row output tile and all
// 16 NT output channels, accumulated in its own LDS tile, with no block barrier: with few chunks per offset and
// tile there is nothing to share between waves.  Per chunk the lane loads its row fragment
// X[src_r][32 kk + 8q .. +7] (split into the three bf16 pieces in registers) and reads the weight fragments
// (three pieces, NT column groups, NKK k-steps) from the per-step weight images of split_weights_kernel
// (KS = 32, NC = 16 NT: one coalesced 1 KiB wave-load per fragment).

// Per-wave tiles with weight runs.  conv_x6p_kernel reloads the lane's weight
// fragments with every chunk (6 of its 8 16-byte loads per chunk at
// c_in = 32), yet a tile's chunks are sorted by offset, so consecutive chunks
// mostly share them (about 3 chunks per offset run at level 0); dropping the
// reloads halved the kernel's time (timing ablation, wrong results).  Here a
// wave first lists its tile's offset runs (ballot over chunk_off: run start
// and offset packed per lane, read back with v_readlane), then keeps two
// weight sets in registers: the current run's and the next run's, loaded at
// the current run's first chunk (uniform branches; the chunk values keep
// their D-deep pipeline across runs).
// TR: output rows per wave tile (128, or 64: half the LDS accumulator tile per wave, so twice the blocks per CU).
#ifdef MSP_EXPERIMENTS
// x [n][c] fp32 (c % 32 == 0) -> its exact split image: row i, 32-channel slice kk, piece p, k-octet q at 16-byte
// unit (i * c / 32 + kk) * 12 + p * 4 + q.  One thread per (row, k-octet).
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ x, int64_t n, int c,
                                                         u32x4* __restrict__ img) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int oc = c / 8;
  if (g >= n * oc) return;
  const int64_t row = g / oc;
  const int o = (int)(g - row * oc), kk = o >> 2, q = o & 3;
  const floatx4* src = reinterpret_cast<const floatx4*>(x + row * c + 8 * o);
  u32x4 pc[3];
  split8(src[0], src[1], pc);
  u32x4* dst = img + (row * (c / 32) + kk) * 12 + q;
#pragma unroll
  for (int p = 0; p < 3; ++p) dst[p * 4] = pc[p];
}
#endif

// PS 1 (experiments build only; measured slower): x is the exact split image of the input rows (split_rows_kernel: per row and 32-channel slice, 3 pieces x 4
// k-octets of 16 bytes, row stride 6 c_in bytes), so the chunk loop loads the pieces instead of splitting every
// gathered row per rule.
// EPI (msp_bn_epilogue, round 6): the BatchNorm sums of the rows written; its own instantiation, so the plain form
// compiles exactly as before.
template <int NT, int NKK, int D, int NW, int TR = 128, int PS = 0, bool EPI = false>
__global__ __launch_bounds__(kThreads) void conv_x6r_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows,
    int64_t n_tiles, int n_y, float* __restrict__ out, BnEpi epi) {
  constexpr int NC = 16 * NT;
  constexpr int WU = 3 * 4 * NC;  // 16-byte units of one (offset, k-slice) image
  __shared__ floatx4 lds4[kWaves][TR * NC / 4];
  __shared__ int runs_s[kWaves][128];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t tile = (lb / n_y) * kWaves + wave;
  if (tile >= n_tiles) return;  // wave-uniform; the kernel has no block barrier
  float* acc_s = reinterpret_cast<float*>(lds4[wave]);
  for (int i = lane; i < TR * NC / 4; i += 64) lds4[wave][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int cy = (int)(lb % n_y);
  const int r = lane & 15, q = lane >> 4;
  const int64_t cb = tile_start[tile], ce = tile_start[tile + 1];
  const int n = (int)(ce - cb);
  const int64_t clast = ce > cb ? ce - 1 : cb;
  const u32x4* wim_c = wimg + (int64_t)cy * NKK * WU + q * NC + r;  // lane's unit in image (o, cy, 0), piece 0

  // offset runs of the tile: packed (first chunk << 8 | offset), at most
  // min(K, n) <= 128 of them
  int n_runs = 0;
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const int ic = i < n ? i : n - 1;
    const int o = chunk_off[cb + ic];
    const int op = chunk_off[cb + (ic > 0 ? ic - 1 : 0)];
    const bool st = i < n && (i == 0 || o != op);
    const unsigned long long m = ballot64(st);
    const int pos = n_runs + mbcnt64(m);
    if (st && pos < 128) runs_s[wave][pos] = (i << 8) | o;
    n_runs += __popcll(m);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nr_c = n_runs > 0 ? n_runs : 1;
  const int run_lo = n_runs > 0 ? runs_s[wave][lane < n_runs ? lane : n_runs - 1] : 0;
  const int run_hi = n_runs > 64 ? runs_s[wave][64 + lane < n_runs ? 64 + lane : n_runs - 1] : run_lo;
  auto run_at = [&](int j) -> int {  // packed run j (clamped to the last), j uniform
    const int jc = j < nr_c ? j : nr_c - 1;
    return jc < 64 ? __builtin_amdgcn_readlane(run_lo, jc) : __builtin_amdgcn_readlane(run_hi, jc - 64);
  };
  auto start_of = [&](int j) -> int { return j < n_runs ? (run_at(j) >> 8) : (1 << 22); };

  struct Wt {
    u32x4 w[NKK][NT][3];
  };
  auto ld_w = [&](int j, Wt& w) {
    const int o = run_at(j) & 255;
    const int ow = flip ? (K - 1 - o) : o;
    const u32x4* wo = wim_c + (int64_t)ow * n_y * NKK * WU;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) w.w[kk][t][p] = wo[kk * WU + p * 4 * NC + 16 * t];
  };
  struct St {
    int src, row;
  };
  struct Val {
    floatx4 a[NKK][PS ? 3 : 2];
  };
  auto ld_idx = [&](int64_t c, St& d) {
    const int64_t cc = c < clast ? c : clast;
    d.src = chunk_src[cc * MSP_CHUNK + r];
    d.row = chunk_row[cc * MSP_CHUNK + r];
  };
  auto ld_val = [&](const St& d, Val& v) {
    if constexpr (PS) {  // the row's units (kk, p, q): 16 bytes each, 12 per 32-channel slice
      const floatx4* xs = reinterpret_cast<const floatx4*>(x) + (uint32_t)d.src * (uint32_t)(NKK * 12) + q;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
        for (int p = 0; p < 3; ++p) v.a[kk][p] = xs[kk * 12 + p * 4];
      return;
    }
    const char* xs = reinterpret_cast<const char*>(x) + (uint32_t)d.src * (uint32_t)c_in * 4u;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int k = min(32 * kk + 8 * q, c_in - 8);  // k past c_in: finite data times zero weights
      const floatx4* pv = reinterpret_cast<const floatx4*>(xs + 4u * (uint32_t)k);
      v.a[kk][0] = pv[0];
      v.a[kk][1] = pv[1];
    }
  };
  auto run = [&](const Val& v, const Wt& w, int row) {
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      u32x4 xp[3];
      if constexpr (PS) {
#pragma unroll
        for (int p = 0; p < 3; ++p) xp[p] = __builtin_bit_cast(u32x4, v.a[kk][p]);
      } else {
        split8(v.a[kk][0], v.a[kk][1], xp);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        floatx4 c = acc[t];
        c = mfma_bf16(w.w[kk][t][2], xp[0], c);
        c = mfma_bf16(w.w[kk][t][1], xp[1], c);
        c = mfma_bf16(w.w[kk][t][0], xp[2], c);
        c = mfma_bf16(w.w[kk][t][1], xp[0], c);
        c = mfma_bf16(w.w[kk][t][0], xp[1], c);
        acc[t] = mfma_bf16(w.w[kk][t][0], xp[0], c);
      }
    }
    if (row < TR) {
#pragma unroll
      for (int t = 0; t < NT; ++t) *reinterpret_cast<floatx4*>(acc_s + acc_pos<NC>(row, 4 * t + q)) += acc[t];
    }
  };
  // Wc: the set the MFMAs read (written only by register copies, so the
  // chunk loop never waits on a weight load); Wn: the next run's set, loaded
  // at the current run's first chunk and copied at the next run's.
  Wt Wc, Wn;
  ld_w(0, Wc);
  ld_w(1, Wn);
  int rho = 0, next_start = start_of(1);
  St J[D];
  int rowR[D];
  Val S[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    ld_idx(cb + k, J[k]);
    rowR[k] = J[k].row;
    ld_val(J[k], S[k]);
  }
#pragma unroll
  for (int k = 0; k < D; ++k) ld_idx(cb + D + k, J[k]);
  for (int64_t c = cb; c < ce; c += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int i = (int)(c - cb) + k;
      if (i == next_start) {  // first chunk of run rho + 1 (never true past the last run)
        ++rho;
        next_start = start_of(rho + 1);
        Wc = Wn;
        ld_w(rho + 1, Wn);
      }
      if (i < n) run(S[k], Wc, rowR[k]);
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        asm volatile("" ::"v"(S[k].a[kk][0]), "v"(S[k].a[kk][1]));
        if constexpr (PS) asm volatile("" ::"v"(S[k].a[kk][PS ? 2 : 0]));
      }
      ld_val(J[k], S[k]);  // chunk c+k+D
      rowR[k] = J[k].row;
      ld_idx(c + k + 2 * D, J[k]);
    }
  }
  const int64_t row0 = tile * TR;
  const int nr = (int)((n_rows - row0) < TR ? (n_rows - row0) : TR);
  constexpr int V4 = NC / 4;
  const int c0 = cy * NC;
  // msp_bn_epilogue (uniform): the BatchNorm sums of the tile's rows, per lane for its column quad lane % V4,
  // then over the wave's lanes into this tile's slot (TR = 128: one slot per tile)
  if constexpr (!EPI) {
    for (int i = lane; i < nr * V4; i += 64) {
      const int rr = i / V4, g = i % V4;
      *reinterpret_cast<floatx4*>(out + (row0 + rr) * c_out + c0 + 4 * g) =
          *reinterpret_cast<const floatx4*>(acc_s + acc_pos<NC>(rr, g));
    }
    return;
  }
  BnEpiAcc ea;
  ea.init(epi, c0 + 4 * (lane % V4));
  // backward: the BN input quads in batches of four loads in flight (16 serial latencies per tile otherwise)
  constexpr int EI = TR * V4 / 64, EB = 4;  // output quads per lane, batch
  static_assert(EI * 64 == TR * V4 && EI % EB == 0, "whole batches of quads per lane");
#pragma unroll
  for (int e0 = 0; e0 < EI; e0 += EB) {
    floatx4 xq[EB];
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int i = lane + 64 * (e0 + e);
      xq[e] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (epi.x != nullptr && i < nr * V4)
        xq[e] = *reinterpret_cast<const floatx4*>(epi.x + (row0 + i / V4) * epi.C + c0 + 4 * (i % V4));
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int i = lane + 64 * (e0 + e);
      if (i < nr * V4) {
        const int rr = i / V4, g = i % V4;
        const floatx4 v = *reinterpret_cast<const floatx4*>(acc_s + acc_pos<NC>(rr, g));
        *reinterpret_cast<floatx4*>(out + (row0 + rr) * c_out + c0 + 4 * g) = v;
        ea.add_x(epi, v, epi.x != nullptr ? xq[e] : v);
      }
    }
  }
  {
    static_assert(!EPI || (TR == 128 && 64 % V4 == 0), "one epilogue slot per 128-row tile");
    ea.wave_reduce<V4>();
    if (lane < V4)
#pragma unroll
      for (int k = 0; k < 8; ++k) *bn_epi_slot(epi, k >> 2, c0 + 4 * lane + (k & 3), tile) = ea.s[k];
  }
}

// Per-wave form for narrow outputs; ws holds the weight images (x6p_ws_bytes).  Two weight register sets per
// offset run, chunk values three deep (profiles/r01/kbench_x6r_r01u.log).
int launch_x6r(const float* x, int c_in, const float* wt, int K, int flip, int c_out, const int64_t* tile_start,
               const uint8_t* chunk_off, const int32_t* chunk_src, const uint16_t* chunk_row, int64_t n_rows,
               float* out, void* ws, hipStream_t s, const msp_bn_epilogue* epi) {
  const BnEpi be = bn_epi_of(epi, c_out, n_rows);
  const int NT = c_out / 16 >= 2 && (c_out / 16) % 2 == 0 ? 2 : 1;
  const int NKK = (c_in + 31) / 32;
  const int n_y = c_out / (16 * NT);
  const int64_t n_tiles = ceil_div(n_rows, 128);
  u32x4* wimg = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)K * c_out * NKK * 32 * 6 / 16;
  if (!(flip & 4))  // bit 2: ws already holds this image (msp_split_weight_images)
    split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, K, c_out, c_in, 16 * NT, 32, wimg,
                                                                         (flip >> 1) & 1);
  flip &= 1;
  const unsigned grid = (unsigned)(ceil_div(n_tiles, kWaves) * n_y);
#define LR(N, C)                                                                                               \
  if (NT == N && NKK == C) {                                                                                   \
    if (epi)                                                                                                   \
      conv_x6r_kernel<N, C, 3, 2, 128, 0, true><<<grid, kThreads, 0, s>>>(                                     \
          x, c_in, wimg, K, flip, c_out, tile_start, chunk_off, chunk_src, chunk_row, n_rows, n_tiles, n_y, out, be); \
    else                                                                                                       \
      conv_x6r_kernel<N, C, 3, 2><<<grid, kThreads, 0, s>>>(x, c_in, wimg, K, flip, c_out, tile_start, chunk_off, \
                                                            chunk_src, chunk_row, n_rows, n_tiles, n_y, out, be); \
    return MSP_OK;                                                                                             \
  }
  LR(2, 1) LR(2, 2) LR(1, 1) LR(1, 2)
#undef LR
  set_error("msp_conv_tile: no per-wave x6 kernel for c_in=%d c_out=%d", c_in, c_out);
  return MSP_EINVAL;
}


size_t x6p_ws_bytes(int K, int c_in, int c_out) { return (size_t)K * c_out * ((c_in + 31) / 32) * 32 * 6; }

#ifdef MSP_EXPERIMENTS
// Per-wave form with the tile height and pipeline depth as parameters (scripts/kbench.py, experiments build):
// variant = 10 * D + (tile_rows == 64); the rulebook must have tile_rows-row tiles.
int launch_x6r_exp(int variant, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                   int tile_rows, const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                   const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, hipStream_t s) {
  const int NT = c_out / 16 >= 2 && (c_out / 16) % 2 == 0 ? 2 : 1;
  const int NKK = (c_in + 31) / 32;
  const int n_y = c_out / (16 * NT);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  u32x4* wimg = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)K * c_out * NKK * 32 * 6 / 16;
  split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, K, c_out, c_in, 16 * NT, 32, wimg,
                                                                       (flip >> 1) & 1);
  flip &= 1;
  const unsigned grid = (unsigned)(ceil_div(n_tiles, kWaves) * n_y);
  // variant 100 + v: pre-split rows (the split pass into the workspace past the weight image, then the PS kernel);
  // 200 + v: the PS kernel alone on whatever the workspace holds (timing only)
  const int ps = variant / 100;
  variant %= 100;
  const int D = variant / 10, T = variant % 10 == 1 ? 64 : 128;
  if (T != tile_rows) return MSP_EINVAL;
  const float* xin = x;
  if (ps) {
    if (c_in % 32) return MSP_EINVAL;
    u32x4* img = wimg + (units + 63) / 64 * 64;
    if (ps == 1)
      split_rows_kernel<<<(unsigned)ceil_div(n_rows * (c_in / 8), 256), 256, 0, s>>>(x, n_rows, c_in, img);
    xin = reinterpret_cast<const float*>(img);
  }
#define LE(N, C, DD, TT)                                                                                        \
  if (NT == N && NKK == C && D == DD && T == TT) {                                                             \
    if (ps)                                                                                                    \
      conv_x6r_kernel<N, C, DD, 2, TT, 1><<<grid, kThreads, 0, s>>>(xin, c_in, wimg, K, flip, c_out,           \
                                                                    tile_start, chunk_off, chunk_src,          \
                                                                    chunk_row, n_rows, n_tiles, n_y, out,      \
                                                                    BnEpi{});                                  \
    else                                                                                                       \
      conv_x6r_kernel<N, C, DD, 2, TT><<<grid, kThreads, 0, s>>>(x, c_in, wimg, K, flip, c_out, tile_start,    \
                                                                 chunk_off, chunk_src, chunk_row, n_rows,      \
                                                                 n_tiles, n_y, out, BnEpi{});                  \
    return MSP_OK;                                                                                             \
  }
  LE(2, 1, 3, 128) LE(2, 1, 3, 64) LE(2, 1, 2, 128) LE(2, 1, 2, 64)
  LE(2, 2, 3, 128) LE(2, 2, 3, 64) LE(2, 2, 2, 64) LE(2, 2, 2, 128)
#undef LE
  set_error("launch_x6r_exp: no variant %d for c_in=%d c_out=%d", variant, c_in, c_out);
  return MSP_EINVAL;
}
#endif

// ---------------------------------------------------------------- one contribution per output row, split-bf16
// msp_conv_pairs_x6 (round 6): the deconvolution forward and the strided convolution's backward-data -- every
// output row has exactly one (source row, offset) pair -- on the x6 MFMAs instead of conv_pairs_kernel's exact
// fp32 16x16x4 ones.  A wave takes one 16-pair chunk of one offset: lane (r, q) gathers pair r's source row at k
// 8q .. +7 per 32-deep slice and splits it into three bf16 pieces, the offset's weight fragments come from the
// per-call image (split_weights_kernel, NC = 16 NT, KS = 32: x6r's layout), and each 16 x 16 output tile is six
// MFMAs per slice summed in a zeroed accumulator (the gather forms' order); lane (r, q) then holds output channels
// 16 t + 4 q .. +3 of pair r and stores them as one float4.  conv_pairs_kernel's fp32 MFMA chain is 8 dependent
// 32-cycle MFMAs per 32 input channels; here it is 6 of 16 cycles.
template <int NT>
__global__ __launch_bounds__(kThreads) void conv_pairs_x6_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ chunk_start, int64_t n_chunks, int n_y, float* __restrict__ out) {
  constexpr int NC = 16 * NT, WU = 3 * 4 * NC;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t chunk = (int64_t)blockIdx.x * kWaves + wave;
  if (chunk >= n_chunks) return;  // wave-uniform; no block barrier
  int lo = 0, hi = K;             // chunk_start[lo] <= chunk < chunk_start[hi]: the chunk's offset
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunk_start[mid] <= chunk) lo = mid;
    else hi = mid;
  }
  const int o = lo, cy = blockIdx.y;
  const int64_t p0 = off_start[o] + (chunk - chunk_start[o]) * MSP_CHUNK, p1 = off_start[o + 1];
  const int r = lane & 15, q = lane >> 4;
  const int src = p0 + r < p1 ? pin[p0 + r] : -1;
  const int nkk = (c_in + 31) / 32;
  const u32x4* wo = wimg + ((int64_t)o * n_y + cy) * nkk * WU + q * NC + r;
  const float* xs = x + (int64_t)(src < 0 ? 0 : src) * c_in;
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int kk = 0; kk < nkk; ++kk) {
    const int k = min(32 * kk + 8 * q, c_in - 8);  // past c_in: finite data times zero weights
    floatx4 a = *reinterpret_cast<const floatx4*>(xs + k), b = *reinterpret_cast<const floatx4*>(xs + k + 4);
    if (src < 0) a = b = floatx4{0.f, 0.f, 0.f, 0.f};
    u32x4 xp[3];
    split8(a, b, xp);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const u32x4 w0 = wo[kk * WU + 0 * 4 * NC + 16 * t], w1 = wo[kk * WU + 1 * 4 * NC + 16 * t],
                  w2 = wo[kk * WU + 2 * 4 * NC + 16 * t];
      floatx4 c = mfma_bf16(w2, xp[0], floatx4{0.f, 0.f, 0.f, 0.f});
      c = mfma_bf16(w1, xp[1], c);
      c = mfma_bf16(w0, xp[2], c);
      c = mfma_bf16(w1, xp[0], c);
      c = mfma_bf16(w0, xp[1], c);
      acc[t] += mfma_bf16(w0, xp[0], c);
    }
  }
  if (p0 + r < p1) {
    float* dst = out + (int64_t)pout[p0 + r] * c_out + cy * NC + 4 * q;
#pragma unroll
    for (int t = 0; t < NT; ++t) *reinterpret_cast<floatx4*>(dst + 16 * t) = acc[t];
  }
}

// The same over a run of consecutive chunks per wave (c_in <= 32 KK): the next chunk's x rows are loaded and the
// indices two chunks ahead read while the current chunk's MFMAs and stores run (the latency chain index -> row
// gather -> MFMA -> scattered store is what bounds the one-chunk form: 2.5 TB/s and 43 TF/s at level 0).  WREG
// keeps the offset's weight fragments in registers across the run (reloaded when the run crosses an offset).
template <int NT, int KK, bool WREG>
__global__ __launch_bounds__(kThreads) void conv_pairs_x6_pipe_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    const int64_t* __restrict__ chunk_start, int64_t n_chunks, int run, int n_y, float* __restrict__ out) {
  constexpr int NC = 16 * NT, WU = 3 * 4 * NC;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t ch0 = ((int64_t)blockIdx.x * kWaves + wave) * run;
  if (ch0 >= n_chunks) return;  // wave-uniform; no block barrier
  const int64_t ch1 = ch0 + run < n_chunks ? ch0 + run : n_chunks;
  const int cy = blockIdx.y, r = lane & 15, q = lane >> 4;
  const int nkk = (c_in + 31) / 32;
  int oi = 0, hi = K;  // chunk_start[oi] <= ch0 < chunk_start[hi]
  while (hi - oi > 1) {
    const int mid = (oi + hi) >> 1;
    if (chunk_start[mid] <= ch0) oi = mid;
    else hi = mid;
  }
  int64_t oi_first = chunk_start[oi], oi_end = chunk_start[oi + 1], pb = off_start[oi], pe = off_start[oi + 1];
  auto indices = [&](int64_t ch, int& src, int& dst, int& o_of) {
    if (ch >= oi_end) {
      do {
        ++oi;
        oi_end = chunk_start[oi + 1];
      } while (ch >= oi_end);
      oi_first = chunk_start[oi];
      pb = off_start[oi];
      pe = off_start[oi + 1];
    }
    const int64_t p = pb + (ch - oi_first) * MSP_CHUNK + r;
    src = p < pe ? pin[p] : -1;
    dst = p < pe ? pout[p] : -1;
    o_of = oi;
  };
  auto load_x = [&](int src, floatx4 (&a)[KK][2]) {
    const float* xs = x + (int64_t)(src < 0 ? 0 : src) * c_in;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      if (kk < nkk) {
        const int k = min(32 * kk + 8 * q, c_in - 8);  // past c_in: finite data times zero weights
        a[kk][0] = *reinterpret_cast<const floatx4*>(xs + k);
        a[kk][1] = *reinterpret_cast<const floatx4*>(xs + k + 4);
      }
  };
  u32x4 w[WREG ? KK : 1][NT][3];
  int ow = -1;
  int s_c, d_c, o_c, s_n = -1, d_n = -1, o_n = 0;
  floatx4 a[KK][2];
  indices(ch0, s_c, d_c, o_c);
  load_x(s_c, a);
  if (ch0 + 1 < ch1) indices(ch0 + 1, s_n, d_n, o_n);
  for (int64_t ch = ch0; ch < ch1; ++ch) {
    const u32x4* wo = wimg + ((int64_t)o_c * n_y + cy) * nkk * WU + q * NC + r;
    if (WREG && o_c != ow) {
      ow = o_c;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        if (kk < nkk) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 3; ++j) w[WREG ? kk : 0][t][j] = wo[kk * WU + j * 4 * NC + 16 * t];
        }
    }
    const bool more = ch + 1 < ch1;
    floatx4 an[KK][2];
    if (more) load_x(s_n, an);
    int s2 = -1, d2 = -1, o2 = o_n;
    if (ch + 2 < ch1) indices(ch + 2, s2, d2, o2);
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      if (kk < nkk) {
        floatx4 lo = a[kk][0], hi4 = a[kk][1];
        if (s_c < 0) lo = hi4 = floatx4{0.f, 0.f, 0.f, 0.f};
        u32x4 xp[3];
        split8(lo, hi4, xp);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          u32x4 w0, w1, w2;
          if (WREG) {
            w0 = w[WREG ? kk : 0][t][0];
            w1 = w[WREG ? kk : 0][t][1];
            w2 = w[WREG ? kk : 0][t][2];
          } else {
            w0 = wo[kk * WU + 0 * 4 * NC + 16 * t];
            w1 = wo[kk * WU + 1 * 4 * NC + 16 * t];
            w2 = wo[kk * WU + 2 * 4 * NC + 16 * t];
          }
          floatx4 c = mfma_bf16(w2, xp[0], floatx4{0.f, 0.f, 0.f, 0.f});
          c = mfma_bf16(w1, xp[1], c);
          c = mfma_bf16(w0, xp[2], c);
          c = mfma_bf16(w1, xp[0], c);
          c = mfma_bf16(w0, xp[1], c);
          acc[t] += mfma_bf16(w0, xp[0], c);
        }
      }
    if (d_c >= 0) {
      float* dst = out + (int64_t)d_c * c_out + cy * NC + 4 * q;
#pragma unroll
      for (int t = 0; t < NT; ++t) *reinterpret_cast<floatx4*>(dst + 16 * t) = acc[t];
    }
    if (more) {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        a[kk][0] = an[kk][0];
        a[kk][1] = an[kk][1];
      }
      s_c = s_n;
      d_c = d_n;
      o_c = o_n;
      s_n = s2;
      d_n = d2;
      o_n = o2;
    }
  }
}

// ---------------------------------------------------------------- dense row groups
// Submanifold convolutions on large levels, straight from the neighbour map
// nbr[K][n] (int32, -1 absent): no tile rulebook and no LDS accumulation.
// A wave owns G groups of 16 consecutive output rows and 16 NT output
// channels, and keeps their accumulators in registers (G x NT MFMA tiles);
// it walks the K x ceil(c_in / 32) steps (offset, 32-deep k-slice) in order,
// gathering the 16 rows' neighbours of each group (absent neighbours and k
// past c_in read as zero) and skipping a group's MFMAs when none of its rows
// has the offset (wave-uniform ballot).  Rows with a neighbour are only
// 30-55 % of a group's (offset, row) slots at levels 0-2, but every wave of a
// block does the same steps, so the block shares each step's split weight
// slice through LDS (double buffered, one barrier per step, staged from
// registers loaded two steps ahead) instead of reloading it per wave.
// Gathered values run two steps ahead, neighbour indices four; each step's six
// piece products are summed in a zeroed accumulator and added once.
template <int NT, int G, int OCC = 1, int LR = 0, int NW = kWaves>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(OCC))) void conv_x6g_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const int32_t* __restrict__ nbr, const int32_t* __restrict__ perm, int64_t n_rows, int n_y,
    float* __restrict__ out) {
  constexpr int NC = 16 * NT;
  constexpr int WU = 3 * 4 * NC;  // 16-byte units of one step's split weight slice
  constexpr int TRW = 16 * G;     // rows per wave
  constexpr int NTH = 64 * NW;    // threads per block (NW waves share each step's weight slice)
  constexpr int WPT = (WU + NTH - 1) / NTH;
  __shared__ u32x4 wl[2][WU];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int cy = (int)(lb % n_y);
  const int64_t row0 = (lb / n_y) * (int64_t)(NW * TRW) + wave * TRW;
  const int nks = (c_in + 31) / 32;
  const int n_steps = K * nks;
  uint32_t rowok = 0;  // lane's rows inside the level
#pragma unroll
  for (int g = 0; g < G; ++g) rowok |= (row0 + 16 * g + r < n_rows ? 1u : 0u) << g;

  struct Wst {
    u32x4 u[WPT];
  };
  struct Ix {
    int v[G];
  };
  struct Xv {
    floatx4 a[G][2];
    uint32_t ok;  // lane: bit g = its row of group g has the neighbour (and k < c_in)
  };
  auto ld_wst = [&](int s, Wst& w) {
    const int sc = s < n_steps ? s : n_steps - 1;
    const int o = sc / nks, ks = sc - o * nks;
    const int ow = flip ? K - 1 - o : o;
    const u32x4* src = wimg + ((int64_t)(ow * n_y + cy) * nks + ks) * WU;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int u = tid + i * NTH;
      w.u[i] = src[u < WU ? u : WU - 1];
    }
  };
  auto st_wst = [&](const Wst& w, int buf) {
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int u = tid + i * NTH;
      if (WU % NTH == 0 || u < WU) wl[buf][u] = w.u[i];
    }
  };
  auto ld_ix = [&](int s, Ix& d) {
    const int sc = s < n_steps ? s : n_steps - 1;
    const int o = sc / nks;
    const int32_t* m = nbr + (int64_t)o * n_rows;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t row = row0 + 16 * g + r;
      d.v[g] = m[row < n_rows ? row : n_rows - 1];
    }
  };
  // values of step s from its neighbour indices; returns the wave's mask of
  // groups with any neighbour
  auto ld_x = [&](int s, const Ix& d, Xv& v) -> uint32_t {
    const int sc = s < n_steps ? s : n_steps - 1;
    const int ks = sc % nks;
    const int k = 32 * ks + 8 * q;
    uint32_t am = 0, ok = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool has = d.v[g] >= 0 && ((rowok >> g) & 1);
      am |= (ballot64(has) != 0 ? 1u : 0u) << g;
      const bool lo = has && k < c_in;
      ok |= (lo ? 1u : 0u) << g;
      const floatx4* pv = reinterpret_cast<const floatx4*>(x + (int64_t)(lo ? d.v[g] : 0) * c_in + (lo ? k : 0));
      // branch-free: lanes without a neighbour read row 0 (hot) and are zeroed at use;
      // exec-masked loads measured 1-4 % slower (profiles/r01/kbench_nbr_masked_r01z.log)
      v.a[g][0] = pv[0];
      v.a[g][1] = pv[1];
    }
    v.ok = ok;
    return am;
  };
  floatx4 acc[G][NT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto run = [&](int buf, const Xv& v, uint32_t am) {
    if constexpr (LR) {
      // column group outer: three weight fragments live at a time
      u32x4 xp[G][3];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const bool lo = (v.ok >> g) & 1;
        const floatx4 z = {0.f, 0.f, 0.f, 0.f};
        if ((am >> g) & 1) split8(lo ? v.a[g][0] : z, lo ? v.a[g][1] : z, xp[g]);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const u32x4 w0 = wl[buf][(0 * 4 + q) * NC + 16 * t + r];
        const u32x4 w1 = wl[buf][(1 * 4 + q) * NC + 16 * t + r];
        const u32x4 w2 = wl[buf][(2 * 4 + q) * NC + 16 * t + r];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if ((am >> g) & 1) {  // wave-uniform
            floatx4 c = {0.f, 0.f, 0.f, 0.f};
            c = mfma_bf16(w2, xp[g][0], c);
            c = mfma_bf16(w1, xp[g][1], c);
            c = mfma_bf16(w0, xp[g][2], c);
            c = mfma_bf16(w1, xp[g][0], c);
            c = mfma_bf16(w0, xp[g][1], c);
            acc[g][t] += mfma_bf16(w0, xp[g][0], c);
          }
        }
      }
      return;
    }
    u32x4 w[NT][3];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) w[t][p] = wl[buf][(p * 4 + q) * NC + 16 * t + r];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if ((am >> g) & 1) {  // wave-uniform
        const bool lo = (v.ok >> g) & 1;
        const floatx4 z = {0.f, 0.f, 0.f, 0.f};
        u32x4 xp[3];
        split8(lo ? v.a[g][0] : z, lo ? v.a[g][1] : z, xp);
#pragma unroll
        for (int t = 0; t < NT; ++t) {  // the step's six products summed apart, then added once
          floatx4 c = {0.f, 0.f, 0.f, 0.f};
          c = mfma_bf16(w[t][2], xp[0], c);
          c = mfma_bf16(w[t][1], xp[1], c);
          c = mfma_bf16(w[t][0], xp[2], c);
          c = mfma_bf16(w[t][1], xp[0], c);
          c = mfma_bf16(w[t][0], xp[1], c);
          acc[g][t] += mfma_bf16(w[t][0], xp[0], c);
        }
      }
    }
  };
  constexpr int NS = LR ? 1 : 2;  // weight staging slots (slices loaded NS steps ahead)
  Wst S[2];
  Ix I[2];
  Xv X[2];
  uint32_t am[2];
  ld_wst(0, S[0]);
  if (NS == 2) ld_wst(1, S[1]);
  ld_ix(0, I[0]);
  ld_ix(1, I[1]);
  st_wst(S[0], 0);
  ld_wst(NS == 2 ? 2 : 1, S[0]);
  am[0] = ld_x(0, I[0], X[0]);
  am[1] = ld_x(1, I[1], X[1]);
  ld_ix(2, I[0]);
  ld_ix(3, I[1]);
  // step s (slot k = s & 1): wl[k] holds its weight slice, X[k] its values,
  // S[k ^ 1] (S[0] with one slot) the slice of s + 1, I[k] the indices of
  // s + 2, I[k ^ 1] of s + 3
  auto step = [&](int s, auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int sk = NS == 2 ? (k ^ 1) : 0;
    __syncthreads();
    st_wst(S[sk], k ^ 1);
    ld_wst(s + 1 + NS, S[sk]);
    run(k, X[k], s < n_steps ? am[k] : 0u);
    am[k] = ld_x(s + 2, I[k], X[k]);
    ld_ix(s + 4, I[k]);
  };
  // an even step count (a trailing step with no work), so both halves of the
  // unrolled loop always run and the wait counts are the same every lap
  for (int s = 0; s < n_steps; s += 2) {
    step(s, std::integral_constant<int, 0>{});
    step(s + 1, std::integral_constant<int, 1>{});
  }
  float* dst = out + cy * NC + 4 * q;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if ((rowok >> g) & 1) {
      const int64_t j = row0 + 16 * g + r;
      float* rowp = dst + (perm ? (int64_t)perm[j] : j) * c_out;
#pragma unroll
      for (int t = 0; t < NT; ++t) *reinterpret_cast<floatx4*>(rowp + 16 * t) = acc[g][t];
    }
  }
}

// Dense row-group form; ws holds the split weight slices (x6g_ws_bytes).  Column-group-outer MFMAs, one staging
// slot, ONE 16-row group per wave at a 4-waves-per-SIMD budget (108 / 94 VGPRs, no spills): conv family +1.5 %
// over two groups at 3 waves (profiles/r01/bench_ab_g1_r01.log); NT = 4 (3 for 96 channels)
// (profiles/r01/kbench_nbr_r01v.log).
int launch_x6g(const float* x, int c_in, const float* wt, int K, int flip, int c_out, const int32_t* nbr,
               const int32_t* perm, int64_t n_rows, float* out, void* ws, hipStream_t s) {
  const int n16 = c_out / 16;
  const int nt = n16 % 4 == 0 ? 4 : (n16 % 3 == 0 ? 3 : (n16 % 2 == 0 ? 2 : 1));
  const int n_y = n16 / nt;
  const int nks = (c_in + 31) / 32;
  u32x4* wimg = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)K * c_out * nks * 32 * 6 / 16;
  if (!(flip & 4))  // bit 2: ws already holds this image (msp_split_weight_images)
    split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, K, c_out, c_in, 16 * nt, 32, wimg,
                                                                         (flip >> 1) & 1);
  flip &= 1;
  const unsigned grid = (unsigned)(ceil_div(n_rows, (int64_t)kWaves * 16) * n_y);
#define LL(N)                                                                                                 \
  if (nt == N) {                                                                                              \
    conv_x6g_kernel<N, 1, 4, 1><<<grid, kThreads, 0, s>>>(x, c_in, wimg, K, flip, c_out, nbr, perm, n_rows,    \
                                                          n_y, out);                                          \
    return MSP_OK;                                                                                            \
  }
  LL(4) LL(3) LL(2) LL(1)
#undef LL
  set_error("msp_conv_nbr: no dense-group kernel for nt=%d", nt);
  return MSP_EINVAL;
}


size_t x6g_ws_bytes(int K, int c_in, int c_out) { return (size_t)K * c_out * ((c_in + 31) / 32) * 32 * 6; }

// ---------------------------------------------------------------- weight gradient
// dW[o] = sum over the pairs (i, j) of offset o of x[i]^T dy[j], on bf16 MFMA
// over exact three-piece splits of both operands (six products per fp32
// multiply-add, as the convolution above).  Block = piece of one offset's
// pair list and one (16 WA x 16 WB) dW tile, as conv_wgrad4_kernel
// (msp_conv.hip), whose slab and reduction it shares.  MFMA k = 32 pairs:
// lane (r, q) takes pairs 8q .. 8q+7 of a super-step and loads WA
// consecutive input channels m0 + WA r .. and WB output channels n0 + WB r ..
// of each (16 lanes read 16 WA contiguous floats of one row), so component
// sa of its 8 x vectors is the lane's A fragment for channel m0 + WA r + sa
// and component sb of its dy vectors its B fragment: accumulator (sa, sb)
// register j holds dW[m0 + WA (4q + j) + sa][n0 + WB r + sb].  Waves take
// super-steps round-robin, two register sets deep; positions past the piece
// are clamped to its last pair and their x values zeroed (uniform branch:
// only the last super-step of a wave in a piece can be partial).
// ABL (timing only, bits): 1 = no splits (raw bits as the pieces), 2 = no MFMAs, 4 = no row loads,
// 8 = no pair-list loads.
// d[j] = v of lane B + j of this lane's row of 16 (DPP row_newbcast), j = 0 .. 7
template <int B, int... J>
__device__ __forceinline__ void row_bcast8_(int32_t v, int32_t (&d)[8], std::integer_sequence<int, J...>) {
  ((d[J] = __builtin_amdgcn_update_dpp(0, v, 0x150 + B + J, 0xF, 0xF, false)), ...);
}
template <int B>
__device__ __forceinline__ void row_bcast8(int32_t v, int32_t (&d)[8]) {
  row_bcast8_<B>(v, d, std::make_integer_sequence<int, 8>{});
}

template <int WA, int WB, int ABL = 0, int D = 2>
__global__ __launch_bounds__(kThreads, D == 1 ? 4 : 1) void wgrad_x6_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out,
    const int32_t* __restrict__ pin, const int32_t* __restrict__ pout, const int64_t* __restrict__ off_start,
    int K, int64_t n_pieces, int n_ty, float* __restrict__ slab) {
  constexpr int TM = 16 * WA, TN = 16 * WB;
  __shared__ float red[TM * TN];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t b = lb / n_ty;
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

  // pair indices: one word per lane per super-step (lanes r < 8 of row q hold pin of pairs 8q .. 8q+7, lanes
  // r >= 8 their pout), handed to the 16 lanes of the row by DPP row broadcasts -- one coalesced load instead
  // of 16 per lane
  struct Ix {
    int32_t w;
  };
  struct Vals {
    float a[8][WA], b[8][WB];
  };
  const int32_t* pix = r < 8 ? pin : pout;
  auto ld_idx = [&](int64_t g, Ix& d) {
    const int64_t pc = min(g + 8 * q + (r & 7), p1 - 1);
    d.w = (ABL & 8) ? (int32_t)(pc >> 4) : pix[pc];  // ABL 8 (timing only): synthetic rows, pc / 16 < n_rows
  };
  const float* xm = x + m0 + WA * r;
  const float* dyn = dy + n0 + WB * r;
  auto ld_val = [&](const Ix& d, Vals& v) {
    int32_t ii[8], oo[8];
    row_bcast8<0>(d.w, ii);
    row_bcast8<8>(d.w, oo);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (ABL & 4) {  // timing only: values from the indices instead of the row loads
#pragma unroll
        for (int i = 0; i < WA; ++i) v.a[k][i] = (float)(ii[k] + i) * 1e-6f;
#pragma unroll
        for (int t = 0; t < WB; ++t) v.b[k][t] = (float)(oo[k] + t) * 1e-6f;
      } else {
        load_vec<WA>(xm + (int64_t)ii[k] * c_in, v.a[k]);
        load_vec<WB>(dyn + (int64_t)oo[k] * c_out, v.b[k]);
      }
    }
  };
  auto compute = [&](int64_t g, Vals& v) {
    auto& a = v.a;
    if (g + 32 > p1) {  // uniform: partial super-step, zero the x values of pairs past the piece
      const int64_t pp = g + 8 * q;
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int i = 0; i < WA; ++i) a[k][i] = pp + k < p1 ? a[k][i] : 0.f;
    }
    auto split = [&](const floatx4& lo, const floatx4& hi, u32x4 (&pc)[3]) {
      if (ABL & 1) {
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          pc[pp] = u32x4{__float_as_uint(lo[pp]), __float_as_uint(lo[pp + 1]), __float_as_uint(hi[pp]),
                         __float_as_uint(hi[pp + 1])};
      } else {
        split8(lo, hi, pc);
      }
    };
    u32x4 bp[WB][3];
#pragma unroll
    for (int t = 0; t < WB; ++t)
      split(floatx4{v.b[0][t], v.b[1][t], v.b[2][t], v.b[3][t]}, floatx4{v.b[4][t], v.b[5][t], v.b[6][t], v.b[7][t]},
            bp[t]);
#pragma unroll
    for (int i = 0; i < WA; ++i) {
      u32x4 ap[3];
      split(floatx4{a[0][i], a[1][i], a[2][i], a[3][i]}, floatx4{a[4][i], a[5][i], a[6][i], a[7][i]}, ap);
#pragma unroll
      for (int t = 0; t < WB; ++t) {
        if (ABL & 2) {
          acc[i][t] += __builtin_bit_cast(floatx4, ap[0] ^ ap[1] ^ ap[2] ^ bp[t][0] ^ bp[t][1] ^ bp[t][2]);
          continue;
        }
        floatx4 c = acc[i][t];
        c = mfma_bf16(ap[2], bp[t][0], c);
        c = mfma_bf16(ap[1], bp[t][1], c);
        c = mfma_bf16(ap[0], bp[t][2], c);
        c = mfma_bf16(ap[1], bp[t][0], c);
        c = mfma_bf16(ap[0], bp[t][1], c);
        acc[i][t] = mfma_bf16(ap[0], bp[t][0], c);
      }
    }
  };
  constexpr int64_t kStride = 32 * kWaves;
  const int64_t g0 = p0 + 32 * wave;
  if (g0 < p1) {  // wave-uniform
    // values run D super-steps ahead, indices U = 2D ahead of their values (one VGPR per set)
    constexpr int U = 2 * D;
    Ix X[U];
    Vals V[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      ld_idx(g0 + k * kStride, X[k]);
      ld_val(X[k], V[k]);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) ld_idx(g0 + (D + k) * kStride, X[k]);
    for (int64_t g = g0; g < p1; g += U * kStride) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        Vals& v = V[k % D];
        if (g + k * kStride < p1) compute(g + k * kStride, v);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {  // mark the set read on every path
#pragma unroll
          for (int i = 0; i < WA; ++i) asm volatile("" ::"v"(v.a[kk][i]));
#pragma unroll
          for (int t = 0; t < WB; ++t) asm volatile("" ::"v"(v.b[kk][t]));
        }
        ld_val(X[k], v);                                 // step + D
        ld_idx(g + (k + D + U) * kStride, X[k]);         // step + D + U
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
          for (int jj = 0; jj < 4; ++jj) {
            float* d = red + (WA * (4 * q + jj) + i) * TN + WB * r + t;
            *d = (w == 0) ? acc[i][t][jj] : (*d + acc[i][t][jj]);
          }
    }
    __syncthreads();
  }
  float* sb = slab + b * (int64_t)c_in * c_out;
  for (int e = threadIdx.x; e < TM * TN; e += kThreads) {
    const int i = e / TN, jn = e % TN;
    sb[(int64_t)(m0 + i) * c_out + n0 + jn] = red[e];
  }
}

// dW tile of the x6 weight gradient: WA in {4, 3, 2, 1} (largest dividing c_in / 16), WB in {2, 1} (registers:
// two value sets of 8 pairs each).
void wgrad_x6_tile(int c_in, int c_out, int& wa, int& wb) {
  const int a = c_in / 16, bb = c_out / 16;
  wa = a % 4 == 0 ? 4 : (a % 3 == 0 ? 3 : (a % 2 == 0 ? 2 : 1));
  wb = bb % 2 == 0 ? 2 : 1;
}

int launch_wgrad_x6(const float* x, int c_in, const float* dy, int c_out, const int32_t* pair_in,
                    const int32_t* pair_out, const int64_t* off_start, int K, int64_t n_pieces, float* slab,
                    hipStream_t s) {
  int WA, WB;
  wgrad_x6_tile(c_in, c_out, WA, WB);
  const int n_ty = (c_in / (16 * WA)) * (c_out / (16 * WB));
  const unsigned grid = (unsigned)(n_pieces * K * n_ty);
#define LW(A, B)                                                                                          \
  if (WA == A && WB == B) {                                                                               \
    wgrad_x6_kernel<A, B><<<grid, kThreads, 0, s>>>(x, c_in, dy, c_out, pair_in, pair_out, off_start, K, \
                                                    n_pieces, n_ty, slab);                               \
    return MSP_OK;                                                                                        \
  }
  LW(1, 1) LW(2, 1) LW(3, 1) LW(4, 1) LW(1, 2) LW(2, 2) LW(3, 2) LW(4, 2)
#undef LW
  return MSP_EINVAL;
}


// Plan (measured on the headline batch's rulebooks, scripts/kbench_x6.py,
// profiles/r01/kbench_x6_*.log): 32-deep k-slices everywhere (fewer
// registers per pipeline slot -> 3 waves per SIMD); NT = 4 output groups per
// block with a single weight buffer (46 KiB of LDS -> 3 blocks per CU) when
// the grid has >= 256 tile x slice blocks, else NT = 3, 4, 2, 1 (first that
// divides) with double-buffered weights.  Small grids split each tile's
// offsets over up to 8 blocks (partials reduced in split order).  Pipeline
// depth 2 (3 and 4 measured no faster).
// Offset split on small grids: aim at 1024 blocks, at most 8 splits; at most 8 tiles (the deepest level, a few
// hundred rows) 2048 blocks and 16 splits (level 6 224 -> 224 0.038 vs 0.042 ms, 448 -> 224 0.055 vs 0.066; the
// wider split lost at level 5's 16 tiles, 0.059 vs 0.048: profiles/r03/kbench_r03_split.log).
PlanX6 plan_x6(int64_t n_rows, int c_out) {
  const int n16 = c_out / 16;
  const int64_t n_tiles = ceil_div(n_rows, 128);
  PlanX6 p{1, 1, 1, 2};
  if (n16 % 4 == 0 && n_tiles * (n16 / 4) >= 256) {
    p.nt = 4;
    p.nb = 1;
  } else {
    for (int nt : {3, 4, 2}) {
      if (n16 % nt == 0) {
        p.nt = nt;
        break;
      }
    }
  }
  p.n_y = n16 / p.nt;
  const int64_t blocks = n_tiles * p.n_y;
  int64_t target = n_tiles <= 8 ? 2048 : 1024, cap = n_tiles <= 8 ? 16 : 8;
#ifdef MSP_EXPERIMENTS  // split sweeps (scripts/kbench.py): MSP_X6D_SPLIT="target_small,cap_small,target,cap"
  if (const char* e = getenv("MSP_X6D_SPLIT")) {
    long v[4] = {2048, 16, 1024, 8};
    sscanf(e, "%ld,%ld,%ld,%ld", &v[0], &v[1], &v[2], &v[3]);
    target = n_tiles <= 8 ? v[0] : v[2];
    cap = n_tiles <= 8 ? v[1] : v[3];
  }
#endif
  if (blocks < target) {
    const int64_t sp = (target + blocks - 1) / blocks;
    p.split = (int)(sp > cap ? cap : sp);
  }
  return p;
}

namespace {
size_t x6_weight_bytes(int K, int c_in, int c_out) {
  const int64_t c_pad = ceil_div(c_in, 32) * 32;
  return (size_t)K * 3 * (size_t)c_out * (size_t)c_pad * 2;
}
size_t round256(size_t b) { return (b + 255) & ~(size_t)255; }
}  // namespace

size_t x6_ws_bytes(int64_t n_rows, int K, int c_in, int c_out, const PlanX6& p) {
  size_t b = round256(x6_weight_bytes(K, c_in, c_out));
  if (p.split > 1) b += (size_t)p.split * (size_t)n_rows * (size_t)c_out * sizeof(float);
  return b;
}

int launch_x6(const PlanX6& p, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
              const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
              const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, hipStream_t s) {
  const int64_t n_tiles = ceil_div(n_rows, 128);
  u32x4* wsp = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)x6_weight_bytes(K, c_in, c_out) / 16;
  if (!(flip & 4))  // bit 2: ws already holds this image (msp_split_weight_images)
    split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, K, c_out, c_in, 16 * p.nt, 32, wsp,
                                                                         (flip >> 1) & 1);
  flip &= 1;
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + round256(x6_weight_bytes(K, c_in, c_out)));
  float* dst = p.split > 1 ? part : out;
  const unsigned grid = (unsigned)(n_tiles * p.n_y * p.split);
  bool launched = false;
#define LD(N, B)                                                                                              \
  if (!launched && p.nt == N && p.nb == B) {                                                                  \
    conv_x6d_kernel<N, 32, 2, 128, 0, B><<<grid, kThreads, 0, s>>>(x, c_in, wsp, K, flip, c_out, tile_start,  \
                                                                   chunk_off, chunk_src, chunk_row, n_rows,  \
                                                                   p.n_y, p.split, dst);                     \
    launched = true;                                                                                          \
  }
  LD(4, 1) LD(4, 2) LD(3, 2) LD(2, 2) LD(1, 2)
#undef LD
  if (!launched) {
    set_error("msp_conv_tile: no x6 kernel for nt=%d nb=%d", p.nt, p.nb);
    return MSP_EINVAL;
  }
  if (p.split > 1) {
    const int64_t n4 = n_rows * c_out / 4;
    split_reduce_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, s>>>(reinterpret_cast<const floatx4*>(part),
                                                                    p.split, n4, reinterpret_cast<floatx4*>(out));
  }
  return MSP_OK;
}

#ifndef MSP_PAIRS_X6_FORM
#define MSP_PAIRS_X6_FORM 2  // runs with the weights in registers: profiles/r06/pairs_bench_r06pb.log
#endif

// form % 10: 0 one chunk per wave, 1 runs of chunks (c_in <= 128), 2 runs with the weights in registers; form / 10:
// the waves the runs are sized for (x 1024; 0 = 8192)
void launch_pairs_x6(int form, const float* x, int c_in, const u32x4* img, int K, int c_out, const int32_t* pair_in,
                     const int32_t* pair_out, const int64_t* off_start, const int64_t* chunk_start, int64_t n_chunks,
                     float* out, hipStream_t s) {
  const int NT = (c_out / 16) % 2 == 0 ? 2 : 1, n_y = c_out / (16 * NT);
  const int kind = form % 10;
  if (kind != 0 && c_in <= 128) {
    const int64_t waves = form / 10 ? (int64_t)(form / 10) * 1024 : 8192;
    int64_t run = n_chunks * n_y / waves;
    run = run < 1 ? 1 : run > 16 ? 16 : run;
    dim3 grid((unsigned)ceil_div(ceil_div(n_chunks, run), kWaves), (unsigned)n_y);
#define PIPE(N, KK, WR)                                                                                          \
  conv_pairs_x6_pipe_kernel<N, KK, WR><<<grid, kThreads, 0, s>>>(x, c_in, img, K, c_out, pair_in, pair_out,     \
                                                                off_start, chunk_start, n_chunks, (int)run, n_y, \
                                                                out)
    const bool wr = kind == 2;
    if (c_in <= 64) {
      if (NT == 2) { if (wr) PIPE(2, 2, true); else PIPE(2, 2, false); }
      else { if (wr) PIPE(1, 2, true); else PIPE(1, 2, false); }
    } else {
      if (NT == 2) { if (wr) PIPE(2, 4, true); else PIPE(2, 4, false); }
      else { if (wr) PIPE(1, 4, true); else PIPE(1, 4, false); }
    }
#undef PIPE
    return;
  }
  dim3 grid((unsigned)ceil_div(n_chunks, kWaves), (unsigned)n_y);
  if (NT == 2)
    conv_pairs_x6_kernel<2><<<grid, kThreads, 0, s>>>(x, c_in, img, K, c_out, pair_in, pair_out, off_start,
                                                      chunk_start, n_chunks, n_y, out);
  else
    conv_pairs_x6_kernel<1><<<grid, kThreads, 0, s>>>(x, c_in, img, K, c_out, pair_in, pair_out, off_start,
                                                      chunk_start, n_chunks, n_y, out);
}

}  // namespace msp

using namespace msp;

extern "C" {

size_t msp_conv_pairs_x6_workspace_size(int K, int c_in, int c_out) {
  return (size_t)K * (size_t)c_out * (size_t)(ceil_div(c_in, 32) * 32) * 6;
}

int msp_conv_pairs_x6(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* pair_in,
                      const int32_t* pair_out, const int64_t* off_start, const int64_t* chunk_start, int64_t n_chunks,
                      float* out, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0 && K >= 1,
              "msp_conv_pairs_x6: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(ws && ws_bytes >= msp_conv_pairs_x6_workspace_size(K, c_in, c_out),
              "msp_conv_pairs_x6: workspace too small");
  if (n_chunks == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  const int NT = (c_out / 16) % 2 == 0 ? 2 : 1, NC = 16 * NT;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)msp_conv_pairs_x6_workspace_size(K, c_in, c_out) / 16;
  split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, K, c_out, c_in, NC, 32, img, 0);
  launch_pairs_x6(MSP_PAIRS_X6_FORM, x, c_in, img, K, c_out, pair_in, pair_out, off_start, chunk_start, n_chunks,
                  out, s);
  return check_launch("msp_conv_pairs_x6");
}

// Dense row-group form on the large levels with c_out >= 64 (measured against msp_conv_tile on the headline
// batch, profiles/r01/kbench_nbr_r01v.log: L0 32->64 -13 %, L1 64->64 -3 %, L2 96->96 -9 %, 192->96 -6 %; the
// narrow per-wave form stays ahead for c_out = 32 and the shared tile below 10^5 rows).  Off since round 5: its
// only remaining call (level 0's 32 -> 64 backward-data; levels 1-4 take the tile-local form) needs the map's
// dense row order, ~0.4 ms of side-stream build per step (a 5-pass radix sort and a permuted copy of the 27 x V
// map), and the per-wave tiles, whose rulebook level 0 builds anyway, now run the call as fast: 50.35-50.42 vs
// 50.43-50.52 ms/step (profiles/r05/ab_r05ag_no_nbr.log).  The kernel stays (msp_conv_nbr, tested directly).
#ifndef MSP_NBR_FORM  // experiments: 1 = the round-1..4 routing above
#define MSP_NBR_FORM 0
#endif
int msp_conv_nbr_preferred(int64_t n_rows, int c_in, int c_out) {
  (void)c_in;
  return MSP_NBR_FORM && n_rows >= 100000 && c_out >= 64 && c_out % 16 == 0 ? 1 : 0;
}

size_t msp_conv_nbr_workspace_size(int K, int c_in, int c_out) {
  if (K <= 0 || c_in <= 0 || c_out <= 0) return 0;
  return x6g_ws_bytes(K, c_in, c_out);
}

int msp_conv_nbr(const float* x, int c_in, const float* wt, int K, int flip, int c_out, const int32_t* nbr,
                 const int32_t* perm, int64_t n_rows, float* out, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_nbr: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= 128, "msp_conv_nbr: K must be in [1, 128] (got %d)", K);
  MSP_REQUIRE(flip >= 0 && flip <= 7, "msp_conv_nbr: flip must be 0..7 (got %d)", flip);
  MSP_REQUIRE(n_rows >= 0, "msp_conv_nbr: n_rows must be >= 0");
  if (n_rows == 0) return MSP_OK;
  MSP_REQUIRE(x && wt && nbr && out, "msp_conv_nbr: null pointer");
  const size_t need = x6g_ws_bytes(K, c_in, c_out);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_nbr: workspace too small (%zu < %zu)", ws_bytes, need);
  const int rc = launch_x6g(x, c_in, wt, K, flip, c_out, nbr, perm, n_rows, out, ws, as_stream(stream));
  return rc ? rc : check_launch("msp_conv_nbr");
}

#ifdef MSP_EXPERIMENTS
int msp_exp_conv_pairs_x6(int variant, const float* x, int c_in, const float* wt, int K, int c_out,
                          const int32_t* pair_in, const int32_t* pair_out, const int64_t* off_start,
                          const int64_t* chunk_start, int64_t n_chunks, float* out, void* ws, size_t ws_bytes,
                          msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0 && K >= 1, "msp_exp_conv_pairs_x6: shape");
  MSP_REQUIRE(ws && ws_bytes >= msp_conv_pairs_x6_workspace_size(K, c_in, c_out), "msp_exp_conv_pairs_x6: ws");
  if (n_chunks == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  const int NT = (c_out / 16) % 2 == 0 ? 2 : 1;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)msp_conv_pairs_x6_workspace_size(K, c_in, c_out) / 16;
  split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, K, c_out, c_in, 16 * NT, 32, img, 0);
  launch_pairs_x6(variant, x, c_in, img, K, c_out, pair_in, pair_out, off_start, chunk_start, n_chunks, out, s);
  return check_launch("msp_exp_conv_pairs_x6");
}

int msp_exp_conv_x6r(int variant, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                     int tile_rows, const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                     const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                     msp_stream_t stream) {
  MSP_REQUIRE(c_out <= 32 && c_in <= 64 && c_in % 16 == 0 && c_out % 16 == 0, "msp_exp_conv_x6r: shape");
  const size_t need = x6p_ws_bytes(K, c_in, c_out) + 1024 + (variant >= 100 ? (size_t)n_rows * c_in * 6 : 0);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_exp_conv_x6r: workspace");
  if (n_rows <= 0) return MSP_OK;
  const int rc = launch_x6r_exp(variant, x, c_in, wt, K, flip, c_out, tile_rows, tile_start, chunk_off, chunk_src,
                                chunk_row, n_rows, out, ws, as_stream(stream));
  return rc ? rc : check_launch("msp_exp_conv_x6r");
}
#endif

}  // extern "C"
