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
// Weights are split once per call into a [K][3][c_out][c_pad] bf16 image
// (c_pad = c_in rounded up to the k-slice, zero padded) by split_weights_
// kernel; the gathered input rows are split in registers (4.5 VALU per value:
// v_cvt_pk_bf16_f32, shift/and back to fp32, v_pk_add_f32).
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
#include "msp_conv_common.h"

namespace msp {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// (a, b) -> packed RNE bf16 pair (v_cvt_pk_bf16_f32), a in the low half
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const floatx2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

__device__ __forceinline__ floatx4 mfma_bf16(const u32x4& a, const u32x4& b, const floatx4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                 0, 0, 0);
}

// 8 consecutive fp32 values -> three bf16x8 pieces, v = p[0] + p[1] + p[2]
__device__ __forceinline__ void split8(const floatx4& a, const floatx4& b, u32x4 (&p)[3]) {
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int s = 0; s < 3; ++s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t h = pk_bf16(v[2 * i], v[2 * i + 1]);
      p[s][i] = h;
      if (s < 2) {
        v[2 * i] -= __uint_as_float(h << 16);
        v[2 * i + 1] -= __uint_as_float(h & 0xffff0000u);
      }
    }
  }
}

// wt [rows = K*c_out][c_in] fp32 -> ws [K][3][c_out][c_pad] bf16 (16-byte
// units of 8 k); k >= c_in is zero.  One thread per unit.
__global__ __launch_bounds__(256) void split_weights_kernel(const float* __restrict__ wt, int64_t rows, int c_out,
                                                            int c_in, int c_pad, u32x4* __restrict__ ws) {
  const int upr = c_pad >> 3;
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= rows * upr) return;
  const int64_t row = u / upr;
  const int k8 = (int)(u - row * upr);
  const int64_t o = row / c_out, n = row - o * c_out;
  u32x4 p[3];
  if (8 * k8 < c_in) {  // c_in % 16 == 0: a unit is all data or all padding
    const floatx4* src = reinterpret_cast<const floatx4*>(wt + row * c_in + 8 * k8);
    split8(src[0], src[1], p);
  } else {
#pragma unroll
    for (int s = 0; s < 3; ++s) p[s] = u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int s = 0; s < 3; ++s) ws[((o * 3 + s) * c_out + n) * upr + k8] = p[s];
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
template <int NT, int KS, int D, int TR>
__global__ __launch_bounds__(kThreads) void conv_x6d_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wsp, int c_pad, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const int32_t* __restrict__ chunk_src, const uint16_t* __restrict__ chunk_row, int64_t n_rows, int n_y,
    int n_split, float* __restrict__ out) {
  static_assert(D >= 2, "the weight slot of step s+1 must differ from step s's");
  constexpr int NC = 16 * NT;
  constexpr int K8 = KS / 8;
  constexpr int NKK = KS / 32;
  constexpr int SWZ = 16 / K8;
  constexpr int WU = 3 * K8 * NC;
  constexpr int SPT = (WU + kThreads - 1) / kThreads;
  constexpr int MJ = TR / (16 * kWaves);
  __shared__ floatx4 acc4[TR * NC / 4];
  __shared__ u32x4 wbuf[2][WU];
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
  // weight staging: per-thread unit offsets are loop constants; a step adds
  // a uniform base (offset, channel slice, k-slice)
  const int upr = c_pad >> 3;
  uint32_t woff[SPT];
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int f = (tid + kThreads * i) < WU ? tid + kThreads * i : WU - 1;
    const int k8 = f % K8, pn = f / K8, n = pn % NC, p = pn / NC;
    woff[i] = (uint32_t)((p * c_out + n) * upr + k8);
  }
  const u32x4* wsp_c = wsp + (int64_t)c0 * upr;
  auto ld_w = [&](const Step& sd, WSt& w) {
    const int ow = flip ? (K - 1 - sd.o) : sd.o;
    const u32x4* wb = wsp_c + ((int64_t)ow * 3 * c_out * upr + sd.ks * K8);
#pragma unroll
    for (int i = 0; i < SPT; ++i) w.u[i] = wb[woff[i]];
  };
  auto st_w = [&](const WSt& w, int buf) {
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int f = tid + kThreads * i;
      const int k8 = f % K8, pn = f / K8, n = pn % NC, p = pn / NC;
      if (f < WU) wbuf[buf][(p * K8 + k8) * NC + (n ^ (SWZ * k8))] = w.u[i];
    }
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
        v.a[j][kk][0] = pv[0];
        v.a[j][kk][1] = pv[1];
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
          if (j < sd.gn) split8(v.a[j][kk][0], v.a[j][kk][1], xp[j]);
        const int k8 = kk * 4 + q;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int un = (16 * t + r) ^ (SWZ * k8);
          const u32x4 w0 = wb[(0 * K8 + k8) * NC + un];
          const u32x4 w1 = wb[(1 * K8 + k8) * NC + un];
          const u32x4 w2 = wb[(2 * K8 + k8) * NC + un];
#pragma unroll
          for (int j = 0; j < MJ; ++j) {
            if (j < sd.gn) {
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
      __syncthreads();  // wbuf[s & 1] holds step s's slice; step s-1's LDS updates are done
      mma(Vd[k], s & 1, V[k]);
      consume_val(V[k]);
      rmw(Vd[k], R[k]);
      consume_row(R[k]);
      st_w(Wr[k1], (s + 1) & 1);  // step s+1's slice (loaded D steps ago)
      ld_w(Sd[k1], Wr[k1]);       // step s+1+D
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

}  // namespace msp

using namespace msp;

namespace msp {

// NT: the widest of 4, 3, 2 dividing the 16-channel output groups (most
// reuse of each gathered and split input row); k-slice 32 for NT = 4 (LDS:
// a 32 KiB accumulator + 2 x 24 KiB weight slices at 64 would not leave room
// for two blocks per CU), 64 otherwise.  Small grids split each tile's
// offsets over up to 8 blocks (partials reduced in split order).  Measured
// on the headline batch (scripts/kbench_x6.py): pipeline depth 2 is as fast
// as 3 or 4.
PlanX6 plan_x6(int64_t n_rows, int c_out, int force_nt, int force_ks) {
  const int n16 = c_out / 16;
  PlanX6 p{1, 64, 1, 1, 2};  // NT = 1 when no wider group count divides (5, 7, ... groups)
  for (int nt : {4, 3, 2}) {
    if (n16 % nt == 0) {
      p.nt = nt;
      break;
    }
  }
  if (force_nt > 0) p.nt = force_nt;
  p.ks = p.nt == 4 ? 32 : 64;
  if (force_ks > 0) p.ks = force_ks;
  p.n_y = n16 / p.nt;
  const int64_t blocks = ceil_div(n_rows, 128) * p.n_y;
  if (blocks < 1024) {
    const int64_t sp = (1024 + blocks - 1) / blocks;
    p.split = (int)(sp > 8 ? 8 : sp);
  }
  return p;
}

namespace {
size_t x6_weight_bytes(int K, int c_in, int c_out, int ks) {
  const int64_t c_pad = ceil_div(c_in, ks) * ks;
  return (size_t)K * 3 * (size_t)c_out * (size_t)c_pad * 2;
}
size_t round256(size_t b) { return (b + 255) & ~(size_t)255; }
}  // namespace

size_t x6_ws_bytes(int64_t n_rows, int K, int c_in, int c_out, const PlanX6& p) {
  size_t b = round256(x6_weight_bytes(K, c_in, c_out, p.ks));
  if (p.split > 1) b += (size_t)p.split * (size_t)n_rows * (size_t)c_out * sizeof(float);
  return b;
}

int launch_x6(const PlanX6& p, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
              const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
              const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, hipStream_t s) {
  const int64_t n_tiles = ceil_div(n_rows, 128);
  const int c_pad = (int)(ceil_div(c_in, p.ks) * p.ks);
  u32x4* wsp = static_cast<u32x4*>(ws);
  const int64_t units = (int64_t)K * c_out * (c_pad / 8);
  split_weights_kernel<<<(unsigned)ceil_div(units, 256), 256, 0, s>>>(wt, (int64_t)K * c_out, c_out, c_in, c_pad,
                                                                      wsp);
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + round256(x6_weight_bytes(K, c_in, c_out, p.ks)));
  float* dst = p.split > 1 ? part : out;
  const unsigned grid = (unsigned)(n_tiles * p.n_y * p.split);
  bool launched = false;
#define LD(N, S, DD)                                                                                          \
  if (!launched && p.nt == N && p.ks == S && p.depth == DD) {                                                 \
    conv_x6d_kernel<N, S, DD, 128><<<grid, kThreads, 0, s>>>(x, c_in, wsp, c_pad, K, flip, c_out, tile_start, \
                                                             chunk_off, chunk_src, chunk_row, n_rows, p.n_y,  \
                                                             p.split, dst);                                   \
    launched = true;                                                                                          \
  }
  LD(1, 64, 2) LD(2, 64, 2) LD(3, 64, 2) LD(4, 32, 2) LD(4, 32, 3) LD(3, 64, 3) LD(2, 64, 3)
#undef LD
  if (!launched) {
    set_error("msp_conv_tile: no x6 kernel for nt=%d ks=%d depth=%d", p.nt, p.ks, p.depth);
    return MSP_EINVAL;
  }
  if (p.split > 1) {
    const int64_t n4 = n_rows * c_out / 4;
    split_reduce_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, s>>>(reinterpret_cast<const floatx4*>(part),
                                                                    p.split, n4, reinterpret_cast<floatx4*>(out));
  }
  return MSP_OK;
}

}  // namespace msp

extern "C" {

// Experiment hook (not part of the public ABI; scripts/kbench_conv.py): the
// x6 shared-tile form with NT / KS forced (0 = the plan's choice).  With
// ws == nullptr returns the workspace bytes needed.
int64_t msp_debug_conv_x6(int nt, int ks, int depth, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                          const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                          const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                          msp_stream_t stream) {
  PlanX6 p = plan_x6(n_rows, c_out, nt, ks);
  if (depth > 0) p.depth = depth;
  MSP_REQUIRE((c_out / 16) % p.nt == 0, "msp_debug_conv_x6: nt %d does not divide c_out/16", p.nt);
  const size_t need = x6_ws_bytes(n_rows, K, c_in, c_out, p);
  if (!ws) return (int64_t)need;
  MSP_REQUIRE(ws_bytes >= need, "msp_debug_conv_x6: workspace too small");
  const int rc = launch_x6(p, x, c_in, wt, K, flip, c_out, tile_start, chunk_off, chunk_src, chunk_row, n_rows, out,
                           ws, as_stream(stream));
  return rc ? rc : check_launch("msp_debug_conv_x6");
}

}  // extern "C"
