// Tile-local submanifold convolution: the input rows a tile of output rows
// needs are staged in LDS once, split into bf16 pieces once, and every rule of
// the tile reads them from there.
//
// Why: in Morton order the 128 output rows of a tile are a small surface patch,
// and their 27-neighbourhoods overlap heavily.  On the headline batch a 128-row
// tile touches 1.6-2.0 x 128 distinct input rows for 7.8-14.9 rules per row
// (scripts/tile_stats.py), so each distinct input row serves 5-7 rules.  The
// gather forms (msp_conv_tile / msp_conv_nbr) fetch and split every rule's row
// from L2/MALL; here a tile fetches each distinct row once, with all its loads
// in flight together, and the rule loop touches only LDS.
//
// Metadata (msp_tile_local, built once per level and reused by the forward and
// the backward-data pass):
//   u_start[t]..u_start[t+1]  the tile's distinct input rows u_rows[], sorted;
//   lidx[o][t*T + i]          position in that list of the neighbour at offset
//                             o of the tile's i-th row (0xFFFF: none);
//   perm[t*T + i]             the tile's i-th row: rows are ordered inside the
//                             tile by their 27-bit neighbour mask, so 16-row
//                             groups share offsets (-1: padding past n).
//
// Kernel (conv_x6s): block = 4 waves on one T-row tile and one 16 NT-wide
// output column slice.  Each wave owns a quarter of the filter offsets
// (o = wave, wave + 4, ...) for ALL the tile's rows, keeping G = T / 16 row
// groups x NT column tiles of accumulators in registers, and loads its own
// weight fragments straight into registers (lane-ordered weight image, two
// steps ahead): no barrier inside the offset loop.  Per (offset, group) the
// wave reads the group's 16 local indices, skips the group when none has the
// offset (wave-uniform ballot), reads the three pre-split pieces of each row
// from LDS and issues 6 NT bf16 MFMAs over the exact splits (the x6 form of
// msp_conv_x6.hip, six piece products summed in a zeroed accumulator and added
// once).  The four waves' partial sums are added in wave order through LDS at
// the end (deterministic).  Input channels are staged 32 at a time.
#include "msp_x6.h"

namespace msp {

constexpr int kLT = 256;          // threads of the metadata kernels
constexpr uint16_t kAbsent = 0xFFFF;
constexpr int kXR = 384;          // LDS rows of a staged 32-channel input slice (last = zero row)
constexpr int kUCap = kXR - 1;    // distinct input rows a tile can stage; more are read from global
constexpr int kXU = 12;           // 16-byte units per staged row: 3 pieces x 4 k-octets
constexpr int kKMax = 27;         // filter volume of the kernel's LDS index tile

// ---------------------------------------------------------------- metadata
template <int N2>
__device__ void bitonic_i32(int32_t* a) {
  for (int k = 2; k <= N2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < N2; i += kLT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const int32_t u = a[i], v = a[ixj];
          if ((u > v) == ((i & k) == 0)) {
            a[i] = v;
            a[ixj] = u;
          }
        }
      }
      __syncthreads();
    }
  }
}

template <int N>
__device__ void bitonic_u64(uint64_t* a) {
  for (int k = 2; k <= N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < N; i += kLT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t u = a[i], v = a[ixj];
          if ((u > v) == ((i & k) == 0)) {
            a[i] = v;
            a[ixj] = u;
          }
        }
      }
      __syncthreads();
    }
  }
}

// The tile's distinct input rows, unordered: its K x T neighbour entries (all loads in flight first) go
// into an open-addressing hash set in LDS (2 N2 int32 slots, load <= 0.42, linear probing by LDS CAS); each
// first insertion appends the row to uq.  Returns the count.  (Round 2 replaced a bitonic sort of all
// N2 entries: a tile names 1.6-2 x T distinct rows of 27 T entries, so sorting only those is ~10x less work.)
template <int T, int N2>
__device__ int tile_distinct(const int32_t* __restrict__ nbr, int K, int64_t n, int64_t t, int32_t* h, int32_t* uq,
                             int* cnt) {
  constexpr int HS = 2 * N2, HB = __builtin_ctz(HS);
  constexpr int PER = N2 / kLT;  // K T <= N2 entries
  for (int i = threadIdx.x; i < HS; i += kLT) h[i] = -1;
  if (threadIdx.x == 0) *cnt = 0;
  int32_t m[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x + kLT * j;
    m[j] = -1;
    if (i < K * T) {
      const int o = i / T, p = i - o * T;
      const int64_t row = t * T + p;
      if (row < n) m[j] = nbr[(int64_t)o * n + row];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int32_t v = m[j];
    if (v < 0) continue;
    uint32_t sl = ((uint32_t)v * 2654435761u) >> (32 - HB);
    while (true) {
      const int32_t prev = atomicCAS(&h[sl], -1, v);
      if (prev == -1) {
        uq[atomicAdd(cnt, 1)] = v;
        break;
      }
      if (prev == v) break;
      sl = (sl + 1) & (HS - 1);
    }
  }
  __syncthreads();
  return *cnt;
}

// ascending bitonic sort of a[0 .. n2) (n2 a power of two, <= N2)
__device__ void bitonic_i32_n(int32_t* a, int n2) {
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n2; i += kLT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const int32_t u = a[i], v = a[ixj];
          if ((u > v) == ((i & k) == 0)) {
            a[i] = v;
            a[ixj] = u;
          }
        }
      }
      __syncthreads();
    }
  }
}

template <int T, int N2>
__global__ __launch_bounds__(kLT) void local_count_kernel(const int32_t* __restrict__ nbr, int K, int64_t n,
                                                          int64_t* __restrict__ cnt,
                                                          unsigned long long* __restrict__ mx) {
  __shared__ int32_t h[2 * N2];
  __shared__ int32_t uq[N2];
  __shared__ int c;
  const int64_t t = blockIdx.x;
  const int tot = tile_distinct<T, N2>(nbr, K, n, t, h, uq, &c);
  if (threadIdx.x == 0) {
    cnt[t] = tot;
    atomicMax(mx, (unsigned long long)tot);
  }
}

template <int T, int N2>
__global__ __launch_bounds__(kLT) void local_fill_kernel(const int32_t* __restrict__ nbr, int K, int64_t n,
                                                         int64_t n_pad, const int64_t* __restrict__ u_start,
                                                         int32_t* __restrict__ u_rows, uint16_t* __restrict__ lidx,
                                                         int32_t* __restrict__ perm, int order) {
  __shared__ int32_t h[2 * N2];
  __shared__ int32_t uq[N2];
  __shared__ uint64_t mk[T];
  __shared__ int c;
  const int64_t t = blockIdx.x;
  const int tot = tile_distinct<T, N2>(nbr, K, n, t, h, uq, &c);
  // the distinct rows in ascending order
  int n2 = 2;
  while (n2 < tot) n2 <<= 1;
  for (int i = tot + threadIdx.x; i < n2; i += kLT) uq[i] = INT32_MAX;
  __syncthreads();
  bitonic_i32_n(uq, n2);
  const int64_t u0 = u_start[t];
  for (int i = threadIdx.x; i < tot; i += kLT) u_rows[u0 + i] = uq[i];
  // rows of the tile ordered by neighbour mask (padding rows last)
  for (int p = threadIdx.x; p < T; p += kLT) {
    const int64_t row = t * T + p;
    uint64_t m = ~0ull >> 8;
    if (row < n) {
      m = 0;
      if (order)
        for (int o = 0; o < K; ++o) m |= (uint64_t)(nbr[(int64_t)o * n + row] >= 0) << o;
    }
    mk[p] = (m << 8) | (uint64_t)p;
  }
  __syncthreads();
  bitonic_u64<T>(mk);
  for (int i = threadIdx.x; i < T; i += kLT) {
    const int64_t row = t * T + (int)(mk[i] & 0xFF);
    perm[t * T + i] = row < n ? (int32_t)row : -1;
  }
  // local index of every (offset, ordered row): binary search in the distinct list
  for (int idx = threadIdx.x; idx < K * T; idx += kLT) {
    const int o = idx / T, i = idx - o * T;
    const int64_t row = t * T + (int)(mk[i] & 0xFF);
    const int32_t v = row < n ? nbr[(int64_t)o * n + row] : -1;
    uint16_t li = kAbsent;
    if (v >= 0) {
      int lo = 0, hi = tot;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (uq[mid] < v) lo = mid + 1;
        else hi = mid;
      }
      li = (uint16_t)lo;
    }
    lidx[(int64_t)o * n_pad + t * T + i] = li;
  }
}

// ---------------------------------------------------------------- weights
// wt -> lane-ordered weight image: unit ((((o * n_y + cy) * nks + ks) * NT + t) * WP + p) * 64 + lane holds,
// for lane = 16 q + r, W^T[out 16 (cy NT + t) + r][k 32 ks + 8 q .. + 7] (zero past c_in) as its three bf16
// pieces p (WP = 3, split once here) or as two fp32 float4 halves p (WP = 2, split by the reader in
// registers: 2/3 of the bytes a step's fragments cost), so a wave loads its fragments of one step as WP NT
// coalesced 1 KiB rows.  wlay 1: wt is [K][c_in][c_out] (the module's layout), else [K][c_out][c_in].
template <int WP>
__global__ __launch_bounds__(256) void split_weights_lane_kernel(const float* __restrict__ wt, int K, int c_out,
                                                                 int c_in, int NT, u32x4* __restrict__ img,
                                                                 int wlay) {
  const int n_y = c_out / (16 * NT), nks = (c_in + 31) / 32;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (o, cy, ks, t, lane)
  if (g >= (int64_t)K * n_y * nks * NT * 64) return;
  const int lane = (int)(g & 63), r = lane & 15, q = lane >> 4;
  int64_t rest = g >> 6;
  const int t = (int)(rest % NT);
  rest /= NT;
  const int ks = (int)(rest % nks);
  rest /= nks;
  const int cy = (int)(rest % n_y);
  const int64_t o = rest / n_y;
  const int oc = 16 * (cy * NT + t) + r, k = 32 * ks + 8 * q;
  floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  if (k < c_in) {  // c_in % 16 == 0: an octet is all data or all padding
    if (wlay) {
      const float* src = wt + (o * c_in + k) * c_out + oc;
      a = floatx4{src[0], src[c_out], src[2 * c_out], src[3 * c_out]};
      b = floatx4{src[4 * c_out], src[5 * c_out], src[6 * c_out], src[7 * c_out]};
    } else {
      const floatx4* src = reinterpret_cast<const floatx4*>(wt + (o * c_out + oc) * c_in + k);
      a = src[0];
      b = src[1];
    }
  }
  u32x4* dst = img + ((g >> 6) * WP) * 64 + lane;
  if constexpr (WP == 3) {
    u32x4 pc[3];
    split8(a, b, pc);
#pragma unroll
    for (int p = 0; p < 3; ++p) dst[p * 64] = pc[p];
  } else {
    dst[0] = __builtin_bit_cast(u32x4, a);
    dst[64] = __builtin_bit_cast(u32x4, b);
  }
}

// a step's weight fragments as the three bf16 pieces the MFMAs take (WP = 2: split here, in registers)
template <int NT, int WP>
__device__ __forceinline__ void weight_pieces(const u32x4 (&w)[NT][WP], u32x4 (&wp)[NT][3]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if constexpr (WP == 3) {
#pragma unroll
      for (int p = 0; p < 3; ++p) wp[t][p] = w[t][p];
    } else {
      split8(__builtin_bit_cast(floatx4, w[t][0]), __builtin_bit_cast(floatx4, w[t][1]), wp[t]);
    }
  }
}

// ---------------------------------------------------------------- convolution
// staged row j of the 32-channel slice: 12 units (piece p, k-octet qq) at p * 4 + (qq ^ ((j >> 2) & 3)):
// the 16 lanes of one ds_read_b128 lane group read 16 rows at their own octet, and the swizzle spreads rows
// j mod 16 over the 16 bank quads
__device__ __forceinline__ int xs_unit(int j, int p, int qq) { return j * kXU + p * 4 + (qq ^ ((j >> 2) & 3)); }

// ABL (timing experiments only, wrong results): bit 1 no weight loads, 2 no LDS input reads, 4 no staging,
// 8 no MFMAs, 16 no index reads (every group active)
template <int NT, int T, int D, int WR, int ABL = 0, int WP = 3, int RI = 0, int XP = 1>
__global__ __launch_bounds__(256 * WR, 2 * WR) void conv_x6s_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const uint16_t* __restrict__ lidx, const int64_t* __restrict__ u_start, const int32_t* __restrict__ u_rows,
    const int32_t* __restrict__ perm, int64_t n_pad, int n_y, float* __restrict__ out) {
  constexpr int NTH = 256 * WR;    // 4 offset classes x WR row parts
  constexpr int G = T / 16 / WR;   // row groups per wave
  constexpr int NC = 16 * NT;
  static_assert(4 * T * NC * 4 <= kXR * kXU * 16, "partial sums must fit the staging area");
  __shared__ u32x4 xs[kXR * kXU];
  __shared__ __attribute__((aligned(16))) uint16_t ls[kKMax * T];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int oc = wave & 3, rp = wave >> 2;  // offset class, row part (rows 16 G rp ..)
  const int r = lane & 15, q = lane >> 4;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int cy = (int)(lb % n_y);
  const int64_t tile = lb / n_y;
  const int64_t u0 = u_start[tile];
  const int U = (int)(u_start[tile + 1] - u0);
  const int Us = U < kUCap ? U : kUCap;
  const int nks = (c_in + 31) / 32;
  if constexpr (RI >= 2) {  // the index tile as 32-bit words, every load in flight before the LDS stores
    constexpr int LW = (kKMax * T / 2 + NTH - 1) / NTH;
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lidx);
    uint32_t wv[LW];
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;  // word i = entries 2i, 2i + 1 of the [K][T] tile (T even: one offset)
      wv[b] = 0u;
      if (i < K * T / 2) {
        const int e = 2 * i, o = e / T, pp = e - o * T;
        wv[b] = lw[((int64_t)o * n_pad + tile * T + pp) >> 1];
      }
    }
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;
      if (i < K * T / 2) reinterpret_cast<uint32_t*>(ls)[i] = wv[b];
    }
  } else {
    for (int i = tid; i < K * T; i += NTH) {
      const int o = i / T, p = i - o * T;
      ls[i] = lidx[(int64_t)o * n_pad + tile * T + p];
    }
  }
  if (tid < kXU) xs[kUCap * kXU + tid] = u32x4{0u, 0u, 0u, 0u};

  // this wave's offsets o = oc + 4 j, j < kNJ (slots past K are empty steps), kNJ per input-channel slice
  constexpr int kNJ = 8;
  const int n_steps = nks * kNJ;
  floatx4 acc[G][NT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto ld_w = [&](int s, u32x4 (&w)[NT][WP]) {
    const int sc = s < n_steps ? s : n_steps - 1;
    const int ks = sc / kNJ, j = sc - ks * kNJ;
    const int o = oc + 4 * j < K ? oc + 4 * j : oc;
    const int ow = flip ? K - 1 - o : o;
    const u32x4* src = wimg + ((((int64_t)ow * n_y + cy) * nks + ks) * NT) * WP * 64 + lane;
    if (ABL & 1) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int p = 0; p < WP; ++p) w[t][p] = u32x4{(uint32_t)(s + t), (uint32_t)p, 0u, 1u};
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int p = 0; p < WP; ++p) w[t][p] = src[(t * WP + p) * 64];
  };
  constexpr int SB = WR == 1 ? 3 : 2;  // staging loads in flight per thread
  // RI: the thread's staged row indices loaded once per tile and kept in registers; every 32-channel slice
  // then issues all of its value loads at once (one global latency per slice instead of index -> value)
  constexpr int MI = (kUCap * 4 + NTH - 1) / NTH;
  int32_t srow[RI ? MI : 1];
  if constexpr (RI != 0) {
#pragma unroll
    for (int b = 0; b < MI; ++b) {
      const int i = tid + NTH * b;
      srow[b] = i < Us * 4 ? u_rows[u0 + (i >> 2)] : 0;
    }
  }
  auto stage_ri = [&](int ks) {
    const int k0 = 32 * ks;
    floatx4 v[MI][2];
#pragma unroll
    for (int b = 0; b < MI; ++b) {
      const int i = tid + NTH * b;
      const int k = k0 + 8 * (i & 3);
      v[b][0] = v[b][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (i < Us * 4 && k < c_in) {
        const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)srow[RI ? b : 0] * c_in + k);
        v[b][0] = src[0];
        v[b][1] = src[1];
      }
    }
#pragma unroll
    for (int b = 0; b < MI; ++b) {
      const int i = tid + NTH * b;
      if (i < Us * 4) {
        u32x4 pc[3];
        split8(v[b][0], v[b][1], pc);
#pragma unroll
        for (int p = 0; p < 3; ++p) xs[xs_unit(i >> 2, p, i & 3)] = pc[p];
      }
    }
  };
  auto stage = [&](int ks) {
    if (ABL & 4) return;
    if constexpr (RI != 0) {
      stage_ri(ks);
      return;
    }
    const int k0 = 32 * ks;
    const int items = Us * 4;
    for (int i0 = tid; i0 < items; i0 += NTH * SB) {
      int32_t rows[SB];
      floatx4 v[SB][2];
#pragma unroll
      for (int b = 0; b < SB; ++b) {
        const int i = i0 + NTH * b;
        rows[b] = i < items ? u_rows[u0 + (i >> 2)] : 0;
      }
#pragma unroll
      for (int b = 0; b < SB; ++b) {
        const int i = i0 + NTH * b;
        const int k = k0 + 8 * (i & 3);
        v[b][0] = v[b][1] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (i < items && k < c_in) {
          const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)rows[b] * c_in + k);
          v[b][0] = src[0];
          v[b][1] = src[1];
        }
      }
#pragma unroll
      for (int b = 0; b < SB; ++b) {
        const int i = i0 + NTH * b;
        if (i < items) {
          u32x4 pc[3];
          split8(v[b][0], v[b][1], pc);
#pragma unroll
          for (int p = 0; p < 3; ++p) xs[xs_unit(i >> 2, p, i & 3)] = pc[p];
        }
      }
    }
  };
  // one (k-slice, offset) step of this wave over the tile's row groups: the 16 local indices of every group
  // first (one LDS wait), the wave-uniform masks of groups with the offset and with rows past the staged
  // capacity, then the groups in order with the next group's three pieces read from LDS before the current
  // group's MFMAs (absent rows read the zero row; inactive groups are read and skipped)
  auto xload = [&](int li, u32x4 (&xp)[3]) {
    const int jr = li < kUCap ? li : kUCap;  // absent (0xFFFF) and far rows -> zero row
    if (ABL & 2) {
#pragma unroll
      for (int p = 0; p < 3; ++p) xp[p] = u32x4{(uint32_t)jr, (uint32_t)p, 7u, 9u};
      return;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) xp[p] = xs[xs_unit(jr, p, q)];
  };
  auto run = [&](int s, const u32x4 (&wl)[NT][WP]) {
    const int ks = s / kNJ, j = s - ks * kNJ;
    const int o = oc + 4 * j;
    if (o >= K) return;  // empty slot (wave-uniform)
    u32x4 w[NT][3];
    weight_pieces<NT, WP>(wl, w);
    const uint16_t* lo = ls + o * T + 16 * G * rp + r;
    int li[G];
#pragma unroll
    for (int g = 0; g < G; ++g) li[g] = (ABL & 16) ? (r + 7 * g + o) : lo[16 * g];
    uint32_t act = 0, far = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool pres = li[g] != kAbsent;
      act |= (ballot64(pres) != 0 ? 1u : 0u) << g;
      far |= (ballot64(pres && li[g] >= kUCap) != 0 ? 1u : 0u) << g;
    }
    u32x4 xa[3], xb[3];  // XP = 0: xb unused
    if (XP) xload(li[0], xa);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4(&cur)[3] = (XP && (g & 1)) ? xb : xa;
      u32x4(&nxt)[3] = (XP && (g & 1)) ? xa : xb;
      if (XP) {
        if (g + 1 < G) xload(li[g + 1], nxt);
      } else if ((act >> g) & 1) {  // XP = 0: the group's pieces read right before its MFMAs (12 fewer VGPRs)
        xload(li[g], cur);
      }
      if ((act >> g) & 1) {  // wave-uniform
        if ((far >> g) & 1) {  // rows past the staged capacity: straight from global memory (rare)
          const bool f = li[g] != kAbsent && li[g] >= kUCap;
          const int k = 32 * ks + 8 * q;
          floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
          if (f && k < c_in) {
            const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)u_rows[u0 + li[g]] * c_in + k);
            a = src[0];
            b = src[1];
          }
          u32x4 fp[3];
          split8(a, b, fp);
#pragma unroll
          for (int p = 0; p < 3; ++p) cur[p] = f ? fp[p] : cur[p];
        }
        floatx4 c[NT];
        if (ABL & 8) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[g][t] += __builtin_bit_cast(floatx4, cur[0] ^ cur[1] ^ cur[2] ^ w[t][0] ^ w[t][1] ^ w[t][2]);
          continue;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][2], cur[0], floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][1], cur[1], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], cur[2], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][1], cur[0], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], cur[1], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], cur[0], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] += c[t];
      }
    }
  };

  static_assert(kNJ % D == 0, "steps per slice must be a multiple of the weight register sets");
  u32x4 wf[D][NT][WP];
#pragma unroll
  for (int d = 0; d < D; ++d) ld_w(d, wf[d]);
  for (int ks = 0; ks < nks; ++ks) {
    __syncthreads();  // previous slice's readers done (and the index tile / zero row written)
    stage(ks);
    __syncthreads();
    for (int j = 0; j < kNJ; j += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int st = ks * kNJ + j + d;
        run(st, wf[d]);
        ld_w(st + D, wf[d]);
      }
    }
  }
  // the four offset classes' partial sums, added in class order
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t)
      *reinterpret_cast<floatx4*>(red + ((int64_t)(oc * T + 16 * (G * rp + g) + r)) * NC + 16 * t + 4 * q) =
          acc[g][t];
  __syncthreads();
  constexpr int QPR = NC / 4;  // float4 quads per row
  for (int i = tid; i < T * QPR; i += NTH) {
    const int row = i / QPR, cq = i - row * QPR;
    const float* pr = red + row * NC + 4 * cq;
    floatx4 v = *reinterpret_cast<const floatx4*>(pr);
#pragma unroll
    for (int w = 1; w < 4; ++w) v += *reinterpret_cast<const floatx4*>(pr + w * T * NC);
    const int32_t dst = perm[tile * T + row];
    if (dst >= 0) *reinterpret_cast<floatx4*>(out + (int64_t)dst * c_out + cy * NC + 4 * cq) = v;
  }
}

// ---------------------------------------------------------------- persistent pipelined form
// conv_x6l: one block of 8 waves per CU (all of its LDS), looping over a contiguous range of work items
// (tile, output column slice); a work item is nks units (32-input-channel slices).  The staging area is
// double buffered: while the waves compute unit u from buffer u & 1, every thread has the next unit's row
// indices, input values and index tile in flight in registers (issued at the start / after the second
// step of unit u) and writes them, split into bf16 pieces, into the other buffer at its end -- the
// staging latency and the per-tile start-up leave the critical path.  Waves = 4 offset classes x 2 column
// halves of the block's 32 NT columns: each wave keeps all 8 row groups of its 16 NT columns in registers
// and loads only its own weight fragments (two steps ahead, across units).  At the end of a work item the
// four offset classes' partial sums meet in LDS in class order (deterministic) and the rows are written
// through the tile's row order.
template <int NT, int WP = 3>
__global__ __launch_bounds__(512, 2) void conv_x6l_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const uint16_t* __restrict__ lidx, const int64_t* __restrict__ u_start, const int32_t* __restrict__ u_rows,
    const int32_t* __restrict__ perm, int64_t n_pad, int n_y, int64_t n_items, float* __restrict__ out) {
  constexpr int T = 128, G = 8, NTH = 512, NCW = 16 * NT, NCB = 2 * NCW;
  constexpr int kNJ = 8;                 // offset slots per wave and unit (o = oc + 4 j; slots past K empty)
  constexpr int SI = (kUCap * 4 + NTH - 1) / NTH;  // staging items (row, k-octet) per thread
  constexpr int LW = (kKMax * T / 2 + NTH - 1) / NTH;  // index-tile words (2 x uint16) per thread
  static_assert(T * NCB * 4 <= kXR * kXU * 16, "the item's sums must fit one staging buffer");
  __shared__ u32x4 xs[2][kXR * kXU];
  __shared__ uint32_t ls[2][kKMax * T / 2];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int oc = wave & 3, ch = wave >> 2;  // offset class, column half
  const int r = lane & 15, q = lane >> 4;
  const int nks = (c_in + 31) / 32;
  // contiguous work items per block (neighbouring tiles share input rows: keep them on one XCD's L2)
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int64_t it0 = lb * n_items / gridDim.x, it1 = (lb + 1) * n_items / gridDim.x;
  const int64_t n_units = (it1 - it0) * nks;
  if (n_units == 0) return;
  auto unit_of = [&](int64_t u, int64_t& tile, int& cy, int& ks) {
    const int64_t it = it0 + u / nks;
    ks = (int)(u % nks);
    cy = (int)(it % n_y);
    tile = it / n_y;
  };

  // ---- staging of a unit: row indices -> values -> split into LDS
  int32_t srow[SI];
  floatx4 sv[SI][2];
  uint32_t slw[LW];
  int s_us = 0;
  int64_t s_u0 = 0;
  auto stage_issue_rows = [&](int64_t u) {  // row indices and the index tile of unit u
    int64_t tile;
    int cy, ks;
    unit_of(u, tile, cy, ks);
    s_u0 = u_start[tile];
    const int U = (int)(u_start[tile + 1] - s_u0);
    s_us = U < kUCap ? U : kUCap;
#pragma unroll
    for (int b = 0; b < SI; ++b) {
      const int i = tid + NTH * b;
      srow[b] = i < s_us * 4 ? u_rows[s_u0 + (i >> 2)] : 0;
    }
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lidx);
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;  // word i = entries 2i, 2i + 1 of the [K][T] tile
      if (i < K * T / 2) {
        const int e = 2 * i, o = e / T, pp = e - o * T;
        slw[b] = lw[((int64_t)o * n_pad + tile * T + pp) >> 1];
      }
    }
  };
  auto stage_issue_values = [&](int64_t u) {
    int64_t tile;
    int cy, ks;
    unit_of(u, tile, cy, ks);
#pragma unroll
    for (int b = 0; b < SI; ++b) {
      const int i = tid + NTH * b;
      const int k = 32 * ks + 8 * (i & 3);
      sv[b][0] = sv[b][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (i < s_us * 4 && k < c_in) {
        const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)srow[b] * c_in + k);
        sv[b][0] = src[0];
        sv[b][1] = src[1];
      }
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int b = 0; b < SI; ++b) {
      const int i = tid + NTH * b;
      if (i < s_us * 4) {
        u32x4 pc[3];
        split8(sv[b][0], sv[b][1], pc);
#pragma unroll
        for (int p = 0; p < 3; ++p) xs[buf][xs_unit(i >> 2, p, i & 3)] = pc[p];
      }
    }
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;
      if (i < K * T / 2) ls[buf][i] = slw[b];
    }
  };

  // ---- weights: step (u, j) -> fragments of offset oc + 4 j, slice ks, columns of this wave
  auto ld_w = [&](int64_t u, int j, u32x4 (&w)[NT][WP]) {
    if (u >= n_units) u = n_units - 1;
    int64_t tile;
    int cy, ks;
    unit_of(u, tile, cy, ks);
    const int o = oc + 4 * j < K ? oc + 4 * j : oc;
    const int ow = flip ? K - 1 - o : o;
    const int cw = 2 * cy + ch;  // this wave's 16 NT-column slice
    const u32x4* src = wimg + ((((int64_t)ow * (2 * n_y) + cw) * nks + ks) * NT) * WP * 64 + lane;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int p = 0; p < WP; ++p) w[t][p] = src[(t * WP + p) * 64];
  };

  floatx4 acc[G][NT];
  int64_t cur_u0 = 0;  // u_start of the unit being computed (rows past the staged capacity)
  auto xload = [&](int buf, int li, u32x4 (&xp)[3]) {
    const int jr = li < kUCap ? li : kUCap;  // absent (0xFFFF) and far rows -> zero row
#pragma unroll
    for (int p = 0; p < 3; ++p) xp[p] = xs[buf][xs_unit(jr, p, q)];
  };
  auto run = [&](int buf, int ks, int j, const u32x4 (&wl)[NT][WP]) {
    const int o = oc + 4 * j;
    if (o >= K) return;  // empty slot (wave-uniform)
    u32x4 w[NT][3];
    weight_pieces<NT, WP>(wl, w);
    const uint16_t* lo = reinterpret_cast<const uint16_t*>(ls[buf]) + o * T + r;
    int li[G];
#pragma unroll
    for (int g = 0; g < G; ++g) li[g] = lo[16 * g];
    uint32_t act = 0, far = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool pres = li[g] != kAbsent;
      act |= (ballot64(pres) != 0 ? 1u : 0u) << g;
      far |= (ballot64(pres && li[g] >= kUCap) != 0 ? 1u : 0u) << g;
    }
    u32x4 xa[3], xb[3];
    xload(buf, li[0], xa);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4(&cur)[3] = (g & 1) ? xb : xa;
      u32x4(&nxt)[3] = (g & 1) ? xa : xb;
      if (g + 1 < G) xload(buf, li[g + 1], nxt);
      if ((act >> g) & 1) {  // wave-uniform
        if ((far >> g) & 1) {  // rows past the staged capacity: straight from global memory (rare)
          const bool f = li[g] != kAbsent && li[g] >= kUCap;
          const int k = 32 * ks + 8 * q;
          floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
          if (f && k < c_in) {
            const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)u_rows[cur_u0 + li[g]] * c_in + k);
            a = src[0];
            b = src[1];
          }
          u32x4 fp[3];
          split8(a, b, fp);
#pragma unroll
          for (int p = 0; p < 3; ++p) cur[p] = f ? fp[p] : cur[p];
        }
        floatx4 c[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][2], cur[0], floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][1], cur[1], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], cur[2], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][1], cur[0], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], cur[1], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], cur[0], c[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] += c[t];
      }
    }
  };

  // ---- prologue: unit 0 staged synchronously, zero rows of both buffers
  stage_issue_rows(0);
  stage_issue_values(0);
  stage_store(0);
  if (tid < 2 * kXU) xs[tid / kXU][kUCap * kXU + tid % kXU] = u32x4{0u, 0u, 0u, 0u};
  u32x4 wf[2][NT][WP];
  ld_w(0, 0, wf[0]);
  ld_w(0, 1, wf[1]);
  __syncthreads();

  for (int64_t u = 0; u < n_units; ++u) {
    const int buf = (int)(u & 1);
    int64_t tile;
    int cy, ks;
    unit_of(u, tile, cy, ks);
    cur_u0 = u_start[tile];
    const bool more = u + 1 < n_units;
    if (more) stage_issue_rows(u + 1);
    if (ks == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < kNJ; j += 2) {
      run(buf, ks, j, wf[0]);
      ld_w(j + 2 < kNJ ? u : u + 1, (j + 2) % kNJ, wf[0]);
      run(buf, ks, j + 1, wf[1]);
      ld_w(j + 3 < kNJ ? u : u + 1, (j + 3) % kNJ, wf[1]);
      if (j == 2 && more) stage_issue_values(u + 1);
    }
    if (more) stage_store(buf ^ 1);
    __syncthreads();  // unit u's reads of buffer buf done; unit u + 1 staged in buf ^ 1
    if (ks == nks - 1) {
      // the item's sums: offset classes 0..3 add into buffer buf in order, then rows are written out
      float* red = reinterpret_cast<float*>(xs[buf]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (oc == c) {
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              floatx4* dst = reinterpret_cast<floatx4*>(red + (16 * g + r) * NCB + ch * NCW + 16 * t + 4 * q);
              *dst = c == 0 ? acc[g][t] : *dst + acc[g][t];
            }
        }
        __syncthreads();
      }
      constexpr int QPR = NCB / 4;
      for (int i = tid; i < T * QPR; i += NTH) {
        const int row = i / QPR, cq = i - row * QPR;
        const int32_t dst = perm[tile * T + row];
        if (dst >= 0)
          *reinterpret_cast<floatx4*>(out + (int64_t)dst * c_out + cy * NCB + 4 * cq) =
              *reinterpret_cast<const floatx4*>(red + row * NCB + 4 * cq);
      }
      __syncthreads();  // buffer buf is free for the unit after next
    }
  }
}

// ---------------------------------------------------------------- tile-local weight gradient
// dW[o][ci][co] = sum over rows i of x[nbr(i, o)][ci] dy[i][co] (submanifold, the forward's [K][c_in][c_out]
// layout), over the same tile-local rulebook.  The pair-list form (msp_conv_wgrad) gathers x and dy per
// rule from global memory and, at levels 0-1, refetches them 7-8x from past L2 (profiles/r01/
// pmc_wgrad_pieces_r01zz.txt); here each tile's distinct x rows and its 128 dy rows are staged in LDS once
// (split into bf16 pieces once) and every offset's rules read them from there.
// Block = 8 waves, persistent over a contiguous range of tiles for one 32 x 32 (input x output channel)
// slice of dW; wave w owns offsets w, w + 8, w + 16, w + 24 (< K) and keeps their 32 x 32 slices in
// registers over the whole range.  MFMA k = 32 tile rows: lane (r, q) reads, for rows 8q .. 8q+7 of the
// step, the bf16 pair (channels 2r, 2r+1) of each piece -- the 16 lanes of a row read 64 contiguous bytes --
// and assembles the A (x, m-tile sa = channel parity) and B (dy, n-tile sb) fragments with byte permutes;
// accumulator [o][sa][sb] register jj holds dW[o][ci0 + 2 (4q + jj) + sa][co0 + 2 r + sb].  The next tile's
// rows are loaded into registers while the current one is computed.  Per range a slab of partial dW is
// written; msp_conv_wgrad_local adds the ranges in order (deterministic).
__device__ __forceinline__ uint32_t lo16x2(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ uint32_t hi16x2(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

__global__ __launch_bounds__(512, 2) void wgrad_x6t_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out, const uint16_t* __restrict__ lidx,
    const int64_t* __restrict__ u_start, const int32_t* __restrict__ u_rows, const int32_t* __restrict__ perm,
    int K, int64_t n_tiles, int64_t n_pad, int n_ranges, float* __restrict__ slab) {
  constexpr int T = 128, NTH = 512, NOW = 4;  // offsets per wave (K <= 32 over 8 waves)
  constexpr int SI = (kUCap * 4 + NTH - 1) / NTH;
  constexpr int LW = (kKMax * T / 2 + NTH - 1) / NTH;
  constexpr int DYU = T * kXU;  // dy stage: T rows x 12 units
  __shared__ u32x4 xs[kXR * kXU];
  __shared__ u32x4 ds[DYU];
  __shared__ uint32_t ls[kKMax * T / 2];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int n_sl_o = c_out / 32;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int slice = (int)(lb % ((c_in / 32) * n_sl_o));
  const int range = (int)(lb / ((c_in / 32) * n_sl_o));
  const int ci0 = 32 * (slice / n_sl_o), co0 = 32 * (slice % n_sl_o);
  const int64_t t0 = (int64_t)range * n_tiles / n_ranges, t1 = (int64_t)(range + 1) * n_tiles / n_ranges;

  floatx4 acc[NOW][2][2];
#pragma unroll
  for (int a = 0; a < NOW; ++a)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[a][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // staging registers of one tile: x rows (SI items of 8 channels), dy row (1 item), index-tile words
  int32_t srow[SI];
  floatx4 sv[SI][2], dv[2];
  uint32_t slw[LW];
  int s_us = 0;
  auto issue_rows = [&](int64_t t) {
    const int64_t u0 = u_start[t];
    const int U = (int)(u_start[t + 1] - u0);
    s_us = U < kUCap ? U : kUCap;
#pragma unroll
    for (int b = 0; b < SI; ++b) {
      const int i = tid + NTH * b;
      srow[b] = i < s_us * 4 ? u_rows[u0 + (i >> 2)] : 0;
    }
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lidx);
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;
      if (i < K * T / 2) {
        const int e = 2 * i, o = e / T, pp = e - o * T;
        slw[b] = lw[((int64_t)o * n_pad + t * T + pp) >> 1];
      }
    }
  };
  auto issue_values = [&](int64_t t) {
#pragma unroll
    for (int b = 0; b < SI; ++b) {
      const int i = tid + NTH * b;
      sv[b][0] = sv[b][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (i < s_us * 4) {
        const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)srow[b] * c_in + ci0 + 8 * (i & 3));
        sv[b][0] = src[0];
        sv[b][1] = src[1];
      }
    }
    // dy: ordered row tid >> 2 of the tile, channel octet tid & 3 (T * 4 = NTH items)
    const int32_t dr = perm[t * T + (tid >> 2)];
    dv[0] = dv[1] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (dr >= 0) {
      const floatx4* src = reinterpret_cast<const floatx4*>(dy + (int64_t)dr * c_out + co0 + 8 * (tid & 3));
      dv[0] = src[0];
      dv[1] = src[1];
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int b = 0; b < SI; ++b) {
      const int i = tid + NTH * b;
      if (i < s_us * 4) {
        u32x4 pc[3];
        split8(sv[b][0], sv[b][1], pc);
#pragma unroll
        for (int p = 0; p < 3; ++p) xs[xs_unit(i >> 2, p, i & 3)] = pc[p];
      }
    }
    {
      u32x4 pc[3];
      split8(dv[0], dv[1], pc);
#pragma unroll
      for (int p = 0; p < 3; ++p) ds[xs_unit(tid >> 2, p, tid & 3)] = pc[p];
    }
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;
      if (i < K * T / 2) ls[i] = slw[b];
    }
  };
  // the bf16 pair (channels 2r, 2r+1) of piece p of staged row j
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(xs);
  const uint32_t* dw = reinterpret_cast<const uint32_t*>(ds);
  auto word = [&](const uint32_t* base, int j, int p) {
    return base[xs_unit(j, p, r >> 2) * 4 + (r & 3)];
  };
  // fragments of 8 rows: f[s][p] = channel parity s of piece p over the rows, packed as 8 bf16
  auto frags = [&](const uint32_t (&w)[8][3], u32x4 (&f)[2][3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        f[0][p][h] = lo16x2(w[2 * h][p], w[2 * h + 1][p]);
        f[1][p][h] = hi16x2(w[2 * h][p], w[2 * h + 1][p]);
      }
  };

  if (t0 < t1) {
    issue_rows(t0);
    issue_values(t0);
    if (tid < kXU) xs[kUCap * kXU + tid] = u32x4{0u, 0u, 0u, 0u};
    store();
    __syncthreads();
    for (int64_t t = t0; t < t1; ++t) {
      const bool more = t + 1 < t1;
      if (more) issue_rows(t + 1);
      const uint16_t* lt = reinterpret_cast<const uint16_t*>(ls);
#pragma unroll
      for (int kk = 0; kk < T / 32; ++kk) {
        if (kk == 1 && more) issue_values(t + 1);
        const int rb = 32 * kk + 8 * q;  // this lane's 8 tile rows
        uint32_t wd[8][3];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int p = 0; p < 3; ++p) wd[j][p] = word(dw, rb + j, p);
        u32x4 bf[2][3];
        frags(wd, bf);
#pragma unroll
        for (int a = 0; a < NOW; ++a) {
          const int o = wave + 8 * a;
          if (o >= K) break;  // wave-uniform
          int li[8];
          bool any = false;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            li[j] = lt[o * T + rb + j];
            any |= li[j] != kAbsent;
          }
          if (ballot64(any) == 0) continue;  // no row of the 32 has this offset
          uint32_t wx[8][3];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int jr = li[j] < kUCap ? li[j] : kUCap;
#pragma unroll
            for (int p = 0; p < 3; ++p) wx[j][p] = word(xw, jr, p);
          }
          bool farj = false;
#pragma unroll
          for (int j = 0; j < 8; ++j) farj |= li[j] >= kUCap && li[j] != kAbsent;
          if (ballot64(farj)) {
            // rows past the staged capacity (rare): their pair straight from global memory, split here
            const int64_t u0 = u_start[t];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if (li[j] >= kUCap && li[j] != kAbsent) {
                const float2 v = *reinterpret_cast<const float2*>(x + (int64_t)u_rows[u0 + li[j]] * c_in + ci0 + 2 * r);
                float a0 = v.x, a1 = v.y;
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                  const uint32_t h = pk_bf16(a0, a1);
                  wx[j][p] = h;
                  a0 -= __uint_as_float(h << 16);
                  a1 -= __uint_as_float(h & 0xffff0000u);
                }
              }
            }
          }
          u32x4 af[2][3];
          frags(wx, af);
#pragma unroll
          for (int sa = 0; sa < 2; ++sa)
#pragma unroll
            for (int sb = 0; sb < 2; ++sb) {
              floatx4 c = mfma_bf16(af[sa][2], bf[sb][0], floatx4{0.f, 0.f, 0.f, 0.f});
              c = mfma_bf16(af[sa][1], bf[sb][1], c);
              c = mfma_bf16(af[sa][0], bf[sb][2], c);
              c = mfma_bf16(af[sa][1], bf[sb][0], c);
              c = mfma_bf16(af[sa][0], bf[sb][1], c);
              acc[a][sa][sb] += mfma_bf16(af[sa][0], bf[sb][0], c);
            }
        }
      }
      __syncthreads();  // reads of tile t done
      if (more) store();
      __syncthreads();
    }
  }
  // partial dW of this range: slab[range][o][ci][co]
  float* sb = slab + (int64_t)range * K * c_in * c_out;
#pragma unroll
  for (int a = 0; a < NOW; ++a) {
    const int o = wave + 8 * a;
    if (o >= K) break;
#pragma unroll
    for (int sa = 0; sa < 2; ++sa)
#pragma unroll
      for (int sbb = 0; sbb < 2; ++sbb)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          sb[((int64_t)o * c_in + ci0 + 2 * (4 * q + jj) + sa) * c_out + co0 + 2 * r + sbb] = acc[a][sa][sbb][jj];
  }
}

// dW[e] = sum over ranges in order of slab[range][e]
__global__ __launch_bounds__(256) void wgrad_ranges_reduce_kernel(const floatx4* __restrict__ slab, int n_ranges,
                                                                  int64_t n4, floatx4* __restrict__ dw) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  floatx4 s = slab[i];
  for (int k = 1; k < n_ranges; ++k) s += slab[(int64_t)k * n4 + i];
  dw[i] = s;
}

// ---------------------------------------------------------------- chunk-local convolution (narrow levels)
// Level 0 of the m = 32 UNet has 32 channels and 7.7 rules per row: the dense 16-row groups of conv_x6s fill
// 0.37 of their MFMA rows there, and the per-wave gather tiles (conv_x6r) fetch every rule's row from L2/MALL
// (1.3 GB per call) and stall on that latency.  This form keeps the compacted chunks of the tile rulebook
// (16 rules of one offset per chunk: 0.71 of the MFMA rows carry a rule with 64-row tiles) but reads their
// input rows from LDS: a 128-row unit (two 64-row rulebook tiles) stages its distinct input rows once per 32
// input channels (fp32, 1.57 x 128 rows on average), and the chunks scatter their 16 x 32 partial products into
// fp32 accumulators in LDS.
//
// Metadata (msp_chunk_local, from the 64-row tile rulebook): per unit the sorted distinct input rows of its
// chunks (first kQCap of them), and per chunk entry a packed word: position in that list (0xFFFF past kQCap:
// read from global memory) | row inside the unit << 16 (128: padding slot).
//
// Kernel (conv_x6q): block = 4 waves on one unit and 32 output columns; wave (h, c) takes half h's chunks
// (tile 2 unit + h), class c = the first or second half of that tile's chunk list.  The two classes own
// separate accumulators (rows of one class never meet in two waves at once: chunks of one offset name
// distinct rows, and a class is processed in order by one wave per half); they are added in class order at
// the end, so results are deterministic.  Weights: the lane-ordered split image of split_weights_lane_kernel,
// one register set per offset run, the next two runs' sets loaded ahead.
constexpr int kQT = 64;        // rulebook tile rows (half a unit)
constexpr int kQUnit = 128;    // rows of a unit
constexpr int kQCap = 320;     // staged distinct rows per unit (slot kQCap: zero row)
constexpr uint32_t kQFar = 0xFFFFu;
constexpr int kWCap = 448;     // distinct rows per 128-row tile the weight gradient stages (msp_conv_wgrad_chunk)

// staged row j (32 fp32 channels = 8 16-byte units): unit u at j*8 + (u ^ ((j >> 1) & 7)) -- the 16 distinct
// rows j mod 16 of one ds_read_b128 lane group land on 16 distinct bank quads at a fixed u
__device__ __forceinline__ int xq_unit(int j, int u) { return j * 8 + (u ^ ((j >> 1) & 7)); }
// accumulator row (AU 16-byte units): the same spreading for AU = 8 (32 columns) and AU = 4 (16 columns)
template <int AU>
__device__ __forceinline__ int aq_unit(int row, int u) {
  return row * AU + (u ^ ((row >> (AU == 8 ? 1 : 2)) & (AU - 1)));
}

// unit = TPU rulebook tiles of TR rows (TPU * TR = 128); list capacity cap per unit; largest count -> *mx
template <int N2, int TPU, int TR>
__global__ __launch_bounds__(kLT) void chunk_local_kernel(const int64_t* __restrict__ tile_start, int64_t n_tiles,
                                                          const int32_t* __restrict__ chunk_src,
                                                          const uint16_t* __restrict__ chunk_row, int cap,
                                                          int32_t* __restrict__ u_rows, int32_t* __restrict__ u_cnt,
                                                          uint32_t* __restrict__ chunk_lr,
                                                          unsigned long long* __restrict__ mx) {
  constexpr int PER = N2 / kLT;
  static_assert(TPU * TR == kQUnit, "a unit is 128 rows");
  __shared__ int32_t a[N2];
  __shared__ int32_t uq[N2];
  const int64_t u = blockIdx.x;
  const int64_t t0 = TPU * u, t1 = t0 + 1 < n_tiles ? t0 + TPU : t0 + 1;
  const int64_t e0 = tile_start[t0] * MSP_CHUNK, e1 = tile_start[t1] * MSP_CHUNK;
  const int64_t emid = tile_start[t0 + 1] * MSP_CHUNK;  // first entry of the second tile
  const int ne = (int)(e1 - e0);                        // <= N2 (host checks the largest tile)
  for (int i = threadIdx.x; i < N2; i += kLT) a[i] = i < ne ? chunk_src[e0 + i] : INT32_MAX;
  __syncthreads();
  bitonic_i32<N2>(a);
  const int base = threadIdx.x * PER;
  int c = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = base + j;
    c += a[i] != INT32_MAX && (i == 0 || a[i] != a[i - 1]);
  }
  int tot;
  int off = block_excl_scan<kLT>(c, &tot);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = base + j;
    if (a[i] != INT32_MAX && (i == 0 || a[i] != a[i - 1])) {
      uq[off] = a[i];
      if (off < cap) u_rows[u * cap + off] = a[i];
      ++off;
    }
  }
  for (int j = tot + threadIdx.x; j < cap; j += kLT) u_rows[u * cap + j] = -1;  // unused slots: -1
  if (threadIdx.x == 0) {
    u_cnt[u] = tot;
    if (mx) atomicMax(mx, (unsigned long long)tot);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ne; i += kLT) {
    const int64_t e = e0 + i;
    const int32_t v = chunk_src[e];
    int lo = 0, hi = tot;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (uq[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    const int rt = chunk_row[e];
    const uint32_t row = rt >= TR ? (uint32_t)kQUnit : (uint32_t)(rt + (TPU == 2 && e >= emid ? TR : 0));
    chunk_lr[e] = (lo < cap ? (uint32_t)lo : kQFar) | (row << 16);
  }
}

// Weight-gradient index from the tile-local rulebook (msp_tile_local, 128-row tiles): the tile's sorted
// distinct input rows are already listed there, so each chunk entry of the 128-row tile rulebook only needs its
// position in that list (binary search; rows past the list's staged capacity are excluded on the host).
__global__ __launch_bounds__(kLT) void chunk_lidx_kernel(const int64_t* __restrict__ tile_start,
                                                         const int32_t* __restrict__ chunk_src,
                                                         const uint16_t* __restrict__ chunk_row,
                                                         const int64_t* __restrict__ u_start,
                                                         const int32_t* __restrict__ u_rows,
                                                         uint32_t* __restrict__ chunk_lr) {
  __shared__ int32_t uq[kWCap];
  const int64_t t = blockIdx.x;
  const int64_t u0 = u_start[t];
  const int U = (int)(u_start[t + 1] - u0);
  const int Us = U < kWCap ? U : kWCap;
  for (int i = threadIdx.x; i < Us; i += kLT) uq[i] = u_rows[u0 + i];
  __syncthreads();
  const int64_t e0 = tile_start[t] * MSP_CHUNK, e1 = tile_start[t + 1] * MSP_CHUNK;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kLT) {
    const int32_t v = chunk_src[e];
    int lo = 0, hi = Us;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (uq[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    const int rt = chunk_row[e];
    chunk_lr[e] = (uint32_t)(lo < Us ? lo : kQFar) | ((uint32_t)(rt >= kQUnit ? kQUnit : rt) << 16);
  }
}

// DV: value lead (chunks; indices lead by 2 DV).  NT = 2: 32 output columns per block.
// ABL (timing experiments only, wrong results): 1 no staging loads, 2 no index loads, 4 no accumulator reads,
// 8 no MFMAs, 16 no weight loads.
template <int NT, int DV, int ABL = 0>
__global__ __launch_bounds__(256) void conv_x6q_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const uint32_t* __restrict__ chunk_lr, const int32_t* __restrict__ chunk_src,
    const int32_t* __restrict__ u_rows, const int32_t* __restrict__ u_cnt, int64_t n_rows, int64_t n_tiles, int n_y,
    float* __restrict__ out) {
  constexpr int NC = 16 * NT, AU = NC / 4, AR = kQUnit + 1;  // accumulator rows per class (+ padding row)
  constexpr int SR = (kQCap * 8 + 255) / 256;                // staging items per thread
  __shared__ floatx4 xs[(kQCap + 1) * 8];
  __shared__ floatx4 as[2 * AR * AU];
  __shared__ int runs_s[4][32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = wave >> 1, cls = wave & 1;
  const int r = lane & 15, q = lane >> 4;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int cy = (int)(lb % n_y);
  const int64_t unit = lb / n_y;
  const int nks = (c_in + 31) / 32;

  // this wave's chunk range: the first or second half of its tile's list
  const int64_t tix = 2 * unit + h;
  int64_t wb = 0, we = 0;
  if (tix < n_tiles) {
    const int64_t cb = tile_start[tix], ce = tile_start[tix + 1];
    const int64_t mid = cb + (ce - cb + 1) / 2;
    wb = cls ? mid : cb;
    we = cls ? ce : mid;
  }
  const int n = (int)(we - wb);

  // staging rows of this thread, the same for every k-slice (-1: slot past the unit's list)
  static_assert(SR * 256 == kQCap * 8, "staging items must cover the list exactly");
  int32_t srow[SR];
#pragma unroll
  for (int b = 0; b < SR; ++b) srow[b] = u_rows[unit * kQCap + ((tid + 256 * b) >> 3)];
  for (int i = tid; i < 2 * AR * AU; i += 256) as[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (tid < 8) xs[kQCap * 8 + tid] = floatx4{0.f, 0.f, 0.f, 0.f};

  // offset runs of the wave's range: (first chunk << 8) | offset, at most K <= 27 (chunks sorted by offset)
  int n_runs = 0;
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const int ic = i < n ? i : n - 1;
    const int o = chunk_off[wb + ic];
    const int op = chunk_off[wb + (ic > 0 ? ic - 1 : 0)];
    const bool st = i < n && (i == 0 || o != op);
    const unsigned long long m = ballot64(st);
    const int pos = n_runs + mbcnt64(m);
    if (st && pos < 32) runs_s[wave][pos] = (i << 8) | o;
    n_runs += __popcll(m);
  }
  __syncthreads();  // runs, zeroed accumulators and zero row visible
  const int nr_c = n_runs > 0 ? n_runs : 1;
  const int run_l = n_runs > 0 ? runs_s[wave][lane < n_runs ? lane : n_runs - 1] : 0;
  auto run_at = [&](int j) -> int { return __builtin_amdgcn_readlane(run_l, j < nr_c ? j : nr_c - 1); };
  auto start_of = [&](int j) -> int { return j < n_runs ? (run_at(j) >> 8) : (1 << 22); };

  struct Wt {
    u32x4 w[NT][3];
  };
  auto ld_w = [&](int j, int ks, Wt& w) {
    const int o = run_at(j) & 255;
    if (ABL & 16) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) w.w[t][p] = u32x4{(uint32_t)(o + t), (uint32_t)p, 3u, 1u};
      return;
    }
    const int ow = flip ? (K - 1 - o) : o;
    const u32x4* src = wimg + ((((int64_t)ow * n_y + cy) * nks + ks) * NT) * 3 * 64 + lane;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) w.w[t][p] = src[(t * 3 + p) * 64];
  };
  struct Val {
    floatx4 a[2];
    int row;
  };
  // last chunk a (clamped) look-ahead may read: an existing entry even for an empty range
  const int64_t clast = we > wb ? we - 1 : (wb > 0 ? wb - 1 : 0);
  auto ld_idx = [&](int i) -> uint32_t {  // chunk wb + i (clamped)
    const int64_t c = wb + i < clast ? wb + i : clast;
    if (ABL & 2) return (uint32_t)((r * 13 + i * 7) & 127) | ((uint32_t)(4 * r + (i & 3)) << 16);
    return chunk_lr[c * MSP_CHUNK + r];
  };
  auto ld_val = [&](uint32_t lr, int i, int ks, Val& v) {
    const int li = (int)(lr & 0xFFFFu);
    const int j = li < kQCap ? li : kQCap;
    v.a[0] = xs[xq_unit(j, 2 * q)];
    v.a[1] = xs[xq_unit(j, 2 * q + 1)];
    v.row = (int)(lr >> 16);
    if (ballot64(li == (int)kQFar) != 0) {  // rows past the staged capacity: from global memory (rare)
      const int64_t c = wb + i < clast ? wb + i : clast;
      const int k = 32 * ks + 8 * q;
      if (li == (int)kQFar && k < c_in) {
        const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)chunk_src[c * MSP_CHUNK + r] * c_in + k);
        v.a[0] = src[0];
        v.a[1] = src[1];
      }
    }
  };
  floatx4* acc = as + cls * AR * AU;
  // the accumulator rows of the next chunk are read right after this chunk's write (LDS operations of a wave
  // complete in order: the read sees the write) and before the next look-ahead row reads, so waiting for them
  // never waits for the look-ahead
  auto rd_old = [&](int row, floatx4 (&old)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
      old[t] = (ABL & 4) ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[aq_unit<AU>(row, 4 * t + q)];
  };
  auto run = [&](const Val& v, const Wt& w, const floatx4 (&old)[NT]) {
    u32x4 xp[3];
    split8(v.a[0], v.a[1], xp);
    floatx4 c[NT];
    if (ABL & 8) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[aq_unit<AU>(v.row, 4 * t + q)] =
            old[t] + __builtin_bit_cast(floatx4, xp[0] ^ xp[1] ^ xp[2] ^ w.w[t][0] ^ w.w[t][1] ^ w.w[t][2]);
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w.w[t][2], xp[0], floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w.w[t][1], xp[1], c[t]);
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w.w[t][0], xp[2], c[t]);
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w.w[t][1], xp[0], c[t]);
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w.w[t][0], xp[1], c[t]);
#pragma unroll
    for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w.w[t][0], xp[0], c[t]);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[aq_unit<AU>(v.row, 4 * t + q)] = old[t] + c[t];
  };

  constexpr int DI = 2 * DV;  // indices lead their values by DV chunks
  for (int ks = 0; ks < nks; ++ks) {
    // this slice's first indices and weights go out before the staging loads
    uint32_t I[DV];
#pragma unroll
    for (int k = 0; k < DV; ++k) I[k] = ld_idx(k);
    Wt Wc, Wn, Wm;
    ld_w(0, ks, Wc);
    ld_w(1, ks, Wn);
    ld_w(2, ks, Wm);
    if (ks > 0) __syncthreads();  // previous slice's row reads done
    {
      const int k0 = 32 * ks;
      floatx4 v[SR];
#pragma unroll
      for (int b = 0; b < SR; ++b) {
        const int i = tid + 256 * b;
        const int k = k0 + 4 * (i & 7);
        v[b] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (!(ABL & 1) && srow[b] >= 0 && k < c_in) v[b] = *reinterpret_cast<const floatx4*>(x + (int64_t)srow[b] * c_in + k);
      }
#pragma unroll
      for (int b = 0; b < SR; ++b) {
        const int i = tid + 256 * b;
        if (srow[b] >= 0) xs[xq_unit(i >> 3, i & 7)] = v[b];
      }
    }
    __syncthreads();
    if (n > 0) {  // wave-uniform
      Val S[DV];
      floatx4 old[NT];
#pragma unroll
      for (int k = 0; k < DV; ++k) {
        ld_val(I[k], k, ks, S[k]);
        I[k] = ld_idx(DV + k);
      }
      rd_old(S[0].row, old);
      int rho = 0, next_start = start_of(1);
      for (int c = 0; c < n; c += DV) {
#pragma unroll
        for (int k = 0; k < DV; ++k) {
          const int i = c + k;
          if (i == next_start) {  // first chunk of run rho + 1
            ++rho;
            next_start = start_of(rho + 1);
            Wc = Wn;
            Wn = Wm;
            ld_w(rho + 2, ks, Wm);
          }
          if (i < n) run(S[k], Wc, old);
          rd_old(S[(k + 1) % DV].row, old);  // chunk i + 1
          ld_val(I[k], i + DV, ks, S[k]);
          I[k] = ld_idx(i + DI);
        }
      }
    }
  }
  __syncthreads();
  const int64_t row0 = unit * kQUnit;
  for (int i = tid; i < kQUnit * AU; i += 256) {
    const int row = i / AU, u = i % AU;
    if (row0 + row < n_rows) {
      const floatx4 v = as[aq_unit<AU>(row, u)] + as[AR * AU + aq_unit<AU>(row, u)];
      *reinterpret_cast<floatx4*>(out + (row0 + row) * c_out + cy * NC + 4 * u) = v;
    }
  }
}

// ---------------------------------------------------------------- chunk-local weight gradient
// dW[o][ci][co] = sum over the rules (i, j) of offset o of x[i][ci] dy[j][co], over the 128-row tile rulebook.
// The pair-list form (wgrad_x6_kernel) gathers x and dy per rule from L2/MALL (7-8x the compulsory bytes at
// levels 0-1) and splits every gathered value per use; the dense tile-local form (wgrad_x6t_kernel) staged
// the rows once but ran 32-row k-steps with ~45 % zero rows.  Here a tile's distinct x rows and its 128 dy rows
// are staged in LDS once per 32 x 32 channel slice as three bf16 piece images ([row][32 channels], 8-byte
// units XOR-spread by row bit 2), and the k-steps are the compacted chunks of the rulebook: two 16-rule chunks
// of one offset per 32-deep MFMA step (an odd last chunk is paired with the zero row).  The MFMA operands
// (A = x^T, B = dy^T: 8 consecutive rules of one channel per lane) come straight out of the gathered rows with
// the transposing LDS read ds_read_b64_tr_b16: lane 4 qq + p of a 16-lane group names rule qq's row and its
// channels 4p .. 4p+3, and lane i receives channel i of the group's 4 rules -- no split or permute in the loop.
// Block = 8 waves, persistent over a contiguous range of tiles for one 32 x 32 slice; wave w owns offsets
// w, w + 8, w + 16, w + 24 and keeps their 32 x 32 tiles in registers over the range; the next tile's rows,
// values and rule words are in flight in registers while the current tile computes.  Per range a slab of
// partial dW is written and the ranges are added in order (deterministic).
constexpr int kWTile = 128;
constexpr int kWMaxCh = 216;                   // chunks of one 128-row tile (K <= 27 offsets x 8)
constexpr int kWXImg = (kWCap + 1) * 32;       // bf16 elements of one x piece image (+ zero row kWCap)
constexpr int kWDImg = (kWTile + 1) * 32;      // dy piece image (+ zero row 128)

// bf16 element offset of 8-byte unit v (channels 4v .. 4v+3 of the slice) of row j in a piece image
__device__ __forceinline__ int wimg_off(int j, int v) { return j * 32 + 4 * (v ^ (((j >> 2) & 1) << 2)); }

typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 tr_read(const uint16_t* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  return __builtin_bit_cast(uint2, v);
}

// 4 fp32 -> three bf16x4 pieces (8 bytes each), v = p[0] + p[1] + p[2] exactly (as split8)
__device__ __forceinline__ void split4(const floatx4& a, uint2 (&p)[3]) {
  float v[4] = {a[0], a[1], a[2], a[3]};
#pragma unroll
  for (int s = 0; s < 3; ++s) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t h = pk_bf16(v[2 * i], v[2 * i + 1]);
      if (i == 0) p[s].x = h;
      else p[s].y = h;
      if (s < 2) {
        v[2 * i] -= __uint_as_float(h << 16);
        v[2 * i + 1] -= __uint_as_float(h & 0xffff0000u);
      }
    }
  }
}

// ABL (timing experiments only, wrong results): 1 no MFMAs, 2 no transposing reads, 4 no value loads,
// 8 no staging stores
template <int NW, int ABL = 0>
__global__ __launch_bounds__(64 * NW, 1) void wgrad_x6c_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out, int K,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const uint32_t* __restrict__ chunk_lr, const int64_t* __restrict__ u_start, const int32_t* __restrict__ u_rows,
    int64_t n_rows, int64_t n_tiles, int n_ranges, float* __restrict__ slab) {
  constexpr int NTH = 64 * NW, NOW = 32 / NW;          // offsets per wave: o = wave + NW a, a < NOW
  constexpr int XI = (kWCap * 8 + NTH - 1) / NTH;     // x staging items (row, 4 channels) per thread
  constexpr int DI = kWTile * 8 / NTH;                // dy staging items per thread
  constexpr int EI = (kWMaxCh * 16 + NTH - 1) / NTH;  // rule words per thread
  static_assert(DI * NTH == kWTile * 8, "dy staging items must divide evenly");
  __shared__ __attribute__((aligned(16))) uint16_t xim[3 * kWXImg];
  __shared__ __attribute__((aligned(16))) uint16_t dim[3 * kWDImg];
  __shared__ uint32_t ent[(kWMaxCh + 1) * 16];  // + one chunk: the partner read of a last odd chunk stays inside
  __shared__ uint8_t offs[kWMaxCh];
  __shared__ int otab[2][32];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, p4 = i16 & 3;
  const int n_sl_o = c_out / 32, n_slices = (c_in / 32) * n_sl_o;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int slice = (int)(lb % n_slices);
  const int range = (int)(lb / n_slices);
  const int ci0 = 32 * (slice / n_sl_o), co0 = 32 * (slice % n_sl_o);
  const int64_t t0 = (int64_t)range * n_tiles / n_ranges, t1 = (int64_t)(range + 1) * n_tiles / n_ranges;

  floatx4 acc[NOW][2][2];
#pragma unroll
  for (int a = 0; a < NOW; ++a)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[a][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // zero rows (never overwritten) and the padding chunk of the rule words
  for (int i = tid; i < 3 * 32; i += NTH) {
    xim[(i / 32) * kWXImg + kWCap * 32 + (i % 32)] = 0;
    dim[(i / 32) * kWDImg + kWTile * 32 + (i % 32)] = 0;
  }
  if (tid < 16) ent[kWMaxCh * 16 + tid] = (uint32_t)kWCap | ((uint32_t)kWTile << 16);

  // ---- staging registers: rows of tile t + 1 (loaded at the start of t), then its values and rule words
  int32_t srow[XI];
  floatx4 xv[XI], dv[DI];
  uint32_t ev[EI];
  int co_v = 255, s_nch = 0;
  auto issue_rows = [&](int64_t t) {  // the tile's distinct rows (<= kWCap: checked on the host)
    const int64_t u0 = u_start[t];
    const int nu = (int)(u_start[t + 1] - u0);
#pragma unroll
    for (int b = 0; b < XI; ++b) {
      const int it = tid + NTH * b;
      srow[b] = it < nu * 8 ? u_rows[u0 + (it >> 3)] : -1;
    }
  };
  auto issue_vals = [&](int64_t t) {  // values of tile t (rows in srow) and its rule words
#pragma unroll
    for (int b = 0; b < XI; ++b) {
      const int u = (tid + NTH * b) & 7;
      xv[b] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (!(ABL & 4) && srow[b] >= 0) xv[b] = *reinterpret_cast<const floatx4*>(x + (int64_t)srow[b] * c_in + ci0 + 4 * u);
    }
#pragma unroll
    for (int b = 0; b < DI; ++b) {
      const int it = tid + NTH * b, u = it & 7;
      const int64_t row = t * kWTile + (it >> 3);
      dv[b] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (!(ABL & 4) && row < n_rows) dv[b] = *reinterpret_cast<const floatx4*>(dy + row * c_out + co0 + 4 * u);
    }
    const int64_t c0 = tile_start[t];
    s_nch = (int)(tile_start[t + 1] - c0);
#pragma unroll
    for (int b = 0; b < EI; ++b) {
      const int e = tid + NTH * b;
      ev[b] = e < s_nch * 16 ? chunk_lr[c0 * 16 + e] : 0u;
    }
    co_v = tid < s_nch ? chunk_off[c0 + tid] : 255;
  };
  auto store = [&]() {  // the staged tile into LDS (two barriers: offset table)
#pragma unroll
    for (int b = 0; b < XI; ++b) {
      if (!(ABL & 8) && srow[b] >= 0) {
        const int it = tid + NTH * b;
        uint2 pc[3];
        split4(xv[b], pc);
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          *reinterpret_cast<uint2*>(xim + pp * kWXImg + wimg_off(it >> 3, it & 7)) = pc[pp];
      }
    }
#pragma unroll
    for (int b = 0; b < DI; ++b) {
      if (ABL & 8) break;
      const int it = tid + NTH * b;
      uint2 pc[3];
      split4(dv[b], pc);
#pragma unroll
      for (int pp = 0; pp < 3; ++pp)
        *reinterpret_cast<uint2*>(dim + pp * kWDImg + wimg_off(it >> 3, it & 7)) = pc[pp];
    }
#pragma unroll
    for (int b = 0; b < EI; ++b) {
      const int e = tid + NTH * b;
      if (e < s_nch * 16) ent[e] = ev[b];
    }
    if (tid < s_nch) offs[tid] = (uint8_t)co_v;
    if (tid < 64) otab[tid >> 5][tid & 31] = 0;
    __syncthreads();
    if (tid < s_nch) {
      const int o = offs[tid];
      if (tid == 0 || offs[tid - 1] != o) otab[0][o] = tid;
      if (tid == s_nch - 1 || offs[tid + 1] != o) otab[1][o] = tid + 1;
    }
    __syncthreads();
  };

  // ---- one 32-rule step over the two chunks cA, cA + 1 (the second only if hasB): the B fragments (dy) of
  // both 16-column halves, then per 16-row half of x its A fragments and 12 MFMAs (36 fragment registers live)
  auto rows_of = [&](int cA, bool hasB, int (&xr)[2], int (&dr)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kp = 8 * g + 4 * h + qq, cs = kp >> 4;
      uint32_t w = ent[(cA + cs) * 16 + (kp & 15)];
      if (cs == 1 && !hasB) w = (uint32_t)kWCap | ((uint32_t)kWTile << 16);
      const int ls = (int)(w & 0xFFFFu);
      xr[h] = ls < kWCap ? ls : kWCap;
      dr[h] = (int)(w >> 16);
    }
  };
  auto frag = [&](const uint16_t* img, const int (&rr)[2], int v) {
    if (ABL & 2) return u32x4{(uint32_t)rr[0], (uint32_t)rr[1], (uint32_t)v, 7u};
    const uint2 lo = tr_read(img + wimg_off(rr[0], v));
    const uint2 hi = tr_read(img + wimg_off(rr[1], v));
    return u32x4{lo.x, lo.y, hi.x, hi.y};
  };
  auto kstep = [&](int cA, bool hasB, floatx4 (&ac)[2][2]) {
    int xr[2], dr[2];
    rows_of(cA, hasB, xr, dr);
    u32x4 fb[2][3], fa[3];
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int pp = 0; pp < 3; ++pp) fb[sb][pp] = frag(dim + pp * kWDImg, dr, 4 * sb + p4);
#pragma unroll
    for (int sa = 0; sa < 2; ++sa) {
#pragma unroll
      for (int pp = 0; pp < 3; ++pp) fa[pp] = frag(xim + pp * kWXImg, xr, 4 * sa + p4);
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        if (ABL & 1) {
          ac[sa][sb] += __builtin_bit_cast(floatx4, fa[0] ^ fa[1] ^ fa[2] ^ fb[sb][0] ^ fb[sb][1] ^ fb[sb][2]);
          continue;
        }
        floatx4 c = mfma_bf16(fa[2], fb[sb][0], floatx4{0.f, 0.f, 0.f, 0.f});
        c = mfma_bf16(fa[1], fb[sb][1], c);
        c = mfma_bf16(fa[0], fb[sb][2], c);
        c = mfma_bf16(fa[1], fb[sb][0], c);
        c = mfma_bf16(fa[0], fb[sb][1], c);
        ac[sa][sb] += mfma_bf16(fa[0], fb[sb][0], c);
      }
    }
  };

  if (t0 < t1) {
    issue_rows(t0);
    issue_vals(t0);
    store();
    for (int64_t t = t0; t < t1; ++t) {
      const bool more = t + 1 < t1;
      if (more) issue_rows(t + 1);
      // this wave's offsets: chunk range and 32-rule steps, flattened over the (up to) four offsets
      int first[NOW + 1], endc[NOW + 1], S[NOW + 1];
      S[0] = 0;
#pragma unroll
      for (int a = 0; a < NOW; ++a) {
        const int o = wave + NW * a;
        first[a] = o < K ? __builtin_amdgcn_readfirstlane(otab[0][o]) : 0;
        endc[a] = o < K ? __builtin_amdgcn_readfirstlane(otab[1][o]) : 0;
        S[a + 1] = S[a] + (endc[a] - first[a] + 1) / 2;
      }
      const int n_st = S[NOW];
      const int s_vals = n_st / 2;  // the next tile's values go out half-way through (their rows have landed)
      int s = 0;
#pragma unroll
      for (int a = 0; a < NOW; ++a) {  // constant slot index: acc[a] stays in registers
        for (int c = first[a]; c < endc[a]; c += 2, ++s) {
          if (s == s_vals && more) issue_vals(t + 1);
          kstep(c, c + 1 < endc[a], acc[a]);
        }
      }
      if (n_st == 0 && more) issue_vals(t + 1);
      __syncthreads();  // reads of tile t done
      if (more) store();
    }
  }
  // partial dW of this range: slab[range][o][ci][co]
  float* sb = slab + (int64_t)range * K * c_in * c_out;
#pragma unroll
  for (int a = 0; a < NOW; ++a) {
    const int o = wave + NW * a;
    if (o >= K) break;
#pragma unroll
    for (int sa = 0; sa < 2; ++sa)
#pragma unroll
      for (int sbb = 0; sbb < 2; ++sbb)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          sb[((int64_t)o * c_in + ci0 + 16 * sa + 4 * g + jj) * c_out + co0 + 16 * sbb + i16] = acc[a][sa][sbb][jj];
  }
}

inline int local_nt(int c_out) { return (c_out / 16) % 2 == 0 ? 2 : 1; }

static int g_local_wr = 2;     // row parts per block (waves = 4 x wr); msp_debug_conv_local (experiments)
static int g_local_order = 1;  // msp_tile_local: order rows inside a tile by neighbour mask
static int g_local_nt = 0;     // forced column tiles per wave (0: local_nt)
static int g_local_abl = 0;    // ablation variant (timing only; msp_debug_conv_local_abl)
// 0: conv_x6s everywhere (default since its staged rows' indices stay in registers and the index tile loads as
// words: 2.5-4 % ahead of conv_x6l at level 1, profiles/r02/kbench_local_l1form_r02.log), 1: conv_x6l wherever it
// applies, 2: conv_x6l for 64 output channels (the round-2 choice before that)
constexpr int kLocalFormDefault = 0;
static int g_local_form = kLocalFormDefault;
static int g_local_d = 2;      // weight register sets of conv_x6s (prefetch depth; msp_debug_conv_local_d)
static int g_local_wp = 3;     // weight image: 3 = bf16 pieces, 2 = fp32 split in registers (msp_debug_conv_local_wp)
static int g_local_ri = 3;       // conv_x6s: row indices held in registers across slices (msp_debug_conv_local_ri)
static int g_local_min_ch = 64;  // msp_conv_local_preferred: channels on both sides from (msp_debug_conv_local_min_ch)

inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

}  // namespace msp

using namespace msp;

extern "C" {

size_t msp_tile_local_workspace_size(int64_t n, int tile_rows) {
  const int64_t n_tiles = ceil_div(n > 0 ? n : 1, tile_rows > 0 ? tile_rows : 1);
  return (size_t)(n_tiles + 1) * sizeof(int64_t) + scan_ws_bytes(n_tiles);
}

int msp_tile_local(const int32_t* nbr, int K, int64_t n, int tile_rows, int64_t* u_start, int32_t* u_rows,
                   int64_t u_cap, uint16_t* lidx, int32_t* perm, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= 32 && n >= 0, "msp_tile_local: K must be in [1, 32] (got %d)", K);
  MSP_REQUIRE(tile_rows == 64 || tile_rows == 128 || tile_rows == 256,
              "msp_tile_local: tile_rows must be 64, 128 or 256 (got %d)", tile_rows);
  MSP_REQUIRE(n < (1ll << 31), "msp_tile_local: too many rows");
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n, tile_rows);
  const size_t need = msp_tile_local_workspace_size(n, tile_rows);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_tile_local: workspace too small (%zu < %zu)", ws_bytes, need);
  if (n_tiles == 0) {
    MSP_HIP(hipMemsetAsync(u_start, 0, 2 * sizeof(int64_t), s), "msp_tile_local");
    return MSP_OK;
  }
  const int64_t n_pad = n_tiles * tile_rows;
  int64_t* cnt = reinterpret_cast<int64_t*>(ws);
  void* sws = cnt + n_tiles + 1;
  const unsigned grid = (unsigned)n_tiles;
  if (u_cap <= 0) {  // counting call: u_start[0..n_tiles] = exclusive scan, u_start[n_tiles + 1] = largest tile
    MSP_HIP(hipMemsetAsync(u_start + n_tiles + 1, 0, sizeof(int64_t), s), "msp_tile_local");
    auto* mx = reinterpret_cast<unsigned long long*>(u_start + n_tiles + 1);
    if (tile_rows == 64) local_count_kernel<64, 2048><<<grid, kLT, 0, s>>>(nbr, K, n, cnt, mx);
    else if (tile_rows == 128) local_count_kernel<128, 4096><<<grid, kLT, 0, s>>>(nbr, K, n, cnt, mx);
    else local_count_kernel<256, 8192><<<grid, kLT, 0, s>>>(nbr, K, n, cnt, mx);
    const int rc = scan_exclusive_i64(cnt, u_start, n_tiles, u_start + n_tiles, sws, scan_ws_bytes(n_tiles), s);
    if (rc) return rc;
  } else {
    MSP_REQUIRE(u_rows && lidx && perm, "msp_tile_local: NULL output");
    if (tile_rows == 64)
      local_fill_kernel<64, 2048><<<grid, kLT, 0, s>>>(nbr, K, n, n_pad, u_start, u_rows, lidx, perm, g_local_order);
    else if (tile_rows == 128)
      local_fill_kernel<128, 4096><<<grid, kLT, 0, s>>>(nbr, K, n, n_pad, u_start, u_rows, lidx, perm, g_local_order);
    else
      local_fill_kernel<256, 8192><<<grid, kLT, 0, s>>>(nbr, K, n, n_pad, u_start, u_rows, lidx, perm, g_local_order);
  }
  return check_launch("msp_tile_local");
}

// Experiment hook (not part of the public ABI; scripts/kbench_local.py): wr = row parts per block (1 or 2),
// order = 1 to order rows inside a tile by neighbour mask (0: key order), nt = forced column tiles per wave
// (0: automatic); negative = keep.
int msp_debug_conv_local(int wr, int order, int nt) {
  if (wr == 1 || wr == 2) g_local_wr = wr;
  if (nt >= 0) g_local_nt = nt;
  if (order >= 0) g_local_order = order ? 1 : 0;
  return MSP_OK;
}

// weight image of msp_conv_local: 3 = split once into bf16 pieces, 2 = fp32, split by the kernels in registers
int msp_debug_conv_local_wp(int wp) {
  if (wp == 2 || wp == 3) g_local_wp = wp;
  return MSP_OK;
}

int msp_debug_conv_local_ri(int ri) {
  g_local_ri = ri < 0 ? 0 : (ri > 3 ? 3 : ri);
  return MSP_OK;
}

int msp_debug_conv_local_d(int d) {
  if (d == 1 || d == 2) g_local_d = d;
  return MSP_OK;
}

int msp_debug_conv_local_abl(int abl) {
  if (abl < 0) {  // -1 / -2 / -3 / -4: persistent form off / wherever it applies / the default / 64 channels only
    g_local_form = abl == -2 ? 1 : (abl == -3 ? kLocalFormDefault : (abl == -4 ? 2 : 0));
    return MSP_OK;
  }
  g_local_abl = abl;
  return MSP_OK;
}

// Measured against the gather forms on the headline batch's rulebooks (scripts/kbench_local.py,
// profiles/r02/kbench_local_r02_levels.log): ahead from 64 channels on both sides and 4096 rows up (levels
// 1-4 of m = 32: 0-34 % less time), behind on the 32-channel level 0 (the per-wave tile form x6r and the
// dense row groups) and on the few-tile levels 5-6 (grids of 16 / 4 tiles).
int msp_wgrad_local_ok(int64_t n_rows, int K, int c_in, int c_out) {
  return (n_rows > 0 && K <= kKMax && c_in % 32 == 0 && c_out % 32 == 0) ? 1 : 0;
}

int64_t msp_wgrad_local_ranges(int64_t n_rows, int c_in, int c_out) {
  const int64_t n_tiles = ceil_div(n_rows > 0 ? n_rows : 1, 128);
  const int64_t slices = (int64_t)(c_in / 32) * (c_out / 32);
  int64_t r = cu_count() / (slices > 0 ? slices : 1);
  if (r < 1) r = 1;
  return r < n_tiles ? r : n_tiles;
}

int msp_conv_wgrad_local(const float* x, int c_in, const float* dy, int c_out, int K, int tile_rows,
                         const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows, const int32_t* perm,
                         int64_t n_rows, int64_t n_ranges, float* slab, float* dw, msp_stream_t stream) {
  MSP_REQUIRE(msp_wgrad_local_ok(n_rows, K, c_in, c_out), "msp_conv_wgrad_local: needs K <= %d and channels in "
              "multiples of 32 (K=%d c_in=%d c_out=%d)", kKMax, K, c_in, c_out);
  MSP_REQUIRE(tile_rows == 128, "msp_conv_wgrad_local: tile_rows must be 128 (got %d)", tile_rows);
  MSP_REQUIRE(n_ranges >= 1, "msp_conv_wgrad_local: n_ranges must be >= 1");
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  const int64_t slices = (int64_t)(c_in / 32) * (c_out / 32);
  wgrad_x6t_kernel<<<(unsigned)(n_ranges * slices), 512, 0, s>>>(x, c_in, dy, c_out, lidx, u_start, u_rows, perm, K,
                                                                   n_tiles, n_tiles * tile_rows, (int)n_ranges, slab);
  const int64_t n4 = (int64_t)K * c_in * c_out / 4;
  wgrad_ranges_reduce_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, s>>>(reinterpret_cast<const floatx4*>(slab),
                                                                         (int)n_ranges, n4,
                                                                         reinterpret_cast<floatx4*>(dw));
  return check_launch("msp_conv_wgrad_local");
}

int64_t msp_chunk_local_cap(int tile_rows) { return tile_rows == kQT ? kQCap : kWCap; }

int msp_chunk_local(const int64_t* tile_start, int64_t n_rows, int tile_rows, int max_chunks,
                    const int32_t* chunk_src, const uint16_t* chunk_row, int32_t* u_rows, int32_t* u_cnt,
                    uint32_t* chunk_lr, int64_t* max_count, msp_stream_t stream) {
  MSP_REQUIRE(tile_rows == 64 || tile_rows == 128, "msp_chunk_local: tile_rows must be 64 or 128 (got %d)",
              tile_rows);
  MSP_REQUIRE(n_rows >= 0 && n_rows < (1ll << 31), "msp_chunk_local: bad row count");
  MSP_REQUIRE(max_chunks >= 0 && (kQUnit / tile_rows) * max_chunks * MSP_CHUNK <= 4096,
              "msp_chunk_local: a tile has %d chunks (K <= 32 allows at most %d)", max_chunks,
              4096 / MSP_CHUNK / (kQUnit / tile_rows));
  const int64_t n_tiles = ceil_div(n_rows, tile_rows), tpu = kQUnit / tile_rows, n_units = ceil_div(n_tiles, tpu);
  hipStream_t s = as_stream(stream);
  if (max_count) MSP_HIP(hipMemsetAsync(max_count, 0, sizeof(int64_t), s), "msp_chunk_local");
  if (n_units == 0) return MSP_OK;
  MSP_REQUIRE(tile_start && chunk_src && chunk_row && u_rows && u_cnt && chunk_lr, "msp_chunk_local: NULL pointer");
  const int cap = (int)msp_chunk_local_cap(tile_rows);
  auto* mx = reinterpret_cast<unsigned long long*>(max_count);
  const bool small = tpu * max_chunks * MSP_CHUNK <= 2048;
#define CL(N2, TPU, TR)                                                                                         \
  chunk_local_kernel<N2, TPU, TR><<<(unsigned)n_units, kLT, 0, s>>>(tile_start, n_tiles, chunk_src, chunk_row, cap, \
                                                                    u_rows, u_cnt, chunk_lr, mx)
  if (tile_rows == 64) {
    if (small) CL(2048, 2, 64);
    else CL(4096, 2, 64);
  } else {
    if (small) CL(2048, 1, 128);
    else CL(4096, 1, 128);
  }
#undef CL
  return check_launch("msp_chunk_local");
}

static int g_chunk_dv = 2;     // value lead of conv_x6q (msp_debug_conv_chunk: experiments)
static int g_chunk_pref = -1;  // -1: msp_conv_chunk_local_preferred's rule, 0 / 1: forced off / on
static int g_chunk_abl = 0;    // ablation variant (timing only)

int msp_debug_conv_chunk(int dv, int pref, int abl) {
  if (dv == 2 || dv == 3 || dv == 4) g_chunk_dv = dv;
  if (pref >= -1 && pref <= 1) g_chunk_pref = pref;
  if (abl >= 0) g_chunk_abl = abl;
  return MSP_OK;
}

// Measured on the headline batch's level 0 (scripts/kbench_chunk.py, profiles/r02/kbench_chunk_r02.log):
// 0.43 / 0.74 / 0.79 ms for 32 -> 32 / 64 -> 32 / 32 -> 64 against 0.34 / 0.56 / 0.78 for the per-wave gather
// tiles and the dense row groups -- the per-unit start-up (row list -> staged rows -> barrier, two blocks per CU)
// costs more than the gathers it saves, so the library does not take it on its own (opt-in: force = 1 through
// msp_debug_conv_chunk).
int msp_conv_chunk_local_preferred(int64_t n_rows, int c_in, int c_out) {
  const int fits = c_in % 16 == 0 && c_out % 32 == 0 && c_in <= 64 && c_out <= 64 && n_rows >= 4096;
  return fits && g_chunk_pref == 1 ? 1 : 0;
}

int msp_conv_chunk_local(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                         const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                         const uint32_t* chunk_lr, const int32_t* u_rows, const int32_t* u_cnt, int64_t n_rows,
                         float* out, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 32 == 0,
              "msp_conv_chunk_local: c_in must be a multiple of 16 and c_out of 32 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= kKMax, "msp_conv_chunk_local: K must be in [1, %d] (got %d)", kKMax, K);
  MSP_REQUIRE(tile_rows == kQT, "msp_conv_chunk_local: tile_rows must be %d (got %d)", kQT, tile_rows);
  MSP_REQUIRE(flip >= 0 && flip <= 3, "msp_conv_chunk_local: flip must be 0..3 (got %d)", flip);
  const size_t need = msp_conv_local_workspace_size(K, c_in, c_out);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_chunk_local: workspace too small (%zu < %zu)", ws_bytes, need);
  const int64_t n_tiles = ceil_div(n_rows, kQT), n_units = ceil_div(n_tiles, 2);
  if (n_units == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  constexpr int NT = 2;
  const int n_y = c_out / (16 * NT), nks = (c_in + 31) / 32;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t lanes = (int64_t)K * n_y * nks * NT * 64;
  split_weights_lane_kernel<3><<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                              (flip >> 1) & 1);
  const unsigned grid = (unsigned)(n_units * n_y);
#define LQ(DV, A)                                                                                              \
  if (g_chunk_dv == DV && g_chunk_abl == A)                                                                    \
    conv_x6q_kernel<NT, DV, A><<<grid, 256, 0, s>>>(x, c_in, img, K, flip & 1, c_out, tile_start, chunk_off,  \
                                                    chunk_lr, chunk_src, u_rows, u_cnt, n_rows, n_tiles, n_y, out);
  LQ(2, 0) LQ(3, 0) LQ(4, 0)
  LQ(4, 1) LQ(4, 2) LQ(4, 4) LQ(4, 8) LQ(4, 16) LQ(4, 31)
#undef LQ
  return check_launch("msp_conv_chunk_local");
}

static int g_wchunk_nw = 8;  // waves per block of wgrad_x6c (8 or 16; msp_debug_wgrad_chunk: experiments)
static int g_wchunk_abl = 0;

int msp_debug_wgrad_chunk(int nw, int abl) {
  if (nw == 8 || nw == 16) g_wchunk_nw = nw;
  if (abl >= 0) g_wchunk_abl = abl;
  return MSP_OK;
}

int msp_wgrad_chunk_ok(int64_t n_rows, int K, int c_in, int c_out) {
  return (n_rows > 0 && K >= 1 && K <= 27 && c_in % 32 == 0 && c_out % 32 == 0) ? 1 : 0;
}

// Measured against the pair lists on the headline batch (scripts/kbench_wgrad_local.py,
// profiles/r02/kbench_wgrad_chunk_r02.log): 0.59 vs 0.65 ms at level 1 64 -> 64, 0.40 vs 0.46 at level 2,
// 0.59 vs 0.68 at level 0 32 -> 64; behind at level 0's 32 and 64 -> 32 (0.36 / 0.60 vs 0.35 / 0.55 ms); the
// few-tile levels (< 2^14 rows) are unmeasured and stay on the pair lists.
int msp_wgrad_chunk_preferred(int64_t n_rows, int K, int c_in, int c_out) {
  return msp_wgrad_chunk_ok(n_rows, K, c_in, c_out) && c_out >= 64 && n_rows >= (1 << 14) ? 1 : 0;
}

int64_t msp_wgrad_chunk_ranges(int64_t n_rows, int c_in, int c_out) {
  const int64_t n_tiles = ceil_div(n_rows > 0 ? n_rows : 1, kWTile);
  const int64_t slices = (int64_t)(c_in / 32) * (c_out / 32);
  int64_t r = cu_count() / (slices > 0 ? slices : 1);
  if (r < 1) r = 1;
  return r < n_tiles ? r : n_tiles;
}

int64_t msp_wgrad_chunk_cap(void) { return kWCap; }

int msp_wgrad_chunk_index(const int64_t* tile_start, const int32_t* chunk_src, const uint16_t* chunk_row,
                          int64_t n_rows, const int64_t* u_start, const int32_t* u_rows, uint32_t* chunk_lr,
                          msp_stream_t stream) {
  MSP_REQUIRE(n_rows >= 0 && n_rows < (1ll << 31), "msp_wgrad_chunk_index: bad row count");
  const int64_t n_tiles = ceil_div(n_rows, kWTile);
  if (n_tiles == 0) return MSP_OK;
  MSP_REQUIRE(tile_start && chunk_src && chunk_row && u_start && u_rows && chunk_lr,
              "msp_wgrad_chunk_index: NULL pointer");
  chunk_lidx_kernel<<<(unsigned)n_tiles, kLT, 0, as_stream(stream)>>>(tile_start, chunk_src, chunk_row, u_start,
                                                                      u_rows, chunk_lr);
  return check_launch("msp_wgrad_chunk_index");
}

int msp_conv_wgrad_chunk(const float* x, int c_in, const float* dy, int c_out, int K, int tile_rows,
                         const int64_t* tile_start, const uint8_t* chunk_off, const uint32_t* chunk_lr,
                         const int64_t* u_start, const int32_t* u_rows, int64_t n_rows, int64_t n_ranges,
                         float* slab, float* dw, msp_stream_t stream) {
  MSP_REQUIRE(msp_wgrad_chunk_ok(n_rows, K, c_in, c_out), "msp_conv_wgrad_chunk: needs K <= 27 and channels in "
              "multiples of 32 (K=%d c_in=%d c_out=%d n=%lld)", K, c_in, c_out, (long long)n_rows);
  MSP_REQUIRE(tile_rows == kWTile, "msp_conv_wgrad_chunk: tile_rows must be %d (got %d)", kWTile, tile_rows);
  MSP_REQUIRE(n_ranges >= 1, "msp_conv_wgrad_chunk: n_ranges must be >= 1");
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n_rows, kWTile);
  const int64_t slices = (int64_t)(c_in / 32) * (c_out / 32);
#define WC(A)                                                                                                  \
  else if (g_wchunk_abl == A) wgrad_x6c_kernel<8, A><<<(unsigned)(n_ranges * slices), 512, 0, s>>>(               \
      x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr, u_start, u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  if (g_wchunk_abl == 0 && g_wchunk_nw == 16)
    wgrad_x6c_kernel<16><<<(unsigned)(n_ranges * slices), 1024, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off,
                                                                        chunk_lr, u_start, u_rows, n_rows, n_tiles,
                                                                        (int)n_ranges, slab);
  WC(1) WC(2) WC(4) WC(8) WC(15)
  else
    wgrad_x6c_kernel<8><<<(unsigned)(n_ranges * slices), 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off,
                                                                      chunk_lr, u_start, u_rows, n_rows, n_tiles,
                                                                      (int)n_ranges, slab);
#undef WC
  const int64_t n4 = (int64_t)K * c_in * c_out / 4;
  wgrad_ranges_reduce_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, s>>>(reinterpret_cast<const floatx4*>(slab),
                                                                         (int)n_ranges, n4,
                                                                         reinterpret_cast<floatx4*>(dw));
  return check_launch("msp_conv_wgrad_chunk");
}

int msp_conv_local_preferred(int64_t n_rows, int c_in, int c_out) {
  return (c_in % 16 == 0 && c_out % 16 == 0 && c_in >= g_local_min_ch && c_out >= g_local_min_ch &&
          n_rows >= 4096) ? 1 : 0;
}

// Experiment hook: the smallest channel count msp_conv_local_preferred takes (64; 32 adds level 0 of m = 32,
// on the persistent form at 32 output channels)
int msp_debug_conv_local_min_ch(int c) {
  if (c == 32 || c == 64) g_local_min_ch = c;
  return MSP_OK;
}

size_t msp_conv_local_workspace_size(int K, int c_in, int c_out) {
  return (size_t)K * c_out * ((c_in + 31) / 32) * 32 * 6;
}

int msp_conv_local(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                   const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows, const int32_t* perm,
                   int64_t n_rows, float* out, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_local: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= kKMax, "msp_conv_local: K must be in [1, %d] (got %d)", kKMax, K);
  MSP_REQUIRE(tile_rows == 128, "msp_conv_local: tile_rows must be 128 (got %d)", tile_rows);
  MSP_REQUIRE(flip >= 0 && flip <= 3, "msp_conv_local: flip must be 0..3 (got %d)", flip);
  const size_t need = msp_conv_local_workspace_size(K, c_in, c_out);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_local: workspace too small (%zu < %zu)", ws_bytes, need);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  if (((g_local_form == 1 && c_out % 32 == 0) ||
       (g_local_form == 2 && (c_out == 64 || (c_out == 32 && g_local_min_ch <= 32)))) && g_local_abl == 0) {
    // persistent pipelined form: 16 NT columns per wave, two column halves per block
    const int NT = c_out % 96 == 0 ? 3 : (c_out % 64 == 0 ? 2 : 1);
    const int n_y = c_out / (32 * NT), nks = (c_in + 31) / 32;
    u32x4* img = static_cast<u32x4*>(ws);
    const int64_t lanes = (int64_t)K * (2 * n_y) * nks * NT * 64;
    const int wp = g_local_wp;
    if (wp == 2)
      split_weights_lane_kernel<2><<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                                  (flip >> 1) & 1);
    else
      split_weights_lane_kernel<3><<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                                  (flip >> 1) & 1);
    const int64_t n_pad = n_tiles * tile_rows, n_items = n_tiles * n_y;
    const unsigned grid = (unsigned)(n_items < cu_count() ? n_items : cu_count());
#define LP(N, P)                                                                                                \
  if (NT == N && wp == P)                                                                                     \
    conv_x6l_kernel<N, P><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start, u_rows, perm,    \
                                               n_pad, n_y, n_items, out);
    LP(1, 3) LP(2, 3) LP(3, 3) LP(1, 2) LP(2, 2) LP(3, 2)
#undef LP
    return check_launch("msp_conv_local");
  }
  const int NT = (g_local_nt == 1 || (g_local_nt == 2 && c_out % 32 == 0)) ? g_local_nt : local_nt(c_out);
  const int n_y = c_out / (16 * NT), nks = (c_in + 31) / 32;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t lanes = (int64_t)K * n_y * nks * NT * 64;
  const int wp = g_local_abl == 0 ? g_local_wp : 3;
  if (wp == 2)
    split_weights_lane_kernel<2><<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                                (flip >> 1) & 1);
  else
    split_weights_lane_kernel<3><<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                                (flip >> 1) & 1);
  const int64_t n_pad = n_tiles * tile_rows;
  const unsigned grid = (unsigned)(n_tiles * n_y);
  const int wr = g_local_wr;
  const int dd = g_local_abl == 0 ? g_local_d : 2;
  const int ri = g_local_abl == 0 && wp == 3 && dd == 2 ? g_local_ri : 0;
  if (ri == 3 && wr == 2 && NT == 2)
    conv_x6s_kernel<2, 128, 2, 2, 0, 3, 2, 0><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start,
                                                                   u_rows, perm, n_pad, n_y, out);
  else if (ri == 2 && wr == 2 && NT == 2)
    conv_x6s_kernel<2, 128, 2, 2, 0, 3, 2><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start,
                                                                u_rows, perm, n_pad, n_y, out);
  else if (ri && wr == 2 && NT == 2)
    conv_x6s_kernel<2, 128, 2, 2, 0, 3, 1><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start,
                                                                u_rows, perm, n_pad, n_y, out);
  else if (ri && wr == 2 && NT == 1)
    conv_x6s_kernel<1, 128, 2, 2, 0, 3, 1><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start,
                                                                u_rows, perm, n_pad, n_y, out);
  else {
#define LX(N, W, A, P, DD)                                                                                    \
  if (NT == N && wr == W && g_local_abl == A && wp == P && dd == DD)                                          \
    conv_x6s_kernel<N, 128, DD, W, A, P><<<grid, 256 * W, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx,      \
                                                                  u_start, u_rows, perm, n_pad, n_y, out);
    LX(2, 1, 0, 3, 2) LX(1, 1, 0, 3, 2) LX(2, 2, 0, 3, 2) LX(1, 2, 0, 3, 2) LX(2, 1, 0, 2, 2) LX(1, 1, 0, 2, 2)
    LX(2, 2, 0, 2, 2) LX(1, 2, 0, 2, 2) LX(2, 2, 0, 3, 1) LX(1, 2, 0, 3, 1) LX(2, 2, 0, 2, 1)
    LX(2, 2, 1, 3, 2) LX(2, 2, 2, 3, 2) LX(2, 2, 4, 3, 2) LX(2, 2, 8, 3, 2) LX(2, 2, 16, 3, 2) LX(2, 2, 15, 3, 2)
    LX(2, 2, 31, 3, 2)
#undef LX
  }
  return check_launch("msp_conv_local");
}

}  // extern "C"
