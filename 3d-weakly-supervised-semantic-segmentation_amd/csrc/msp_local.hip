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
#include <type_traits>

#include "msp_x6.h"
#include "msp_bn_epi.h"

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

// The tile's distinct input rows, unordered: its K x T neighbour entries (all loads in flight first) go
// into an open-addressing hash set in LDS (kHashMult N2 int32 slots, linear probing by LDS CAS); each first
// insertion appends the row to uq.  Returns the count.  (Round 2 replaced a bitonic sort of all N2 entries: a
// tile names 1.6-2 x T distinct rows of 27 T entries, so sorting only those is ~10x less work.)  Slots: N2 since
// round 5 (load 0.05-0.1 on surfaces, at most 0.84 for a map whose 27 T entries are all distinct): 32 KB of LDS per
// block instead of 48, so a build block beside the compute stream's one-block-per-CU weight gradient (125 KB) no
// longer keeps it off that CU.
#ifndef MSP_LOCAL_HASH_MULT  // experiments: 2 = the round-2..4 table (2 N2 slots)
#define MSP_LOCAL_HASH_MULT 1
#endif
template <int T, int N2>
__device__ int tile_distinct(const int32_t* __restrict__ nbr, int K, int64_t n, int64_t t, int32_t* h, int32_t* uq,
                             int* cnt, int32_t (&m)[N2 / kLT], uint32_t* msk = nullptr) {
  // m: this thread's entries (offset i / T, row i % T for i = threadIdx.x + kLT j; -1 absent), kept in registers
  // for the caller (the fill's local indices).  msk (optional, T words): each row's neighbour mask, set here from
  // those same entries by LDS OR.
  constexpr int HS = MSP_LOCAL_HASH_MULT * N2, HB = __builtin_ctz(HS);
  constexpr int PER = N2 / kLT;  // K T <= N2 entries
  for (int i = threadIdx.x; i < HS; i += kLT) h[i] = -1;
  if (msk)
    for (int i = threadIdx.x; i < T; i += kLT) msk[i] = 0u;
  if (threadIdx.x == 0) *cnt = 0;
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
    if (msk) {
      const int i = threadIdx.x + kLT * j, o = i / T;
      atomicOr(&msk[i - o * T], 1u << o);
    }
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

// The hash slot of v (present in h: inserted by tile_distinct).
template <int HS>
__device__ __forceinline__ int hash_slot(const int32_t* h, int32_t v) {
  constexpr int HB = __builtin_ctz(HS);
  uint32_t sl = ((uint32_t)v * 2654435761u) >> (32 - HB);
  while (h[sl] != v) sl = (sl + 1) & (HS - 1);
  return (int)sl;
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
                                                          int64_t* __restrict__ cnt) {
  __shared__ int32_t h[MSP_LOCAL_HASH_MULT * N2];
  __shared__ int32_t uq[N2];
  __shared__ int c;
  const int64_t t = blockIdx.x;
  int32_t m[N2 / kLT];
  const int tot = tile_distinct<T, N2>(nbr, K, n, t, h, uq, &c, m);
  if (threadIdx.x == 0) cnt[t] = tot;  // (the largest count: the scan's max_out)
}

// Rows of a tile into 16-row groups that share filter offsets (one wave, T / 64 rows per lane): each group is
// seeded with the free row of most neighbours and grown by the row that adds the fewest offsets to the group's
// union (ties: more neighbours, then the lower row).  conv_x6s runs one 16-row MFMA per (group, offset in the
// union), so the union sizes are its work: on the headline batch this fills 0.66 / 0.69 / 0.68 of those rows at
// levels 1-3 against 0.61 / 0.66 / 0.66 for rows sorted by mask (scripts/tile_fill.py).  Rows past nv (the
// padding of the last tile) come last.  ord[i] = tile row at position i; gmask[g] = group g's offset union.
// Wave-wide minimum of x (every lane gets it): DPP shifts inside each 16-lane row, then the four row minima by
// readlane -- no LDS round trips (a __shfl_xor ladder is six dependent ds_bpermute, and group_rows below runs
// one reduction per row of a tile, 128 in sequence).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  constexpr int kId = -1;  // 0xFFFFFFFF: what a lane shifted in from outside its row contributes
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)x, 0x111, 0xF, 0xF, false));  // row_shr:1
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)x, 0x112, 0xF, 0xF, false));  // row_shr:2
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)x, 0x114, 0xF, 0xF, false));  // row_shr:4
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)x, 0x118, 0xF, 0xF, false));  // row_shr:8
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)x, 15), b = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)x, 47), d = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return min(min(a, b), min(c, d));
}

template <int T>
__device__ void group_rows(const uint32_t* __restrict__ msk, int nv, uint8_t* __restrict__ ord,
                           uint32_t* __restrict__ gmask) {
  constexpr int RPL = T / 64;
  const int lane = threadIdx.x & 63;
  uint32_t m[RPL];
  int pc[RPL];
  bool fr[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int p = lane + 64 * j;
    m[j] = msk[p];
    pc[j] = __popc(m[j]);
    fr[j] = p < nv;
  }
  uint32_t um = 0;
  for (int pos = 0; pos < nv; ++pos) {
    const bool seed = (pos & 15) == 0;
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const int score = seed ? 64 - pc[j] : __popc(um | m[j]) * 64 - pc[j];
      const uint32_t key = ((uint32_t)score << 8) | (uint32_t)(lane + 64 * j);
      best = fr[j] && key < best ? key : best;
    }
    best = wave_min_u32(best);
    const int p = (int)(best & 0xFF);
#pragma unroll
    for (int j = 0; j < RPL; ++j)
      if (p == lane + 64 * j) fr[j] = false;
    uint32_t mp = m[0];  // row p's mask from its lane's registers (p is wave-uniform): no LDS round trip
#pragma unroll
    for (int j = 1; j < RPL; ++j)
      if ((p >> 6) == j) mp = m[j];
    um = (seed ? 0u : um) | (uint32_t)__builtin_amdgcn_readlane((int)mp, p & 63);
    if (lane == 0) ord[pos] = (uint8_t)p;
    if ((pos & 15) == 15 || pos == nv - 1) {
      if (lane == 0) gmask[pos >> 4] = um;
    }
  }
  for (int pos = nv + lane; pos < T; pos += 64) ord[pos] = (uint8_t)pos;
  for (int g = (nv + 15) / 16 + lane; g < T / 16; g += 64) gmask[g] = 0u;
}

// conv_x6s's offset lists of one 128-row tile: for row half h (groups h, h + 2, h + 4, h + 6) the offsets with
// at least one row in those groups, dealt to the half's 4 waves longest-first onto the least-loaded wave (load
// = 4 x groups + 1 per offset; at most 8 offsets a wave).  Interleaving the halves over the groups evens them
// out, and the lists even out the waves: the slowest of the 8 waves carries 0.94 of the mean against 0.86 for
// offsets dealt round-robin (headline batch, levels 1-3).  wo[h][c][k]: offset k of wave c (0xFF: none).
#ifndef MSP_SHARED_LISTS  // experiments: 1 = both halves walk one list dealt from all 8 groups (their weight loads
#define MSP_SHARED_LISTS 0  // then coincide, which the vector L1 can serve once)
#endif
// One wave deals both halves: lanes 32 h + o hold offset o's cost in half h; each lane ranks its offset (cost
// descending, then offset ascending: the order an insertion sort by cost gives) with K shuffles, the ranked lists
// go to LDS, and lanes 0 and 32 deal them out greedily from registers.  (Round 4's form ran the ranking as an
// insertion sort through LDS on one lane per half: ~K^2 / 2 dependent LDS round trips per tile.)
__device__ void deal_offsets(const uint32_t* __restrict__ gmask, int K, uint8_t* __restrict__ item,
                             int* __restrict__ cost, uint8_t* __restrict__ wo2) {
  const int lane = threadIdx.x & 63, h = lane >> 5, o = lane & 31;
  int a = 0;  // item / cost: [2][kKMax] LDS scratch; wo2: the tile's two halves' lists (2 x 32 bytes)
  if (o < K)
    for (int g = MSP_SHARED_LISTS ? 0 : h; g < 8; g += MSP_SHARED_LISTS ? 1 : 2) a += (gmask[g] >> o) & 1u;
  int r = 0;
  for (int q = 0; q < K; ++q) {
    const int aq = __shfl(a, (h << 5) + q, 64);
    r += (aq > a || (aq == a && q < o)) ? 1 : 0;
  }
  const unsigned long long nz = __ballot(a > 0);
  const int n = __popcll(h ? (nz >> 32) : (nz & 0xFFFFFFFFull));
  if (a > 0) {
    item[h * kKMax + r] = (uint8_t)o;
    cost[h * kKMax + r] = a;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (o != 0) return;
  int cs[kKMax];
#pragma unroll
  for (int i = 0; i < kKMax; ++i) cs[i] = cost[h * kKMax + i];
  uint8_t* wo = wo2 + h * 32;
  int l0 = 0, l1 = 0, l2 = 0, l3 = 0, n0 = 0, n1 = 0, n2 = 0, n3 = 0;  // load and count per wave
#pragma unroll
  for (int i = 0; i < kKMax; ++i) {
    if (i >= n) continue;  // (not break: the loop stays unrolled, cs[] in registers)
    int c = -1, lc = 0;
    if (n0 < 8) c = 0, lc = l0;
    if (n1 < 8 && (c < 0 || l1 < lc)) c = 1, lc = l1;
    if (n2 < 8 && (c < 0 || l2 < lc)) c = 2, lc = l2;
    if (n3 < 8 && (c < 0 || l3 < lc)) c = 3, lc = l3;
    const int add = 4 * cs[i] + 1;
    const int k = c == 0 ? n0++ : c == 1 ? n1++ : c == 2 ? n2++ : n3++;
    if (c == 0) l0 += add;
    else if (c == 1) l1 += add;
    else if (c == 2) l2 += add;
    else l3 += add;
    wo[c * 8 + k] = item[h * kKMax + i];
  }
  for (int k = n0; k < 8; ++k) wo[k] = 0xFF;
  for (int k = n1; k < 8; ++k) wo[8 + k] = 0xFF;
  for (int k = n2; k < 8; ++k) wo[16 + k] = 0xFF;
  for (int k = n3; k < 8; ++k) wo[24 + k] = 0xFF;
}

// conv_x6s's row order and offset lists of the tile-local rulebook (msp_tile_local, before the fill), one wave per
// tile: the rows' neighbour masks from nbr, group_rows' greedy 16-row groups, deal_offsets' per-wave lists, the
// order as perm.  group_rows is a serial chain of T wave-wide minima; run inside the fill's 256-thread block, only
// that block's first wave worked on it while three waited at the barrier, and the fill's LDS allowed four blocks
// per CU (~460 us over the headline batch's seven levels, scripts/build_bench.py).  Here a CU keeps up to 32
// tiles' chains in flight.
template <int T>
__global__ __launch_bounds__(256) void local_group_kernel(const int32_t* __restrict__ nbr, int K, int64_t n,
                                                          int64_t n_tiles, int32_t* __restrict__ perm,
                                                          uint8_t* __restrict__ wave_off) {
  __shared__ uint32_t msk[4][T];
  __shared__ uint8_t ord[4][T];
  __shared__ uint32_t gmask[4][T / 16];
  __shared__ uint8_t ditem[4][2 * kKMax];
  __shared__ int dcost[4][2 * kKMax];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + w;
  if (t >= n_tiles) return;  // wave-uniform: nothing below synchronises the block
  const int nv = (int)(n - t * T < T ? n - t * T : T);
  for (int p = lane; p < T; p += 64) {  // each lane's own rows (group_rows reads them back on the same lane)
    uint32_t m = 0;
    if (p < nv) {
      const int32_t* col = nbr + t * T + p;
#pragma unroll 9
      for (int o = 0; o < K; ++o) m |= (uint32_t)(col[(int64_t)o * n] >= 0) << o;
    }
    msk[w][p] = m;
  }
  group_rows<T>(msk[w], nv, ord[w], gmask[w]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // lane 0's ord / gmask stores before the other lanes read
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (T == 128 && wave_off && K <= kKMax) deal_offsets(gmask[w], K, ditem[w], dcost[w], wave_off + t * 64);
  for (int i = lane; i < T; i += 64) perm[t * T + i] = i < nv ? (int32_t)(t * T + ord[w][i]) : -1;
}

// MODE 0: the distinct-row lists only (the chunk-local weight gradient needs no row order; the block keeps to the
// 32 KB of the hash set and the list).  MODE 1: also the row order and offset lists, grouped inside the block by
// its first wave (few tiles: one kernel's latency), and the local indices.  MODE 2: the local indices in the order
// local_group_kernel wrote to perm (many tiles: that kernel keeps many tiles' grouping chains in flight).
template <int T, int N2, int MODE>
__global__ __launch_bounds__(kLT) void local_fill_kernel(const int32_t* __restrict__ nbr, int K, int64_t n,
                                                         int64_t n_pad, const int64_t* __restrict__ u_start,
                                                         int32_t* __restrict__ u_rows, uint16_t* __restrict__ lidx,
                                                         int32_t* __restrict__ perm, uint8_t* __restrict__ wave_off) {
  constexpr int HS = MSP_LOCAL_HASH_MULT * N2;
  __shared__ int32_t h[HS];
  __shared__ int32_t uq[N2];
  __shared__ uint8_t iord[MODE ? T : 1];  // where tile row p goes in the chosen order
  __shared__ uint32_t msk[MODE == 1 ? T : 1];
  __shared__ uint8_t ord[MODE == 1 ? T : 1];
  __shared__ uint32_t gmask[MODE == 1 ? T / 16 : 1];
  __shared__ uint8_t ditem[MODE == 1 ? 2 * kKMax : 1];
  __shared__ int dcost[MODE == 1 ? 2 * kKMax : 1];
  __shared__ int c;
  const int64_t t = blockIdx.x;
  int32_t m[N2 / kLT];
  const int tot = tile_distinct<T, N2>(nbr, K, n, t, h, uq, &c, m, MODE == 1 ? msk : nullptr);
  // the distinct rows in ascending order
  int n2 = 2;
  while (n2 < tot) n2 <<= 1;
  for (int i = tot + threadIdx.x; i < n2; i += kLT) uq[i] = INT32_MAX;
  __syncthreads();
  bitonic_i32_n(uq, n2);
  const int64_t u0 = u_start[t];
  for (int i = threadIdx.x; i < tot; i += kLT) u_rows[u0 + i] = uq[i];
  if constexpr (MODE == 0) return;
  // each distinct row's slot now holds the row's sorted position (slots found first, then rewritten: a probe
  // compares uq[h[slot]] with the row from here on)
  {
    int sl[N2 / kLT];
#pragma unroll
    for (int j = 0; j < N2 / kLT; ++j) {
      const int i = threadIdx.x + kLT * j;
      sl[j] = i < tot ? hash_slot<HS>(h, uq[i]) : -1;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < N2 / kLT; ++j)
      if (sl[j] >= 0) h[sl[j]] = threadIdx.x + kLT * j;
  }
  if constexpr (MODE == 1) {  // rows grouped by shared offsets (padding rows last); msk was set by tile_distinct
    const int nv = (int)(n - t * T < T ? n - t * T : T);
    if (threadIdx.x < 64) group_rows<T>(msk, nv, ord, gmask);
    __syncthreads();
    if (T == 128 && wave_off && K <= kKMax && threadIdx.x < 64) deal_offsets(gmask, K, ditem, dcost, wave_off + t * 64);
    for (int i = threadIdx.x; i < T; i += kLT) {
      perm[t * T + i] = i < nv ? (int32_t)(t * T + ord[i]) : -1;
      iord[ord[i]] = (uint8_t)i;
    }
  } else {
    for (int i = threadIdx.x; i < T; i += kLT) {  // perm: local_group_kernel's row order (padding last, in place)
      const int32_t r = perm[t * T + i];
      iord[r >= 0 ? (int)(r - t * T) : i] = (uint8_t)i;
    }
  }
  __syncthreads();
  // local index of every (offset, row) entry this thread holds, written at the row's ordered position
#pragma unroll
  for (int j = 0; j < N2 / kLT; ++j) {
    const int i = threadIdx.x + kLT * j;
    if (i < K * T) {
      const int o = i / T, p = i - o * T;
      const int32_t v = m[j];
      uint16_t li = kAbsent;
      if (v >= 0) {
        constexpr int HB = __builtin_ctz(HS);
        uint32_t q = ((uint32_t)v * 2654435761u) >> (32 - HB);
        int pos;
        while (uq[pos = h[q]] != v) q = (q + 1) & (HS - 1);  // the probe path of v holds only inserted rows
        li = (uint16_t)pos;
      }
      lidx[(int64_t)o * n_pad + t * T + iord[p]] = li;
    }
  }
}

// ---------------------------------------------------------------- weights
// wt -> lane-ordered weight image: unit ((((o * n_y + cy) * nks + ks) * NT + t) * 3 + p) * 64 + lane holds,
// for lane = 16 q + r, W^T[out 16 (cy NT + t) + r][k 32 ks + 8 q .. + 7] (zero past c_in) as its three bf16
// pieces p (split once here), so a wave loads its fragments of one step as 3 NT coalesced 1 KiB rows.  wlay 1:
// wt is [K][c_in][c_out] (the module's layout), else [K][c_out][c_in].
__global__ __launch_bounds__(256) void split_weights_lane_kernel(const float* __restrict__ wt, int K, int c_out,
                                                                 int c_in, int NT, u32x4* __restrict__ img,
                                                                 int wlay) {
  split_weights_lane_unit(wt, K, c_out, c_in, NT, img, wlay, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// Every image of a step in one launch (msp_split_weight_images): the block's first unit finds its image by one
// binary search in the units' prefix sums (thread 0; a per-thread search was seven dependent global loads per
// unit), and each thread steps forward from there to its own image (a block spans one or two images).
__global__ __launch_bounds__(256) void split_images_kernel(const msp_weight_image* __restrict__ d, int n,
                                                           const int64_t* __restrict__ start, int64_t total) {
  __shared__ int s_lo;
  const int64_t g0 = (int64_t)blockIdx.x * 256, g = g0 + threadIdx.x;
  if (threadIdx.x == 0) {
    int lo = 0, hi = n;  // start[lo] <= g0 < start[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (start[mid] <= g0) lo = mid;
      else hi = mid;
    }
    s_lo = lo;
  }
  __syncthreads();
  if (g >= total) return;
  int lo = s_lo;
  while (lo + 1 < n && start[lo + 1] <= g) ++lo;
  const msp_weight_image e = d[lo];
  const int64_t u = g - start[lo];
  u32x4* img = static_cast<u32x4*>(e.img);
  if (e.kind == 2) split_weights_lane_unit(e.wt, e.K, e.c_out, e.c_in, e.p, img, e.wlay, u);
  else split_weights_unit(e.wt, e.K, e.c_out, e.c_in, e.p, 32, img, e.wlay, u);
}

// ---------------------------------------------------------------- convolution
// staged row j of the 32-channel slice: 12 units (piece p, k-octet qq) at p * 4 + (qq ^ sw(j)).  A ds_read_b128
// lane group on gfx950 is lanes {0-3, 12-15, 20-27} (and three more like it, MI355X_MICROARCH.md §LDS): with lane
// = 16 qq + r it holds the 16 row positions r once each, at octet qq = c for r in 0-3 / 12-15 and c ^ 1 for r in
// 4-11.  Row j's units start at quad 12 j mod 16 = 4 ((-j) mod 4); sw(j) = h ^ [h in {1, 2}] with h = (j >> 2) & 3
// cancels that octet flip, so 16 rows with distinct j mod 16 read 16 distinct bank quads (the plain h swizzle,
// written for contiguous 16-lane groups, paired r with r + 4 on one quad).
__device__ __forceinline__ int xs_sw(int j) {
  const int h = (j >> 2) & 3;
  return h ^ ((h ^ (h >> 1)) & 1);
}
__device__ __forceinline__ int xs_unit(int j, int p, int qq) { return j * kXU + p * 4 + (qq ^ xs_sw(j)); }

// conv_x6s: block = 8 waves = 2 row halves x 4 waves on one 128-row tile and 16 NT output columns.  Half h
// holds the tile's 16-row groups h, h + 2, h + 4, h + 6 (the groups are ordered by how many offsets they
// carry, so interleaving evens the halves out); wave c of half h walks the offsets wave_off lists for it
// (msp_tile_local: every offset some row of the half has, dealt longest-first; NULL: o = c + 4 j), keeping its
// G = 4 groups x NT column tiles of accumulators in registers.  Per 32-input-channel slice the tile's distinct
// rows (row indices loaded once per tile and kept in registers; the slice's value loads all in flight at once)
// are staged as exact bf16 pieces; per offset a wave reads its groups' 16 local indices (one LDS wait), takes
// wave-uniform masks of the groups with the offset and with rows past the staged capacity, and per active
// group issues three LDS reads and 6 NT MFMAs.  Weight fragments come from the lane-ordered image one offset
// ahead.  The four waves' partial sums of a half are added in wave order through LDS at the end (deterministic).
// AB (experiments build only; wrong results): bit 0 stages without the global value loads, bit 2 keeps the
// first offset's weight fragments, bit 3 reads staged row 16 g + r for every present rule (16 distinct j mod 16 per
// lane group: no bank conflict) -- the ablations that price the staging, weight-load and LDS-conflict costs.
// AC (accumulation): 1 = the six piece products of a step go straight into the group's running sums, smallest
// first (the product form); 0 = summed in a zeroed accumulator and added with a vector add (round 2-3 form:
// about a third of the rounding error, 6-9 % slower -- profiles/r03/kbexp_r03x_accumulate.log).
// WB (weight fragment register sets): 1 = one set, the next step's fragments loaded after the step's MFMAs (their
// latency exposed at the next step's start); 2 = two sets alternating, the next step's fragments loaded before the
// step's MFMAs, so a whole step hides their latency (the first step of each slice loads after the staging).
// EPI (msp_bn_epilogue, round 6): the BatchNorm sums of the rows written; its own instantiation, so the plain form
// compiles exactly as before (the epilogue's registers and loads never touch it).
template <int NT, int AB = 0, int AC = 1, int WB = 1, bool EPI = false>
__global__ __launch_bounds__(512, 4) void conv_x6s_kernel(
    const float* __restrict__ x, int c_in, const u32x4* __restrict__ wimg, int K, int flip, int c_out,
    const uint16_t* __restrict__ lidx, const int64_t* __restrict__ u_start, const int32_t* __restrict__ u_rows,
    const int32_t* __restrict__ perm, const uint8_t* __restrict__ wave_off, int64_t n_pad, int n_y,
    float* __restrict__ out, BnEpi epi) {
  constexpr int T = 128, NTH = 512, G = 4;
  constexpr int NC = 16 * NT;
  static_assert(4 * T * NC * 4 <= kXR * kXU * 16, "partial sums must fit the staging area");
  __shared__ u32x4 xs[kXR * kXU];
  __shared__ __attribute__((aligned(16))) uint16_t ls[kKMax * T];
  __shared__ uint32_t wl[16];  // the tile's offset lists, [half][wave][8 bytes]
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wc = wave & 3, rp = wave >> 2;  // wave of the half, row half
  const int r = lane & 15, q = lane >> 4;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int cy = (int)(lb % n_y);
  const int64_t tile = lb / n_y;
  const int64_t u0 = u_start[tile];
  const int U = (int)(u_start[tile + 1] - u0);
  const int Us = U < kUCap ? U : kUCap;
  const int nks = (c_in + 31) / 32;
  {  // the index tile as 32-bit words, every load in flight before the LDS stores
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
    uint32_t lv = 0u;
    if (tid < 16) {
      if (wave_off) {
        lv = reinterpret_cast<const uint32_t*>(wave_off)[tile * 16 + tid];
      } else {  // word tid: half tid / 8, wave (tid / 2) % 4, slots 4 (tid % 2) .. + 3 of o = wave + 4 j
        const int c = (tid >> 1) & 3, j0 = 4 * (tid & 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int o = c + 4 * (j0 + k);
          lv |= (uint32_t)(o < K ? o : 0xFF) << (8 * k);
        }
      }
    }
#pragma unroll
    for (int b = 0; b < LW; ++b) {
      const int i = tid + NTH * b;
      if (i < K * T / 2) reinterpret_cast<uint32_t*>(ls)[i] = wv[b];
    }
    if (tid < 16) wl[tid] = lv;
  }
  if (tid < kXU) xs[kUCap * kXU + tid] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();  // index tile, offset lists, zero row
  // this wave's offsets (wave-uniform): up to 8 bytes, packed from the first, 0xFF past the last
  const uint64_t list = (uint64_t)__builtin_amdgcn_readfirstlane(wl[rp * 8 + wc * 2]) |
                        ((uint64_t)__builtin_amdgcn_readfirstlane(wl[rp * 8 + wc * 2 + 1]) << 32);
  int n_j = 0;
  while (n_j < 8 && ((list >> (8 * n_j)) & 0xFF) != 0xFF) ++n_j;
  auto off_of = [&](int j) { return (int)((list >> (8 * j)) & 0xFF); };

  floatx4 acc[G][NT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int n_steps = nks * n_j;
  auto ld_w = [&](int s, u32x4 (&w)[NT][3]) {  // fragments of step s = (slice, list position)
    const int sc = s < n_steps ? s : n_steps - 1;
    const int ks = sc / n_j, j = sc - ks * n_j;
    const int o = off_of(j);
    const int ow = flip ? K - 1 - o : o;
    if constexpr (WB == 2) {  // wave-uniform row base (scalar registers) + the lane's 32-bit byte offset
      const u32x4* src = wimg + ((((int64_t)ow * n_y + cy) * nks + ks) * NT) * 3 * 64;
      const char* b = reinterpret_cast<const char*>(src);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          w[t][p] = *reinterpret_cast<const u32x4*>(b + (uint32_t)(((t * 3 + p) * 64 + lane) * 16));
      return;
    }
    const u32x4* src = wimg + ((((int64_t)ow * n_y + cy) * nks + ks) * NT) * 3 * 64 + lane;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) w[t][p] = src[(t * 3 + p) * 64];
  };
  // the thread's staged row indices, loaded once per tile; every 32-channel slice then issues all of its value
  // loads at once (one global latency per slice instead of index -> value)
  constexpr int MI = (kUCap * 4 + NTH - 1) / NTH;
  int32_t srow[MI];
#pragma unroll
  for (int b = 0; b < MI; ++b) {
    const int i = tid + NTH * b;
    srow[b] = i < Us * 4 ? u_rows[u0 + (i >> 2)] : 0;
  }
  auto stage = [&](int ks) {
    const int k0 = 32 * ks;
    floatx4 v[MI][2];
#pragma unroll
    for (int b = 0; b < MI; ++b) {
      // WB 2: the row addresses are formed here, per slice (hoisted out of the slice loop they hold 6 registers
      // for the whole kernel, which the second weight set needs)
      if constexpr (WB == 2) asm volatile("" : "+v"(srow[b]));
      const int i = tid + NTH * b;
      const int k = k0 + 8 * (i & 3);
      v[b][0] = v[b][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (i < Us * 4 && k < c_in) {
        if constexpr (AB & 1) {
          v[b][0] = v[b][1] = floatx4{(float)srow[b], 1.f, 2.f, 3.f};
        } else {
          const floatx4* src = reinterpret_cast<const floatx4*>(x + (int64_t)srow[b] * c_in + k);
          v[b][0] = src[0];
          v[b][1] = src[1];
        }
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
  // one (k-slice, offset) step of this wave over its row groups; FAR: the tile lists rows past the staged capacity
  auto run = [&](int ks, int o, const u32x4 (&w)[NT][3], auto FAR) {
    const uint16_t* lo = ls + o * T + 16 * rp + r;
    int li[G];
#pragma unroll
    for (int g = 0; g < G; ++g) li[g] = lo[32 * g];  // group 2 g + rp
    uint32_t act = 0, far = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool pres = li[g] != kAbsent;
      act |= (ballot64(pres) != 0 ? 1u : 0u) << g;
      if constexpr (decltype(FAR)::value) far |= (ballot64(pres && li[g] >= kUCap) != 0 ? 1u : 0u) << g;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if ((act >> g) & 1) {  // wave-uniform
        u32x4 cur[3];
        int jr = li[g] < kUCap ? li[g] : kUCap;  // absent (0xFFFF) and far rows -> zero row
        if constexpr ((AB & 8) != 0) jr = li[g] < kUCap ? 16 * g + r : kUCap;  // ablation: conflict-free reads
#pragma unroll
        for (int p = 0; p < 3; ++p) cur[p] = xs[xs_unit(jr, p, q)];
        if (decltype(FAR)::value && ((far >> g) & 1)) {  // rows past the staged capacity: from global memory (rare)
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
        if constexpr (AC == 1) {  // smallest products first, straight into the running sums
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_bf16(w[t][2], cur[0], acc[g][t]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_bf16(w[t][1], cur[1], acc[g][t]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_bf16(w[t][0], cur[2], acc[g][t]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_bf16(w[t][1], cur[0], acc[g][t]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_bf16(w[t][0], cur[1], acc[g][t]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_bf16(w[t][0], cur[0], acc[g][t]);
        } else {
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
    }
  };

  // msp_bn_epilogue, backward: the BN input rows the epilogue reads (its output rows' quads), loaded at the start of
  // the last k-slice so their latency hides under that slice's MFMAs instead of ending the block
  constexpr int QPR = NC / 4;  // float4 quads per output row
  constexpr int EPR = T * QPR / NTH;
  static_assert(EPR * NTH == T * QPR && 64 % QPR == 0, "a thread keeps one column quad in the epilogue");
  floatx4 epx[EPR];
  int32_t epd[EPR];
  auto epi_prefetch = [&]() {
    if constexpr (!EPI) return;
#pragma unroll
    for (int e = 0; e < EPR; ++e) {
      const int i = tid + NTH * e, row = i / QPR, cq = i - row * QPR;
      epd[e] = perm[tile * T + row];
      epx[e] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (epi.x != nullptr && epd[e] >= 0)
        epx[e] = *reinterpret_cast<const floatx4*>(epi.x + (int64_t)epd[e] * epi.C + cy * NC + 4 * cq);
    }
  };

  using Far = std::true_type;
  using Near = std::false_type;
  if (WB == 2 && U <= kUCap) {  // block-uniform: every listed row is staged (all but 0-0.09 % of tiles)
    // Two fragment sets: step j of a slice runs on set j & 1 while the next step's fragments load into the other.
    // The step loop has a fixed trip count of 8 (the longest offset list) and is unrolled, with every load
    // unconditional (steps past the list reload a valid step; the last one of a slice loads the next slice's
    // first), so the compiler's in-order load count waits only for the older set at each step's first MFMA --
    // data-dependent branches around the loads would leave a vmcnt(0) there instead.
    u32x4 wa[NT][3], wb[NT][3];
    auto ld_next = [&](int ks, int j, u32x4 (&w)[NT][3]) {  // fragments of the step after (ks, j)
      const int s1 = j + 1 < n_j ? ks * n_j + j + 1 : (ks + 1 < nks ? (ks + 1) * n_j : ks * n_j + n_j - 1);
      ld_w(s1, w);
    };
    if (n_j) ld_w(0, wa);
    for (int ks = 0; ks < nks; ++ks) {
      if (ks) __syncthreads();  // previous slice's readers done
      stage(ks);
      __syncthreads();
      if (ks == nks - 1) epi_prefetch();
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        ld_next(ks, j, wb);
        if (j < n_j) run(ks, off_of(j), wa, Near{});
        ld_next(ks, j + 1, wa);
        if (j + 1 < n_j) run(ks, off_of(j + 1), wb, Near{});
      }
    }
  } else {
    u32x4 wf[NT][3];
    if (n_j) ld_w(0, wf);
    for (int ks = 0; ks < nks; ++ks) {
      if (ks) __syncthreads();  // previous slice's readers done
      stage(ks);
      __syncthreads();
      if (ks == nks - 1) epi_prefetch();
      for (int j = 0; j < n_j; ++j) {
        run(ks, off_of(j), wf, Far{});
        if constexpr (!(AB & 4)) ld_w(ks * n_j + j + 1, wf);
      }
    }
  }
  // the four waves' partial sums of each half, added in wave order
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t)
      *reinterpret_cast<floatx4*>(red + ((int64_t)(wc * T + 16 * (2 * g + rp) + r)) * NC + 16 * t + 4 * q) =
          acc[g][t];
  __syncthreads();
  // msp_bn_epilogue (block-uniform): the BatchNorm sums of the rows written, per thread for its column quad
  // tid % QPR, then over the wave's lanes and the 8 waves in order into this tile's slot
  if constexpr (!EPI) {
    for (int i = tid; i < T * QPR; i += NTH) {
      const int row = i / QPR, cq = i - row * QPR;
      const float* pr = red + row * NC + 4 * cq;
      floatx4 v = *reinterpret_cast<const floatx4*>(pr);
#pragma unroll
      for (int w = 1; w < 4; ++w) v += *reinterpret_cast<const floatx4*>(pr + w * T * NC);
      const int32_t dst = perm[tile * T + row];
      if (dst >= 0) *reinterpret_cast<floatx4*>(out + (int64_t)dst * c_out + cy * NC + 4 * cq) = v;
    }
    return;
  }
  BnEpiAcc ea;
  ea.init(epi, cy * NC + 4 * (tid % QPR));
#pragma unroll
  for (int e = 0; e < EPR; ++e) {
    const int i = tid + NTH * e, row = i / QPR, cq = i - row * QPR;
    const float* pr = red + row * NC + 4 * cq;
    floatx4 v = *reinterpret_cast<const floatx4*>(pr);
#pragma unroll
    for (int w = 1; w < 4; ++w) v += *reinterpret_cast<const floatx4*>(pr + w * T * NC);
    const int32_t dst = epd[e];
    if (dst >= 0) {
      *reinterpret_cast<floatx4*>(out + (int64_t)dst * c_out + cy * NC + 4 * cq) = v;
      ea.add_x(epi, v, epx[e]);
    }
  }
  {
    ea.wave_reduce<QPR>();
    double* scr = reinterpret_cast<double*>(ls);  // the index tile is no longer read: NTH / 64 x QPR x 8 doubles
    static_assert((NTH / 64) * QPR * 8 * 8 <= (int)sizeof(ls), "epilogue scratch must fit the index tile");
    if (lane < QPR)
#pragma unroll
      for (int k = 0; k < 8; ++k) scr[(wave * QPR + lane) * 8 + k] = ea.s[k];
    __syncthreads();
    if (tid < QPR * 8) {
      const int cq = tid >> 3, k = tid & 7;
      double a = 0.0;
#pragma unroll
      for (int w = 0; w < NTH / 64; ++w) a += scr[(w * QPR + cq) * 8 + k];
      *bn_epi_slot(epi, k >> 2, cy * NC + 4 * cq + (k & 3), tile) = a;
    }
  }
}

// dW[e] = sum of slab[range][e] over the ranges: 16 consecutive runs of ranges, each added in range order by one
// thread (eight loads in flight), then the 16 run sums in run order (deterministic).  Block = 16 float4 elements x
// 16 runs: the slab (256 ranges x K c_in c_out floats, 28 MB at every shape) is read with 16x the loads in flight
// of one thread per element walking all ranges (a latency-bound 17 us per call, 0.8 ms per step).
constexpr int kRRuns = 16;
__global__ __launch_bounds__(256) void wgrad_ranges_reduce_kernel(const floatx4* __restrict__ slab, int n_ranges,
                                                                  int64_t n4, floatx4* __restrict__ dw) {
  __shared__ floatx4 part[kRRuns][16];
  const int el = threadIdx.x & 15, run = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + el;
  const int k0 = n_ranges * run / kRRuns, k1 = n_ranges * (run + 1) / kRRuns;
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    int k = k0;
    for (; k + 8 <= k1; k += 8) {
      floatx4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)(k + u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < k1; ++k) s += slab[(int64_t)k * n4 + i];
  }
  part[run][el] = s;
  __syncthreads();
  if (run == 0 && i < n4) {
    floatx4 t = part[0][el];
#pragma unroll
    for (int r = 1; r < kRRuns; ++r) t += part[r][el];
    dw[i] = t;
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
#ifndef MSP_X6C_CAP  // experiments: 384 keeps the block (with 72-byte rows) + one 32 KB build block within a CU's LDS
#define MSP_X6C_CAP 448
#endif
constexpr int kWCap = MSP_X6C_CAP;  // distinct rows per 128-row tile the weight gradient stages (msp_conv_wgrad_chunk)
constexpr uint32_t kWFar = 0xFFFFu;  // chunk entry whose input row lies past kWCap (never staged)

constexpr int kWTile = 128;

// Weight-gradient index from the tile-local rulebook (msp_tile_local, 128-row tiles): the tile's sorted
// distinct input rows are already listed there, so each chunk entry of the 128-row tile rulebook only needs its
// position in that list (binary search; rows past the list's staged capacity are excluded on the host).
// The chunk weight gradient's index straight from the full tile-local rulebook (msp_local_chunk_index, round 5):
// per 128-row tile and offset, the present entries of lidx (in natural row order) compacted into 16-entry
// chunks, offsets ascending, chunk_lr = local position | natural row << 16, padding slots (position 0, row 128:
// the zero dy row).  Where a tile-local convolution built that rulebook anyway (levels 1-4), this replaces the
// 128-row tile rulebook's two passes over the K x n map and msp_wgrad_chunk_index's binary searches.
constexpr int kLCE = (kKMax * kWTile + kLT - 1) / kLT;  // lidx entries per thread (entry tid + kLT j)
__global__ __launch_bounds__(kLT) void lchunk_count_kernel(const uint16_t* __restrict__ lidx, int K, int64_t n_pad,
                                                           int64_t* __restrict__ cnt) {
  __shared__ int cs[kKMax];
  const int64_t t = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid < kKMax) cs[tid] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kLCE; ++j) {
    const int e = tid + kLT * j, o = e >> 7;  // a wave's 64 entries share one offset
    const bool pres = o < K && lidx[(int64_t)o * n_pad + t * kWTile + (e & 127)] != kAbsent;
    const unsigned long long b = __ballot(pres);
    if ((tid & 63) == 0 && o < K) atomicAdd(&cs[o], __popcll(b));
  }
  __syncthreads();
  if (tid < 64) {
    int64_t c = tid < K ? (cs[tid] + MSP_CHUNK - 1) / MSP_CHUNK : 0;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    if (tid == 0) cnt[t] = c;
  }
}

__global__ __launch_bounds__(kLT) void lchunk_fill_kernel(const uint16_t* __restrict__ lidx,
                                                          const int32_t* __restrict__ perm, int K, int64_t n_pad,
                                                          const int64_t* __restrict__ tile_start,
                                                          uint8_t* __restrict__ chunk_off,
                                                          uint32_t* __restrict__ chunk_lr) {
  __shared__ int hc[kKMax][2];  // present entries per (offset, half of the tile's rows)
  __shared__ int cst[kKMax];    // first chunk of each offset (relative to the tile)
  __shared__ uint8_t iord[kWTile];  // natural row -> the rulebook's position of it (inverse of perm)
  const int64_t t = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < kWTile) {
    const int32_t r = perm[t * kWTile + tid];
    iord[r >= 0 ? (int)(r - t * kWTile) : tid] = (uint8_t)tid;
  }
  __syncthreads();
  // entries in natural row order: a chunk's dy rows are then mostly consecutive (the transposing dy reads of
  // wgrad_x6c; in the rulebook's grouped order they scatter: +0.25 ms/step of wgrad_x6c, ab_r05ak_local_chunk)
  uint16_t v[kLCE];
#pragma unroll
  for (int j = 0; j < kLCE; ++j) {
    const int e = tid + kLT * j, o = e >> 7;
    v[j] = o < K ? lidx[(int64_t)o * n_pad + t * kWTile + iord[e & 127]] : kAbsent;
    const unsigned long long b = __ballot(v[j] != kAbsent);
    if (lane == 0 && o < K) hc[o][(e >> 6) & 1] = __popcll(b);
  }
  __syncthreads();
  if (tid < 64) {  // chunk starts: exclusive prefix over offsets of ceil(count / 16)
    const int c = tid < K ? (hc[tid][0] + hc[tid][1] + MSP_CHUNK - 1) / MSP_CHUNK : 0;
    int incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (tid < K) cst[tid] = incl - c;
  }
  __syncthreads();
  const int64_t c0 = tile_start[t];
#pragma unroll
  for (int j = 0; j < kLCE; ++j) {
    const int e = tid + kLT * j, o = e >> 7, i = e & 127;
    const bool pres = v[j] != kAbsent;
    const unsigned long long b = __ballot(pres);
    if (pres) {
      const int rank = ((e >> 6) & 1 ? hc[o][0] : 0) + __popcll(b & ((1ull << lane) - 1ull));
      chunk_lr[(c0 + cst[o]) * MSP_CHUNK + rank] = (uint32_t)v[j] | ((uint32_t)i << 16);
    }
  }
  if (tid < K) {  // the offset's chunks: their offset byte and the padding slots of the last one
    const int c = hc[tid][0] + hc[tid][1], nch = (c + MSP_CHUNK - 1) / MSP_CHUNK;
    for (int k = 0; k < nch; ++k) chunk_off[c0 + cst[tid] + k] = (uint8_t)tid;
    for (int r = c; r < nch * MSP_CHUNK; ++r) chunk_lr[(c0 + cst[tid]) * MSP_CHUNK + r] = (uint32_t)kWTile << 16;
  }
}

__global__ __launch_bounds__(kLT) void chunk_lidx_kernel(const int64_t* __restrict__ tile_start,
                                                         const int32_t* __restrict__ chunk_src,
                                                         const uint16_t* __restrict__ chunk_row,
                                                         const int64_t* __restrict__ u_start,
                                                         const int32_t* __restrict__ u_rows,
                                                         uint32_t* __restrict__ chunk_lr,
                                                         unsigned long long* __restrict__ n_far) {
  __shared__ int32_t uq[kWCap];
  const int64_t t = blockIdx.x;
  const int64_t u0 = u_start[t];
  const int U = (int)(u_start[t + 1] - u0);
  const int Us = U < kWCap ? U : kWCap;
  for (int i = threadIdx.x; i < Us; i += kLT) uq[i] = u_rows[u0 + i];
  __syncthreads();
  const int64_t e0 = tile_start[t] * MSP_CHUNK, e1 = tile_start[t + 1] * MSP_CHUNK;
  int n_over = 0;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kLT) {
    const int32_t v = chunk_src[e];
    int lo = 0, hi = Us;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (uq[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    const int rt = chunk_row[e];
    const bool far = lo >= Us && rt < kWTile;  // a rule (not a padding slot) whose row is not staged
    n_over += far;
    chunk_lr[e] = (uint32_t)(lo < Us ? lo : kWFar) | ((uint32_t)(rt >= kWTile ? kWTile : rt) << 16);
  }
  if (n_far && n_over) atomicAdd(n_far, (unsigned long long)n_over);
}

// Rules whose input row lies past a tile's staged capacity (chunk_lr 0xFFFF with a real row): one block per tile
// hands each such entry a slot of the list (slots in arrival order; msp_wgrad_far_list then sorts the list by
// (offset, entry), so the correction below sums in a fixed order).
constexpr int kFarShift = 40;  // far_key = offset << 40 | chunk entry
__global__ __launch_bounds__(kLT) void far_collect_kernel(const int64_t* __restrict__ tile_start,
                                                          const uint8_t* __restrict__ chunk_off,
                                                          const uint32_t* __restrict__ chunk_lr, int64_t n_far,
                                                          unsigned long long* __restrict__ ctr,
                                                          uint64_t* __restrict__ keys, int32_t* __restrict__ tiles) {
  const int64_t t = blockIdx.x;
  const int64_t e0 = tile_start[t] * MSP_CHUNK, e1 = tile_start[t + 1] * MSP_CHUNK;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kLT) {
    const uint32_t w = chunk_lr[e];
    if ((w & 0xFFFFu) != kWFar || (w >> 16) >= (uint32_t)kWTile) continue;
    const unsigned long long slot = atomicAdd(ctr, 1ull);
    if ((int64_t)slot >= n_far) continue;  // more than counted: cannot happen for the index that counted them
    keys[slot] = ((uint64_t)chunk_off[e / MSP_CHUNK] << kFarShift) | (uint64_t)e;
    tiles[slot] = (int32_t)t;
  }
}

// dw[o][ci0 .. +32][co0 .. +32] += the far rules of offset o, in list order (fp64 sums): block = one (offset,
// 32 x 32 slice), thread = (one input channel, four output channels).
__global__ __launch_bounds__(256) void wgrad_far_kernel(const float* __restrict__ x, int c_in,
                                                        const float* __restrict__ dy, int c_out,
                                                        const int32_t* __restrict__ chunk_src,
                                                        const uint16_t* __restrict__ chunk_row,
                                                        const uint64_t* __restrict__ keys,
                                                        const int32_t* __restrict__ tiles, int64_t n_far,
                                                        float* __restrict__ dw) {
  const int n_sl_o = c_out / 32, n_slices = (c_in / 32) * n_sl_o;
  const int o = (int)(blockIdx.x / n_slices), sl = (int)(blockIdx.x % n_slices);
  const int ci0 = 32 * (sl / n_sl_o), co0 = 32 * (sl % n_sl_o);
  const int ci = threadIdx.x >> 3, co = 4 * (threadIdx.x & 7);
  auto first_at_least = [&](uint64_t k) {  // first list position with key >= k
    int64_t lo = 0, hi = n_far;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const int64_t k0 = first_at_least((uint64_t)o << kFarShift), k1 = first_at_least((uint64_t)(o + 1) << kFarShift);
  if (k0 >= k1) return;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // fp64: exact products, the list's sum rounded once into dw
  for (int64_t k = k0; k < k1; ++k) {
    const int64_t e = (int64_t)(keys[k] & ((1ull << kFarShift) - 1));
    const int64_t i = chunk_src[e], j = (int64_t)tiles[k] * kWTile + chunk_row[e];
    const double xv = x[i * c_in + ci0 + ci];
    const floatx4 d = *reinterpret_cast<const floatx4*>(dy + j * c_out + co0 + co);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += xv * (double)d[q];
  }
  floatx4* out = reinterpret_cast<floatx4*>(dw + ((int64_t)o * c_in + ci0 + ci) * c_out + co0 + co);
  floatx4 v = *out;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = (float)((double)v[q] + acc[q]);
  *out = v;
}

constexpr int kWMaxCh = 216;                   // chunks of one 128-row tile (K <= 27 offsets x 8)
// wgrad_x6c's offset deal (DL 1): the offsets of wave w, one per byte from the low end, 0xFF past the last
__device__ __constant__ const uint32_t kX6cDeal[8] = {0x1a150a06u, 0x19141103u, 0x120f0502u, 0xff130c01u,
                                                      0xff090704u, 0xffff0e0du, 0xff161000u, 0x18170b08u};

// bf16 element offset of 8-byte unit v (channels 4v .. 4v+3 of the slice) of row j in a piece image
__device__ __forceinline__ int wimg_off(int j, int v) { return j * 32 + 4 * (v ^ (((j >> 2) & 1) << 2)); }
// RS (row stride of the piece images, bf16 elements): 32 = the XOR-swizzled layout above; 36 = rows padded to 72
// bytes, unswizzled, so the 16 rows one transposing read names start at 8-byte granules spread over the banks instead
// of eight 32-byte windows (experiments: the round-4 PMC put bank conflicts at 0.42 of the kernel's LDS cycles)
#ifndef MSP_X6C_RS  // the product's image row stride (experiments: 32 = the round-2..4 swizzled rows)
#define MSP_X6C_RS 36
#endif
template <int RS>
__device__ __forceinline__ int wimg_off_rs(int j, int v) {
  if constexpr (RS == 32) return wimg_off(j, v);
  return j * RS + 4 * v;
}

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

// AC as conv_x6s: 1 (the product form) accumulates the six piece products straight into the running tile sums,
// 0 sums each step in a zeroed accumulator first (12-16 % slower, profiles/r03/kbexp_r03x_accumulate.log).
// PW 1 (the product form): the next k-step's rule words are read from LDS at the start of the current one (within
// an offset), so a k-step no longer opens with an LDS read -> address -> transposing-read chain: 1-6 % faster at
// levels 0-3 (profiles/r03/kbexp_r03pw.log); PW 0 reads them at the k-step's start.
// ABL (experiments build only; wrong results): bit 0 keeps the first tile's LDS images for every tile (no split and
// no image writes after the first tile; the rule words and offsets are still staged), bit 1 drops the next tile's
// value loads -- the ablations that price the per-tile staging (round 6: -20 %, profiles/r06/kbexp_r06m_x6c_staging.log).
// DT 1 (direct offset table, the product since round 6): each chunk's neighbours' offsets come with its own from
// global memory, so the table of the offsets' chunk ranges is written in the same phase as the images
// (double-buffered, the idle buffer zeroed there): one block barrier per tile instead of two, 7-15 % faster at
// levels 0-3 (profiles/r06/kbexp_r06o_x6c_table_balance_split.log).  DT 0: the table built through LDS after the
// images (round 2-5).  Measured there and not kept: splitting the next tile's values in registers before the
// barrier (38 VGPRs past the 256 two waves per SIMD allow: spills, 20-40 % slower) and dealing the offsets over the
// waves by the range's chunk counts (no gain: -2 % to +8 %).
// BR > 0 (balanced ranges): the blocks' contiguous tile ranges hold equal cost, chunks + BR per tile (the staging's
// share), instead of equal tile counts; each block finds its bounds in tile_start (a prefix sum of chunks) with two
// rounds of block-wide counts.  Still a fixed function of the index: deterministic.  The product runs BR = 128:
// against equal tile counts 2-4 % faster at levels 0-1, 8 % at level 2, 10-12 % at level 3, 3-6 % at level 4 (the
// few-tile levels' ranges of 17 or 18 tiles differed by a tile; profiles/r06/kbexp_r06{q,r}_x6c_balanced_ranges.log).
// DL 1 (offset deal table, NW = 8): wave w owns the offsets of kX6cDeal[w] instead of w, w + 8, ...  Every tile
// waits at its barrier for its slowest wave, and on surfaces the round-robin deal stacks one plane's heavy offsets
// on a few waves: the slowest wave carries 1.38 / 1.31 / 1.28 / 1.24 / 1.21 x the mean k-steps at levels 0-4 of the
// headline batch.  The table was chosen offline by local search over those per-tile counts (scripts/kbench.py
// X6C_DUMP; weighted by each level's share of the step): 1.18 / 1.17 / 1.16 / 1.17 / 1.17 x, and fitted on levels
// 0-1 alone it gives the held-out levels 2-4 the same 1.17 -- it follows the scenes' axis-aligned planes, not the
// batch.  An offset's sums are the same k-steps in the same order whichever wave runs them: bit-identical.
template <int NW, int AC = 1, int PW = 1, int RS = 32, int ABL = 0, int DT = 0, int BR = 0, int DL = 0>
__global__ __launch_bounds__(64 * NW, 1) void wgrad_x6c_kernel(
    const float* __restrict__ x, int c_in, const float* __restrict__ dy, int c_out, int K,
    const int64_t* __restrict__ tile_start, const uint8_t* __restrict__ chunk_off,
    const uint32_t* __restrict__ chunk_lr, const int64_t* __restrict__ u_start, const int32_t* __restrict__ u_rows,
    int64_t n_rows, int64_t n_tiles, int n_ranges, float* __restrict__ slab) {
  constexpr int NTH = 64 * NW, NOW = 32 / NW;          // offsets per wave: o = wave + NW a, a < NOW (DL: the table)
  static_assert(!DL || NW == 8, "the offset deal table is for 8 waves");
  constexpr int XI = (kWCap * 8 + NTH - 1) / NTH;     // x staging items (row, 4 channels) per thread
  constexpr int DI = kWTile * 8 / NTH;                // dy staging items per thread
  constexpr int EI = (kWMaxCh * 16 + NTH - 1) / NTH;  // rule words per thread
  static_assert(DI * NTH == kWTile * 8, "dy staging items must divide evenly");
  // bf16 elements of one x piece image (+ zero row kWCap) and of one dy piece image (+ zero row 128)
  constexpr int kWXImg = (kWCap + 1) * RS, kWDImg = (kWTile + 1) * RS;
  __shared__ __attribute__((aligned(16))) uint16_t xim[3 * kWXImg];
  __shared__ __attribute__((aligned(16))) uint16_t dim[3 * kWDImg];
  __shared__ uint32_t ent[(kWMaxCh + 1) * 16];  // + one chunk: the partner read of a last odd chunk stays inside
  __shared__ uint8_t offs[kWMaxCh];
  __shared__ int otab[2][2][32];  // [buffer][first, end][offset]; DT 0: buffer 0 only
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, p4 = i16 & 3;
  const uint32_t deal = DL ? kX6cDeal[wave & 7] : 0u;
  auto off_of = [&](int a) { return DL ? (int)((deal >> (8 * a)) & 0xFFu) : wave + NW * a; };  // 0xFF >= K: none
  const int n_sl_o = c_out / 32, n_slices = (c_in / 32) * n_sl_o;
  const int64_t lb = xcd_linear(blockIdx.x, gridDim.x);
  const int slice = (int)(lb % n_slices);
  const int range = (int)(lb / n_slices);
  const int ci0 = 32 * (slice / n_sl_o), co0 = 32 * (slice % n_sl_o);
  int64_t t0 = (int64_t)range * n_tiles / n_ranges, t1 = (int64_t)(range + 1) * n_tiles / n_ranges;
  if constexpr (BR > 0) {
    if (n_tiles <= (int64_t)NTH * NTH) {  // block-uniform
      __shared__ int bcnt[2][2][NW];
      auto cost = [&](int64_t t) { return tile_start[t] + (int64_t)BR * t; };
      const int64_t c0 = cost(0), total = cost(n_tiles) - c0;
      const int64_t tg[2] = {c0 + (int64_t)range * total / n_ranges, c0 + (int64_t)(range + 1) * total / n_ranges};
      // bound(tg) = the first tile of cost >= tg (cost is increasing): round 0 counts the samples t = i st below
      // each target, round 1 the tiles of the interval that leaves
      const int64_t st = (n_tiles + NTH - 1) / NTH;
      int64_t base[2] = {0, 0};
#pragma unroll
      for (int rd = 0; rd < 2; ++rd) {
        int64_t c[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int64_t t = rd == 0 ? (int64_t)tid * st : base[k] + tid;
          const bool ok = rd == 0 ? t < n_tiles : (tid < st - 1 && t < n_tiles);
          c[k] = ok ? cost(t) : INT64_MAX;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int n = __popcll(ballot64(c[k] < tg[k]));
          if (lane == 0) bcnt[rd][k][wave] = n;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          int n = 0;
#pragma unroll
          for (int w = 0; w < NW; ++w) n += bcnt[rd][k][w];
          base[k] = rd == 0 ? (n > 0 ? (int64_t)(n - 1) * st + 1 : 0) : base[k] + n;
        }
      }
      t0 = base[0] < n_tiles ? base[0] : n_tiles;
      t1 = base[1] < n_tiles ? base[1] : n_tiles;
    }
  }

  floatx4 acc[NOW][2][2];
#pragma unroll
  for (int a = 0; a < NOW; ++a)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[a][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // zero rows (never overwritten) and the padding chunk of the rule words
  for (int i = tid; i < 3 * 32; i += NTH) {
    xim[(i / 32) * kWXImg + kWCap * RS + (i % 32)] = 0;
    dim[(i / 32) * kWDImg + kWTile * RS + (i % 32)] = 0;
  }
  if (tid < 16) ent[kWMaxCh * 16 + tid] = (uint32_t)kWCap | ((uint32_t)kWTile << 16);
  if (DT && tid < 128) otab[tid >> 6][(tid >> 5) & 1][tid & 31] = 0;
  if (DT) __syncthreads();

  // ---- staging registers: rows of tile t + 1 (loaded at the start of t), then its values and rule words
  int32_t srow[XI];
  floatx4 xv[XI], dv[DI];
  uint32_t ev[EI];
  int co_v = 255, co_p = 255, co_n = 255, s_nch = 0;
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
      if ((ABL & 2) && t != t0) break;
      const int u = (tid + NTH * b) & 7;
      xv[b] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (srow[b] >= 0) xv[b] = *reinterpret_cast<const floatx4*>(x + (int64_t)srow[b] * c_in + ci0 + 4 * u);
    }
#pragma unroll
    for (int b = 0; b < DI; ++b) {
      if ((ABL & 2) && t != t0) break;
      const int it = tid + NTH * b, u = it & 7;
      const int64_t row = t * kWTile + (it >> 3);
      dv[b] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (row < n_rows) dv[b] = *reinterpret_cast<const floatx4*>(dy + row * c_out + co0 + 4 * u);
    }
    const int64_t c0 = tile_start[t];
    s_nch = (int)(tile_start[t + 1] - c0);
#pragma unroll
    for (int b = 0; b < EI; ++b) {
      const int e = tid + NTH * b;
      ev[b] = e < s_nch * 16 ? chunk_lr[c0 * 16 + e] : 0u;
    }
    co_v = tid < s_nch ? chunk_off[c0 + tid] : 255;
    if (DT) {
      co_p = tid < s_nch && tid > 0 ? chunk_off[c0 + tid - 1] : 255;
      co_n = tid + 1 < s_nch ? chunk_off[c0 + tid + 1] : 255;
    }
  };
  int buf = 0;  // DT: the offset-table buffer of the staged tile
  bool first_store = true;
  auto store = [&]() {  // the staged tile into LDS (DT: one barrier; DT 0: two, the offset table through LDS)
    const bool images = !(ABL & 1) || first_store;
    first_store = false;
#pragma unroll
    for (int b = 0; b < XI; ++b) {
      if (images && srow[b] >= 0) {
        const int it = tid + NTH * b;
        uint2 pc[3];
        split4(xv[b], pc);
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          *reinterpret_cast<uint2*>(xim + pp * kWXImg + wimg_off_rs<RS>(it >> 3, it & 7)) = pc[pp];
      }
    }
#pragma unroll
    for (int b = 0; b < DI; ++b) {
      if (!images) break;
      const int it = tid + NTH * b;
      uint2 pc[3];
      split4(dv[b], pc);
#pragma unroll
      for (int pp = 0; pp < 3; ++pp)
        *reinterpret_cast<uint2*>(dim + pp * kWDImg + wimg_off_rs<RS>(it >> 3, it & 7)) = pc[pp];
    }
#pragma unroll
    for (int b = 0; b < EI; ++b) {
      const int e = tid + NTH * b;
      if (e < s_nch * 16) ent[e] = ev[b];
    }
    if constexpr (DT) {  // this tile's table into buffer buf, the other buffer (read by the last tile) zeroed
      if (tid < 64) otab[buf ^ 1][tid >> 5][tid & 31] = 0;
      if (tid < s_nch) {
        if (co_p != co_v) otab[buf][0][co_v] = tid;
        if (co_n != co_v) otab[buf][1][co_v] = tid + 1;
      }
      __syncthreads();
      return;
    }
    if (tid < s_nch) offs[tid] = (uint8_t)co_v;
    if (tid < 64) otab[0][tid >> 5][tid & 31] = 0;
    __syncthreads();
    if (tid < s_nch) {
      const int o = offs[tid];
      if (tid == 0 || offs[tid - 1] != o) otab[0][0][o] = tid;
      if (tid == s_nch - 1 || offs[tid + 1] != o) otab[0][1][o] = tid + 1;
    }
    __syncthreads();
  };

  // ---- one 32-rule step over the two chunks cA, cA + 1 (the second only if hasB): the B fragments (dy) of
  // both 16-column halves, then per 16-row half of x its A fragments and 12 MFMAs (36 fragment registers live)
  auto words_of = [&](int cA, uint32_t (&wd)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kp = 8 * g + 4 * h + qq, cs = kp >> 4;
      wd[h] = ent[(cA + cs) * 16 + (kp & 15)];
    }
  };
  auto rows_from = [&](const uint32_t (&wd)[2], bool hasB, int (&xr)[2], int (&dr)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kp = 8 * g + 4 * h + qq, cs = kp >> 4;
      uint32_t w = wd[h];
      if (cs == 1 && !hasB) w = (uint32_t)kWCap | ((uint32_t)kWTile << 16);
      const int ls = (int)(w & 0xFFFFu);
      xr[h] = ls < kWCap ? ls : kWCap;
      dr[h] = (int)(w >> 16);
    }
  };
  auto rows_of = [&](int cA, bool hasB, int (&xr)[2], int (&dr)[2]) {
    uint32_t wd[2];
    words_of(cA, wd);
    rows_from(wd, hasB, xr, dr);
  };
  auto frag = [&](const uint16_t* img, const int (&rr)[2], int v) {
    const uint2 lo = tr_read(img + wimg_off_rs<RS>(rr[0], v));
    const uint2 hi = tr_read(img + wimg_off_rs<RS>(rr[1], v));
    return u32x4{lo.x, lo.y, hi.x, hi.y};
  };
  uint32_t wcur[2] = {0u, 0u}, wnxt[2] = {0u, 0u};  // PW: this and the next k-step's rule words
  auto kstep = [&](int cA, bool hasB, floatx4 (&ac)[2][2]) {
    int xr[2], dr[2];
    if constexpr (PW) rows_from(wcur, hasB, xr, dr);
    else rows_of(cA, hasB, xr, dr);
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
        if constexpr (AC == 1) {
          floatx4& d = ac[sa][sb];
          d = mfma_bf16(fa[2], fb[sb][0], d);
          d = mfma_bf16(fa[1], fb[sb][1], d);
          d = mfma_bf16(fa[0], fb[sb][2], d);
          d = mfma_bf16(fa[1], fb[sb][0], d);
          d = mfma_bf16(fa[0], fb[sb][1], d);
          d = mfma_bf16(fa[0], fb[sb][0], d);
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
        const int o = off_of(a);
        first[a] = o < K ? __builtin_amdgcn_readfirstlane(otab[buf][0][o]) : 0;
        endc[a] = o < K ? __builtin_amdgcn_readfirstlane(otab[buf][1][o]) : 0;
        S[a + 1] = S[a] + (endc[a] - first[a] + 1) / 2;
      }
      const int n_st = S[NOW];
      const int s_vals = n_st / 2;  // the next tile's values go out half-way through (their rows have landed)
      int s = 0;
#pragma unroll
      for (int a = 0; a < NOW; ++a) {  // constant slot index: acc[a] stays in registers
        for (int c = first[a]; c < endc[a]; c += 2, ++s) {
          if (s == s_vals && more) issue_vals(t + 1);
          if constexpr (PW) {
            if (c == first[a]) {
              words_of(c, wcur);
            } else {
              wcur[0] = wnxt[0];
              wcur[1] = wnxt[1];
            }
            if (c + 2 < endc[a]) words_of(c + 2, wnxt);
          }
          kstep(c, c + 1 < endc[a], acc[a]);
        }
      }
      if (n_st == 0 && more) issue_vals(t + 1);
      __syncthreads();  // reads of tile t done
      if (DT) buf ^= 1;
      if (more) store();
    }
  }
  // partial dW of this range: slab[range][o][ci][co]
  float* sb = slab + (int64_t)range * K * c_in * c_out;
#pragma unroll
  for (int a = 0; a < NOW; ++a) {
    const int o = off_of(a);
    if (o >= K) continue;
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

inline int cu_count() { return device_cu_count(); }

}  // namespace msp

using namespace msp;

extern "C" {

size_t msp_tile_local_workspace_size(int64_t n, int tile_rows) {
  const int64_t n_tiles = ceil_div(n > 0 ? n : 1, tile_rows > 0 ? tile_rows : 1);
  return (size_t)(n_tiles + 1) * sizeof(int64_t) + scan_ws_bytes(n_tiles);
}

// From this many tiles on, the row grouping runs in its own one-wave-per-tile kernel (MODE 2 above); below, inside
// the fill (MODE 1).  scripts/build_bench.py, headline batch: L1 (4307 tiles) 284 vs 347 us, L2 (1140) 155 vs 164,
// L3 (277) 134 vs 109, L4 (66) 132 vs 108 (count + fill + one host read).
constexpr int64_t kGroupSplitTiles = 1024;

int msp_tile_local(const int32_t* nbr, int K, int64_t n, int tile_rows, int64_t* u_start, int32_t* u_rows,
                   int64_t u_cap, uint16_t* lidx, int32_t* perm, uint8_t* wave_off, void* ws, size_t ws_bytes,
                   msp_stream_t stream) {
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
    if (tile_rows == 64) local_count_kernel<64, 2048><<<grid, kLT, 0, s>>>(nbr, K, n, cnt);
    else if (tile_rows == 128) local_count_kernel<128, 4096><<<grid, kLT, 0, s>>>(nbr, K, n, cnt);
    else local_count_kernel<256, 8192><<<grid, kLT, 0, s>>>(nbr, K, n, cnt);
    const int rc = scan_exclusive_i64(cnt, u_start, n_tiles, u_start + n_tiles, sws, scan_ws_bytes(n_tiles), s,
                                      u_start + n_tiles + 1);
    if (rc) return rc;
  } else {
    MSP_REQUIRE(u_rows && (lidx == nullptr) == (perm == nullptr), "msp_tile_local: NULL output");
#define LF(T_, N2_)                                                                                              \
  if (lidx && n_tiles >= kGroupSplitTiles) {                                                                     \
    local_group_kernel<T_><<<(unsigned)ceil_div(n_tiles, 4), 256, 0, s>>>(nbr, K, n, n_tiles, perm, wave_off);   \
    local_fill_kernel<T_, N2_, 2><<<grid, kLT, 0, s>>>(nbr, K, n, n_pad, u_start, u_rows, lidx, perm, wave_off);  \
  } else if (lidx) {                                                                                             \
    local_fill_kernel<T_, N2_, 1><<<grid, kLT, 0, s>>>(nbr, K, n, n_pad, u_start, u_rows, lidx, perm, wave_off);  \
  } else {                                                                                                       \
    local_fill_kernel<T_, N2_, 0><<<grid, kLT, 0, s>>>(nbr, K, n, n_pad, u_start, u_rows, nullptr, nullptr,       \
                                                       nullptr);                                                \
  }
    if (tile_rows == 64) {
      LF(64, 2048)
    } else if (tile_rows == 128) {
      LF(128, 4096)
    } else {
      LF(256, 8192)
    }
#undef LF
  }
  return check_launch("msp_tile_local");
}

int msp_wgrad_chunk_ok(int64_t n_rows, int K, int c_in, int c_out) {
  return (n_rows > 0 && K >= 1 && K <= 27 && c_in % 32 == 0 && c_out % 32 == 0) ? 1 : 0;
}

// Measured against the pair lists on the headline batch's rulebooks (scripts/kbench.py, profiles/r03/kbench_r03*.log):
// ahead for 64+ output channels at every level (level 1 64 -> 64 0.53 vs 0.58 ms, level 4 160 -> 160 0.082 vs
// 0.107, level 5 192 -> 192 0.041 vs 0.052, level 6 224 -> 224 0.027 vs 0.036).  Level 0's 32 -> 32 is ahead too
// in isolation since the products accumulate straight into the tile sums (0.327 vs 0.347 ms,
// profiles/r03/kbench_r03y_level0.log) but needs level 0's tile-local rulebook (see msp_conv_local_preferred):
// 32 output channels stay on the pair lists.
#ifndef MSP_CHUNK_NARROW  // 1: c_out = 32 too (level 0's 32 x 32 and, since round 5's 72-byte image rows, the
#define MSP_CHUNK_NARROW 1  // decoder's 64 x 32: 0.490 vs 0.517 ms on the pair lists, profiles/r05/kbench_r05p_*)
#endif
int msp_wgrad_chunk_preferred(int64_t n_rows, int K, int c_in, int c_out) {
  return msp_wgrad_chunk_ok(n_rows, K, c_in, c_out) && (c_out >= 64 || (MSP_CHUNK_NARROW && c_out == 32)) ? 1
                                                                                                             : 0;
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
                          int64_t* n_far, msp_stream_t stream) {
  MSP_REQUIRE(n_rows >= 0 && n_rows < (1ll << 31), "msp_wgrad_chunk_index: bad row count");
  hipStream_t s = as_stream(stream);
  if (n_far) MSP_HIP(hipMemsetAsync(n_far, 0, sizeof(int64_t), s), "msp_wgrad_chunk_index");
  const int64_t n_tiles = ceil_div(n_rows, kWTile);
  if (n_tiles == 0) return MSP_OK;
  MSP_REQUIRE(tile_start && chunk_src && chunk_row && u_start && u_rows && chunk_lr,
              "msp_wgrad_chunk_index: NULL pointer");
  chunk_lidx_kernel<<<(unsigned)n_tiles, kLT, 0, s>>>(tile_start, chunk_src, chunk_row, u_start, u_rows, chunk_lr,
                                                      reinterpret_cast<unsigned long long*>(n_far));
  return check_launch("msp_wgrad_chunk_index");
}

size_t msp_wgrad_far_workspace_size(int64_t n_far) {
  const int64_t n = n_far > 0 ? n_far : 0;
  return 8 + (size_t)n * 8 + (size_t)((n * 4 + 7) / 8) * 8 + msp_sort_workspace_size(n, kFarShift + 5);
}

int msp_local_chunk_index(const uint16_t* lidx, const int32_t* perm, int K, int64_t n, int64_t* tile_start,
                          uint8_t* chunk_off, uint32_t* chunk_lr, int64_t chunk_cap, void* ws, size_t ws_bytes,
                          msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= kKMax && n >= 0 && n < (1ll << 31), "msp_local_chunk_index: K must be in [1, %d]",
              kKMax);
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n, kWTile), n_pad = n_tiles * kWTile;
  const size_t need = msp_tile_local_workspace_size(n, kWTile);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_local_chunk_index: workspace too small (%zu < %zu)", ws_bytes, need);
  if (n_tiles == 0) {
    if (chunk_cap <= 0) MSP_HIP(hipMemsetAsync(tile_start, 0, 2 * sizeof(int64_t), s), "msp_local_chunk_index");
    return MSP_OK;
  }
  int64_t* cnt = reinterpret_cast<int64_t*>(ws);
  void* sws = cnt + n_tiles + 1;
  if (chunk_cap <= 0) {  // counting call: tile_start[0..n_tiles] = exclusive scan, tile_start[n_tiles + 1] = largest
    lchunk_count_kernel<<<(unsigned)n_tiles, kLT, 0, s>>>(lidx, K, n_pad, cnt);
    const int rc = scan_exclusive_i64(cnt, tile_start, n_tiles, tile_start + n_tiles, sws, scan_ws_bytes(n_tiles), s,
                                      tile_start + n_tiles + 1);
    if (rc) return rc;
  } else {
    MSP_REQUIRE(perm && chunk_off && chunk_lr, "msp_local_chunk_index: NULL output");
    lchunk_fill_kernel<<<(unsigned)n_tiles, kLT, 0, s>>>(lidx, perm, K, n_pad, tile_start, chunk_off, chunk_lr);
  }
  return check_launch("msp_local_chunk_index");
}

int msp_wgrad_far_list(const int64_t* tile_start, const uint8_t* chunk_off, const uint32_t* chunk_lr,
                       int64_t n_rows, int64_t n_far, int64_t* far_key, int32_t* far_tile, void* ws,
                       size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(n_rows >= 0 && n_rows < (1ll << 31) && n_far >= 0 && n_far < (1ll << 31),
              "msp_wgrad_far_list: bad sizes (n_rows=%lld n_far=%lld)", (long long)n_rows, (long long)n_far);
  if (n_far == 0) return MSP_OK;
  MSP_REQUIRE(tile_start && chunk_off && chunk_lr && far_key && far_tile, "msp_wgrad_far_list: NULL pointer");
  const size_t need = msp_wgrad_far_workspace_size(n_far);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_wgrad_far_list: workspace too small (%zu < %zu)", ws_bytes, need);
  hipStream_t s = as_stream(stream);
  char* w = static_cast<char*>(ws);
  auto* ctr = reinterpret_cast<unsigned long long*>(w);
  auto* keys = reinterpret_cast<uint64_t*>(w + 8);
  auto* tiles = reinterpret_cast<int32_t*>(w + 8 + n_far * 8);
  void* sws = w + 8 + n_far * 8 + ((n_far * 4 + 7) / 8) * 8;
  MSP_HIP(hipMemsetAsync(ctr, 0, 8, s), "msp_wgrad_far_list");
  const int64_t n_tiles = ceil_div(n_rows, kWTile);
  far_collect_kernel<<<(unsigned)n_tiles, kLT, 0, s>>>(tile_start, chunk_off, chunk_lr, n_far, ctr, keys, tiles);
  const int rc = check_launch("msp_wgrad_far_list");
  if (rc != MSP_OK) return rc;
  return msp_sort_pairs(keys, reinterpret_cast<uint64_t*>(far_key), tiles, far_tile, n_far, kFarShift + 5, sws,
                        msp_sort_workspace_size(n_far, kFarShift + 5), stream);
}

int msp_conv_wgrad_far(const float* x, int c_in, const float* dy, int c_out, int K, const int32_t* chunk_src,
                       const uint16_t* chunk_row, const int64_t* far_key, const int32_t* far_tile, int64_t n_far,
                       float* dw, msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= 32 && c_in > 0 && c_in % 32 == 0 && c_out > 0 && c_out % 32 == 0 && n_far >= 0,
              "msp_conv_wgrad_far: needs K <= 32 and channels in multiples of 32 (K=%d c_in=%d c_out=%d)", K, c_in,
              c_out);
  if (n_far == 0) return MSP_OK;
  MSP_REQUIRE(x && dy && chunk_src && chunk_row && far_key && far_tile && dw, "msp_conv_wgrad_far: NULL pointer");
  MSP_REQUIRE(((uintptr_t)dy & 15) == 0 && ((uintptr_t)dw & 15) == 0,
              "msp_conv_wgrad_far: dy and dw must be 16-byte aligned (float4 rows)");
  hipStream_t s = as_stream(stream);
  const unsigned grid = (unsigned)(K * (c_in / 32) * (c_out / 32));
  wgrad_far_kernel<<<grid, 256, 0, s>>>(x, c_in, dy, c_out, chunk_src, chunk_row,
                                        reinterpret_cast<const uint64_t*>(far_key), far_tile, n_far, dw);
  return check_launch("msp_conv_wgrad_far");
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
  // 72-byte image rows (RS = 36): 9-15 % faster than the swizzled 64-byte rows at every level
  // (profiles/r05/kbexp_r05m_x6c_row_stride.log)
  // the offset deal table was fitted to the 27 offsets of a 3^3 submanifold filter; other maps deal round-robin
  if (K == 27)
    wgrad_x6c_kernel<8, 1, 1, MSP_X6C_RS, 0, 1, 128, 1><<<(unsigned)(n_ranges * slices), 512, 0, s>>>(
        x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr, u_start, u_rows, n_rows, n_tiles, (int)n_ranges,
        slab);
  else
    wgrad_x6c_kernel<8, 1, 1, MSP_X6C_RS, 0, 1, 128, 0><<<(unsigned)(n_ranges * slices), 512, 0, s>>>(
        x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr, u_start, u_rows, n_rows, n_tiles, (int)n_ranges,
        slab);
  const int64_t n4 = (int64_t)K * c_in * c_out / 4;
  wgrad_ranges_reduce_kernel<<<(unsigned)ceil_div(n4, 16), 256, 0, s>>>(reinterpret_cast<const floatx4*>(slab),
                                                                         (int)n_ranges, n4,
                                                                         reinterpret_cast<floatx4*>(dw));
  return check_launch("msp_conv_wgrad_chunk");
}

// The image a convolution entry point splits its weights into for one call (msp_weight_image, the header).
int msp_conv_weight_image(int entry, int64_t n_rows, int K, int c_in, int c_out, int flip, msp_weight_image* d) {
  MSP_REQUIRE(d && K >= 1 && c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_weight_image: bad shape (K=%d c_in=%d c_out=%d)", K, c_in, c_out);
  d->K = K;
  d->c_in = c_in;
  d->c_out = c_out;
  d->wlay = (flip >> 1) & 1;
  const int nks = (c_in + 31) / 32;
  if (entry == 1) {  // msp_conv_local: lane-ordered image
    d->kind = 2;
    d->p = local_nt(c_out);
    d->units = (int64_t)K * (c_out / (16 * d->p)) * nks * d->p * 64;
    d->bytes = (int64_t)msp_conv_local_workspace_size(K, c_in, c_out);
    return MSP_OK;
  }
  d->kind = 1;
  d->units = (int64_t)K * c_out * nks * 12;
  if (entry == 0) {  // msp_conv_tile, 128-row tiles
    if (msp_conv_tile_form(n_rows, c_in, c_out, 128) == 1) {  // per-wave tiles (launch_x6r's NT)
      d->p = 16 * (c_out / 16 >= 2 && (c_out / 16) % 2 == 0 ? 2 : 1);
    } else {
      d->p = 16 * plan_x6(n_rows, c_out).nt;
    }
    d->bytes = (int64_t)msp_conv_tile_workspace_size(n_rows, K, c_in, c_out, 128);
    return MSP_OK;
  }
  if (entry == 2) {  // msp_conv_nbr
    const int n16 = c_out / 16;
    d->p = 16 * (n16 % 4 == 0 ? 4 : (n16 % 3 == 0 ? 3 : (n16 % 2 == 0 ? 2 : 1)));
    d->bytes = (int64_t)msp_conv_nbr_workspace_size(K, c_in, c_out);
    return MSP_OK;
  }
  set_error("msp_conv_weight_image: entry must be 0 (tile), 1 (local) or 2 (nbr), got %d", entry);
  return MSP_EINVAL;
}

int msp_split_weight_images(const msp_weight_image* descs, int n, const int64_t* unit_start, int64_t total_units,
                            msp_stream_t stream) {
  MSP_REQUIRE(n >= 0 && total_units >= 0, "msp_split_weight_images: n=%d total=%lld", n, (long long)total_units);
  if (n == 0 || total_units == 0) return MSP_OK;
  MSP_REQUIRE(descs && unit_start, "msp_split_weight_images: null pointer");
  split_images_kernel<<<(unsigned)ceil_div(total_units, 256), 256, 0, as_stream(stream)>>>(descs, n, unit_start,
                                                                                             total_units);
  return check_launch("msp_split_weight_images");
}

// Measured against the gather forms on the headline batch's rulebooks (profiles/r02/kbench_local_r02_levels.log):
// ahead from 64 channels on both sides and 4096 rows up (levels 1-4 of m = 32: 0-34 % less time), behind on the
// 32-channel level 0 and on the few-tile levels 5-6 (grids of 16 / 4 tiles).
// From 64 channels on both sides and 4096 rows; from 1024 rows when the output is at least twice the input (level
// 5's backward-data 192 -> 384: 0.063 vs 0.086 ms on the shared tiles, profiles/r03/kbench_r03_split.log).  Level
// 0's 32 -> 64 backward-data is faster here in isolation (0.685 vs 0.711 ms, profiles/r03/kbench_r03y_level0.log),
// but it needs level 0's tile-local rulebook, whose side-stream build cost more than that: 57.1 vs 56.7 ms/step
// with MSP_LOCAL_MIN_CIN 32 and MSP_CHUNK_NARROW 1 (profiles/r03/ab_r03_level0_local.log).
#ifndef MSP_LOCAL_MIN_CIN  // experiments build: -DMSP_LOCAL_MIN_CIN=32 takes level 0's 32 -> 64
#define MSP_LOCAL_MIN_CIN 64
#endif
int msp_conv_local_preferred(int64_t n_rows, int c_in, int c_out) {
  return (c_in % 16 == 0 && c_out % 16 == 0 && c_in >= MSP_LOCAL_MIN_CIN && c_out >= 64 &&
          (n_rows >= 4096 || (n_rows >= 1024 && c_out >= 2 * c_in))) ? 1 : 0;
}

size_t msp_conv_local_workspace_size(int K, int c_in, int c_out) {
  return (size_t)K * c_out * ((c_in + 31) / 32) * 32 * 6;
}

int msp_conv_local(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                   const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows, const int32_t* perm,
                   const uint8_t* wave_off, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                   msp_stream_t stream) {
  return msp_conv_local_bn(x, c_in, wt, K, flip, c_out, tile_rows, lidx, u_start, u_rows, perm, wave_off, n_rows,
                           out, ws, ws_bytes, nullptr, stream);
}

int msp_conv_local_bn(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                      const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows, const int32_t* perm,
                      const uint8_t* wave_off, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                      const msp_bn_epilogue* epi, msp_stream_t stream) {
  MSP_REQUIRE(epi == nullptr || epi->partial != nullptr, "msp_conv_local_bn: epilogue without a partial buffer");
  MSP_REQUIRE(epi == nullptr || epi->x == nullptr || epi->stats != nullptr,
              "msp_conv_local_bn: backward epilogue needs the BatchNorm's stats");
  MSP_REQUIRE(c_in > 0 && c_in % 16 == 0 && c_out > 0 && c_out % 16 == 0,
              "msp_conv_local: channels must be positive multiples of 16 (c_in=%d c_out=%d)", c_in, c_out);
  MSP_REQUIRE(K >= 1 && K <= kKMax, "msp_conv_local: K must be in [1, %d] (got %d)", kKMax, K);
  MSP_REQUIRE(tile_rows == 128, "msp_conv_local: tile_rows must be 128 (got %d)", tile_rows);
  MSP_REQUIRE(flip >= 0 && flip <= 7, "msp_conv_local: flip must be 0..7 (got %d)", flip);
  const size_t need = msp_conv_local_workspace_size(K, c_in, c_out);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_conv_local: workspace too small (%zu < %zu)", ws_bytes, need);
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  const int NT = local_nt(c_out);
  const int n_y = c_out / (16 * NT), nks = (c_in + 31) / 32;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t lanes = (int64_t)K * n_y * nks * NT * 64;
  if (!(flip & 4))  // bit 2: ws already holds this image (msp_split_weight_images)
    split_weights_lane_kernel<<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                             (flip >> 1) & 1);
  const int64_t n_pad = n_tiles * tile_rows;
  const unsigned grid = (unsigned)(n_tiles * n_y);
  const BnEpi be = bn_epi_of(epi, c_out, n_rows);
#define X6S(N, E)                                                                                                \
  conv_x6s_kernel<N, 0, 1, 1, E><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start, u_rows, perm, \
                                                     wave_off, n_pad, n_y, out, be)
  if (NT == 2) {
    if (epi) X6S(2, true);
    else X6S(2, false);
  } else {
    if (epi) X6S(1, true);
    else X6S(1, false);
  }
#undef X6S
  return check_launch("msp_conv_local");
}

#ifdef MSP_EXPERIMENTS
// Kernel-variant entry for scripts/kbench.py (built only into lib/libmi3dsparse_exp.so by
// scripts/build_exp.sh; the product library has no such symbol): msp_conv_local with the conv_x6s
// template form selected by `variant` = 1000 (WB - 1) + 100 AB + 10 AC + RR (RR = 1: offsets dealt round-robin,
// wave_off ignored).
int msp_exp_conv_local(int variant, const float* x, int c_in, const float* wt, int K, int flip, int c_out,
                       int tile_rows, const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows,
                       const int32_t* perm, const uint8_t* wave_off, int64_t n_rows, float* out, void* ws,
                       size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(tile_rows == 128 && c_out % 32 == 0 && c_in % 16 == 0, "msp_exp_conv_local: shape");
  const int64_t n_tiles = ceil_div(n_rows, tile_rows);
  if (n_tiles == 0) return MSP_OK;
  MSP_REQUIRE(ws && ws_bytes >= msp_conv_local_workspace_size(K, c_in, c_out), "msp_exp_conv_local: ws");
  hipStream_t s = as_stream(stream);
  const int NT = 2, n_y = c_out / 32, nks = (c_in + 31) / 32;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t lanes = (int64_t)K * n_y * nks * NT * 64;
  split_weights_lane_kernel<<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(wt, K, c_out, c_in, NT, img,
                                                                           (flip >> 1) & 1);
  const unsigned grid = (unsigned)(n_tiles * n_y);
  const int64_t n_pad = n_tiles * tile_rows;
  const uint8_t* wo = variant % 10 == 1 ? nullptr : wave_off;
  const int wbv = variant / 1000 + 1;
  variant %= 1000;
#define EV(A, C, W)                                                                                            \
  if (wbv == W && variant / 100 == A && (variant / 10) % 10 == C) {                                            \
    conv_x6s_kernel<2, A, C, W><<<grid, 512, 0, s>>>(x, c_in, img, K, flip & 1, c_out, lidx, u_start, u_rows,  \
                                                     perm, wo, n_pad, n_y, out, BnEpi{});                      \
    return check_launch("msp_exp_conv_local");                                                                 \
  }
  EV(0, 0, 1) EV(0, 1, 1) EV(1, 0, 1) EV(1, 1, 1) EV(4, 0, 1) EV(5, 0, 1) EV(8, 1, 1) EV(0, 1, 2)
#undef EV

  set_error("msp_exp_conv_local: no variant %d", variant);
  return MSP_EINVAL;
}

// msp_conv_wgrad_chunk with the wgrad_x6c template form selected by `variant` = AC (0 or 1).
int msp_exp_wgrad_chunk(int variant, const float* x, int c_in, const float* dy, int c_out, int K, int tile_rows,
                        const int64_t* tile_start, const uint8_t* chunk_off, const uint32_t* chunk_lr,
                        const int64_t* u_start, const int32_t* u_rows, int64_t n_rows, int64_t n_ranges,
                        float* slab, float* dw, msp_stream_t stream) {
  MSP_REQUIRE(msp_wgrad_chunk_ok(n_rows, K, c_in, c_out) && tile_rows == kWTile && n_ranges >= 1,
              "msp_exp_wgrad_chunk: shape");
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n_rows, kWTile);
  const int64_t slices = (int64_t)(c_in / 32) * (c_out / 32);
  const unsigned grid = (unsigned)(n_ranges * slices);
  if (variant == 0)
    wgrad_x6c_kernel<8, 0, 0><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr, u_start,
                                                u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 1)
    wgrad_x6c_kernel<8, 1, 0><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr, u_start,
                                                u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 3)
    wgrad_x6c_kernel<8, 1, 1><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr, u_start,
                                                   u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 43)  // the product form with 72-byte image rows (RS = 36)
    wgrad_x6c_kernel<8, 1, 1, 36><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr,
                                                       u_start, u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 143)  // ablation: no image staging after the first tile
    wgrad_x6c_kernel<8, 1, 1, 36, 1><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr,
                                                          u_start, u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 343)  // ablation: no image staging and no value loads after the first tile
    wgrad_x6c_kernel<8, 1, 1, 36, 3><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr,
                                                          u_start, u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 2043)  // the round-6 product: direct offset table (DT)
    wgrad_x6c_kernel<8, 1, 1, 36, 0, 1><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off, chunk_lr,
                                                             u_start, u_rows, n_rows, n_tiles, (int)n_ranges, slab);
  else if (variant == 32043)  // + ranges of equal cost, 32 chunks per tile of staging
    wgrad_x6c_kernel<8, 1, 1, 36, 0, 1, 32><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off,
                                                                 chunk_lr, u_start, u_rows, n_rows, n_tiles,
                                                                 (int)n_ranges, slab);
  else if (variant == 64043)  // + ranges of equal cost, 64 chunks per tile of staging
    wgrad_x6c_kernel<8, 1, 1, 36, 0, 1, 64><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off,
                                                                 chunk_lr, u_start, u_rows, n_rows, n_tiles,
                                                                 (int)n_ranges, slab);
  else if (variant == 1128043)  // the round-6 product: + the offset deal table
    wgrad_x6c_kernel<8, 1, 1, 36, 0, 1, 128, 1><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off,
                                                                     chunk_lr, u_start, u_rows, n_rows, n_tiles,
                                                                     (int)n_ranges, slab);
  else if (variant == 128043)  // + ranges of equal cost, 128 chunks per tile of staging
    wgrad_x6c_kernel<8, 1, 1, 36, 0, 1, 128><<<grid, 512, 0, s>>>(x, c_in, dy, c_out, K, tile_start, chunk_off,
                                                                  chunk_lr, u_start, u_rows, n_rows, n_tiles,
                                                                  (int)n_ranges, slab);
  else {
    set_error("msp_exp_wgrad_chunk: no variant %d", variant);
    return MSP_EINVAL;
  }
  const int64_t n4 = (int64_t)K * c_in * c_out / 4;
  wgrad_ranges_reduce_kernel<<<(unsigned)ceil_div(n4, 16), 256, 0, s>>>(reinterpret_cast<const floatx4*>(slab),
                                                                         (int)n_ranges, n4,
                                                                         reinterpret_cast<floatx4*>(dw));
  return check_launch("msp_exp_wgrad_chunk");
}
#endif

}  // extern "C"
