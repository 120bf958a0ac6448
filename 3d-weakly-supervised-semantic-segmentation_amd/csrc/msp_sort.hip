// Stable LSD radix sort of (uint64 key, int32 value) pairs on key bits [0, end_bit): the voxel dedup of the
// InputLayer (point keys -> sorted keys -> segments, msp_meta.hip), the row order of the dense row-group
// convolution (msp_dense_order) and the deterministic index_add_ (msp_tail.hip).  Written for gfx950 instead of
// a library sort so that no third-party kernel runs in the step.
//
// 8-bit digits, one pass per digit.  Tiles of kTile = 4096 pairs (256 threads x 16 rounds of one pair per thread,
// each round 256 consecutive pairs).  Per pass:
//   radix_hist_kernel     per-tile digit counts (LDS integer atomics), written digit-major: counts[d][tile];
//   scan_exclusive_i64    over the counts -> for every (digit, tile) the first output position;
//   radix_scatter_kernel  per round, each wave ranks its 64 pairs among the lanes with the same digit by a
//                         wavefront ballot per digit bit (peers = AND of matching ballots, rank = popcount of the
//                         peers below the lane), the waves' digit counts meet in LDS in wave order, and every pair
//                         goes to (tile's digit start + pairs of that digit in earlier rounds + earlier waves +
//                         rank): stable, deterministic, no atomics on the output.
// Keys and values ping-pong between the output and a workspace copy so that the last pass writes the output.
#include "msp_common.h"

namespace msp {

constexpr int kSortT = 256;
constexpr int kSortRounds = 16;
constexpr int kSortTile = kSortT * kSortRounds;
constexpr int kRadix = 256;

__global__ __launch_bounds__(kSortT) void radix_hist_kernel(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                            int bits, int64_t n_tiles, int64_t* __restrict__ counts) {
  __shared__ int h[kRadix];
  const int t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile + t;
  const uint64_t mask = (1ull << bits) - 1;
  uint64_t k[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t i = base + (int64_t)r * kSortT;
    k[r] = i < n ? keys[i] : 0;
  }
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r)
    if (base + (int64_t)r * kSortT < n) atomicAdd(&h[(int)((k[r] >> shift) & mask)], 1);
  __syncthreads();
  counts[(int64_t)t * n_tiles + blockIdx.x] = h[t];
}

__global__ __launch_bounds__(kSortT) void radix_scatter_kernel(const uint64_t* __restrict__ kin,
                                                               const int32_t* __restrict__ vin,
                                                               uint64_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                               int64_t n, int shift, int bits, int64_t n_tiles,
                                                               const int64_t* __restrict__ offs) {
  __shared__ int64_t base_s[kRadix];
  __shared__ int cnt_s[kSortT / 64][kRadix];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  base_s[t] = offs[(int64_t)t * n_tiles + blockIdx.x];
#pragma unroll
  for (int w = 0; w < kSortT / 64; ++w) cnt_s[w][t] = 0;
  const uint64_t mask = (1ull << bits) - 1;
  const int64_t tile0 = (int64_t)blockIdx.x * kSortTile + t;
  uint64_t k[kSortRounds];
  int32_t v[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t i = tile0 + (int64_t)r * kSortT;
    k[r] = i < n ? kin[i] : 0;
    v[r] = i < n ? vin[i] : 0;
  }
  const unsigned long long below = (1ull << lane) - 1;
  __syncthreads();
#pragma unroll 1
  for (int r = 0; r < kSortRounds; ++r) {
    const bool live = tile0 + (int64_t)r * kSortT < n;
    const int d = (int)((k[r] >> shift) & mask);
    unsigned long long peers = ballot64(live);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (d >> b) & 1;
      const unsigned long long m = ballot64(bit);
      peers &= bit ? m : ~m;
    }
    const int rank = __popcll(peers & below);
    if (live && rank == 0) cnt_s[wave][d] = __popcll(peers);
    __syncthreads();
    if (live) {
      int64_t pos = base_s[d] + rank;
      for (int w = 0; w < wave; ++w) pos += cnt_s[w][d];
      kout[pos] = k[r];
      vout[pos] = v[r];
    }
    __syncthreads();
    int add = 0;
#pragma unroll
    for (int w = 0; w < kSortT / 64; ++w) {
      add += cnt_s[w][t];
      cnt_s[w][t] = 0;
    }
    base_s[t] += add;
    __syncthreads();
  }
}

inline size_t al256s(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace msp

using namespace msp;

extern "C" {

size_t msp_sort_workspace_size(int64_t n, int end_bit) {
  (void)end_bit;
  if (n <= 0) return 256;
  const int64_t n_tiles = ceil_div(n, kSortTile);
  const int64_t m = (int64_t)kRadix * n_tiles;
  return al256s((size_t)n * 8) + al256s((size_t)n * 4) + 2 * al256s((size_t)m * 8) + al256s(8) +
         al256s(scan_ws_bytes(m));
}

int msp_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in, int32_t* vals_out,
                   int64_t n, int end_bit, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(end_bit > 0 && end_bit <= 64, "msp_sort_pairs: bad end_bit %d", end_bit);
  MSP_REQUIRE(n >= 0 && n < (1ll << 31), "msp_sort_pairs: bad n %lld", (long long)n);
  if (n == 0) return MSP_OK;
  const size_t need = msp_sort_workspace_size(n, end_bit);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_sort_pairs: workspace too small (%zu < %zu)", ws_bytes, need);
  MSP_REQUIRE(keys_out != keys_in && vals_out != vals_in, "msp_sort_pairs: outputs must not alias the inputs");
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n, kSortTile);
  const int64_t m = (int64_t)kRadix * n_tiles;
  char* w = static_cast<char*>(ws);
  uint64_t* kt = reinterpret_cast<uint64_t*>(w);
  w += al256s((size_t)n * 8);
  int32_t* vt = reinterpret_cast<int32_t*>(w);
  w += al256s((size_t)n * 4);
  int64_t* counts = reinterpret_cast<int64_t*>(w);
  w += al256s((size_t)m * 8);
  int64_t* offs = reinterpret_cast<int64_t*>(w);
  w += al256s((size_t)m * 8);
  int64_t* total = reinterpret_cast<int64_t*>(w);
  w += al256s(8);
  void* sws = w;
  const int passes = (end_bit + 7) / 8;
  const uint64_t* ksrc = keys_in;
  const int32_t* vsrc = vals_in;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p, bits = end_bit - shift < 8 ? end_bit - shift : 8;
    const bool to_out = ((passes - 1 - p) & 1) == 0;  // the last pass writes the output
    uint64_t* kdst = to_out ? keys_out : kt;
    int32_t* vdst = to_out ? vals_out : vt;
    radix_hist_kernel<<<(unsigned)n_tiles, kSortT, 0, s>>>(ksrc, n, shift, bits, n_tiles, counts);
    const int rc = scan_exclusive_i64(counts, offs, m, total, sws, scan_ws_bytes(m), s);
    if (rc) return rc;
    radix_scatter_kernel<<<(unsigned)n_tiles, kSortT, 0, s>>>(ksrc, vsrc, kdst, vdst, n, shift, bits, n_tiles, offs);
    ksrc = kdst;
    vsrc = vdst;
  }
  return check_launch("msp_sort_pairs");
}

}  // extern "C"
