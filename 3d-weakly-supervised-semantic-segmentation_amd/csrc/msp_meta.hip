// Metadata on the device: voxel keys, dedup, hash grid, submanifold neighbour
// maps, strided child maps and the two rulebook forms the convolutions use.
//
// What this replaces: SparseConvNet builds the same structures on the HOST
// (per-sample hash maps + OpenMP) inside `scn.InputLayer` and lazily in the
// first convolution of each spatial size, then copies the rules to the device
// per call.  Here everything stays in HBM.
#include "msp_common.h"

namespace msp {

constexpr int kThreads = 256;

// ---------------------------------------------------------------- keys
__global__ __launch_bounds__(kThreads) void point_keys_kernel(const int64_t* __restrict__ coords, int64_t n,
                                                              int64_t stride, int log2s, int64_t size,
                                                              uint64_t* __restrict__ keys,
                                                              int32_t* __restrict__ vals,
                                                              int64_t* __restrict__ stats) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  bool bad = false;
  int64_t b = 0;
  if (i < n) {
    const int64_t* c = coords + i * stride;
    const int64_t x = c[0], y = c[1], z = c[2];
    b = c[3];
    bad = x < 0 || y < 0 || z < 0 || x >= size || y >= size || z >= size || b < 0;
    keys[i] = bad ? kEmptyKey : make_key(b, x, y, z, log2s);
    vals[i] = (int32_t)i;
  }
  // batch column non-decreasing along the points? (the fused encoder tail
  // relies on scene b being the point range of batch id b)
  const bool desc = i > 0 && i < n && b < coords[(i - 1) * stride + 3];
  // wave reductions, then one pair of atomics per block (per-wave atomics on
  // two addresses serialised the kernel at ~25k waves)
  __shared__ int64_t red_bad[kThreads / 64], red_max[kThreads / 64], red_desc[kThreads / 64];
  const unsigned long long badm = ballot64(bad);
  const unsigned long long descm = ballot64(desc);
  int64_t bmax = (i < n && !bad) ? b : 0;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) bmax = max(bmax, (int64_t)__shfl_xor(bmax, d, 64));
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red_bad[wave] = __popcll(badm);
    red_max[wave] = bmax;
    red_desc[wave] = __popcll(descm);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t nb = 0, mx = 0, nd = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
      nb += red_bad[w];
      mx = max(mx, red_max[w]);
      nd += red_desc[w];
    }
    if (nb) atomicAdd((unsigned long long*)&stats[0], (unsigned long long)nb);
    if (mx) atomicMax((unsigned long long*)&stats[1], (unsigned long long)mx);
    if (nd) atomicAdd((unsigned long long*)&stats[2], (unsigned long long)nd);
  }
}

// starts[b] = first row whose batch id is >= b (lower bound over a non-decreasing
// batch column), b = 0..n_batch; one thread per entry, a binary search each.
__global__ __launch_bounds__(kThreads) void batch_starts_kernel(const int64_t* __restrict__ coords, int64_t n,
                                                                int64_t stride, int64_t n_batch,
                                                                int64_t* __restrict__ starts) {
  const int64_t b = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (b > n_batch) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (coords[mid * stride + 3] < b) lo = mid + 1;
    else hi = mid;
  }
  starts[b] = lo;
}

// ---------------------------------------------------------------- segment
constexpr int kSegItems = 8;
constexpr int kSegTile = kThreads * kSegItems;

__device__ inline bool seg_flag(const uint64_t* k, int64_t i, int shift) {
  return i == 0 || (k[i] >> shift) != (k[i - 1] >> shift);
}

__global__ __launch_bounds__(kThreads) void seg_count_kernel(const uint64_t* __restrict__ k, int64_t n,
                                                             int shift, int64_t* __restrict__ block_sums) {
  const int64_t base = (int64_t)blockIdx.x * kSegTile + (int64_t)threadIdx.x * kSegItems;
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < kSegItems; ++j) {
    const int64_t i = base + j;
    if (i < n) c += seg_flag(k, i, shift);
  }
  int64_t tot;
  block_excl_scan<kThreads>(c, &tot);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kThreads) void seg_apply_kernel(
    const uint64_t* __restrict__ k, int64_t n, int shift, const int64_t* __restrict__ block_off,
    const int32_t* __restrict__ perm, int32_t* __restrict__ seg_of, int32_t* __restrict__ p2v,
    uint64_t* __restrict__ uniq, int32_t* __restrict__ seg_start) {
  const int64_t base = (int64_t)blockIdx.x * kSegTile + (int64_t)threadIdx.x * kSegItems;
  bool f[kSegItems];
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < kSegItems; ++j) {
    const int64_t i = base + j;
    f[j] = (i < n) && seg_flag(k, i, shift);
    c += f[j];
  }
  int64_t tot;
  int64_t g = block_excl_scan<kThreads>(c, &tot) + block_off[blockIdx.x] - 1;  // group of the previous row
#pragma unroll
  for (int j = 0; j < kSegItems; ++j) {
    const int64_t i = base + j;
    if (i >= n) break;
    if (f[j]) {
      ++g;
      uniq[g] = k[i] >> shift;
      seg_start[g] = (int32_t)i;
    }
    seg_of[i] = (int32_t)g;
    if (p2v) p2v[perm[i]] = (int32_t)g;
    if (i == n - 1) seg_start[g + 1] = (int32_t)n;
  }
}

// ---------------------------------------------------------------- hash grid
// Byte fill with 16-byte stores over a grid sized to the chip (hipMemsetAsync's fill of a 64 MB table or a
// 17 MB map ran at ~0.8 TB/s on the side stream, profiles/r05/prof_r05final).
__global__ __launch_bounds__(kThreads) void fill16_kernel(uint4* __restrict__ p, int64_t n16, uint4 v) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n16; i += (int64_t)gridDim.x * kThreads) p[i] = v;
}

static int fill_bytes(void* p, uint8_t value, size_t bytes, hipStream_t s, const char* what) {
  if (bytes == 0) return MSP_OK;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0 && (bytes & 15) == 0) {
    const uint32_t w = 0x01010101u * value;
    const int64_t n16 = (int64_t)(bytes / 16);
    const int64_t blocks = ceil_div(n16, kThreads);
    fill16_kernel<<<(unsigned)(blocks < 4096 ? blocks : 4096), kThreads, 0, s>>>(static_cast<uint4*>(p), n16,
                                                                                  make_uint4(w, w, w, w));
    return check_launch(what);
  }
  MSP_HIP(hipMemsetAsync(p, value, bytes, s), what);
  return MSP_OK;
}

// Block hash of a level's sorted keys (msp_hash_build / msp_subm_map): one slot per occupied block of 32
// consecutive Morton codes (2 x 4 x 4 sites), {key >> 5, first row << 32 | occupancy mask}.  The keys being
// sorted, a block's rows are contiguous, so row(key) = first + popc(mask below key's code): one 16-byte load
// answers every site of the block.  The slot is the block key's low bits (Morton-adjacent blocks share cache
// lines, a wave's 64 rows look up a handful of lines) plus a mix of the bits above the table size (batch, far
// regions), so scenes land apart.  Round 1-4 hashed every site with a mixing hash into a table of 2n random
// slots and wrote the map's mirror half by scatter after a memset of all K n entries.
constexpr int kBlockBits = 5;
constexpr unsigned kMapBlocks = 4096;  // grid cap of the counted submanifold map
#ifndef MSP_BLOCK_SLOT_LOCAL  // experiments: 1 = the slot is the block key's low bits (+ a mix of the rest)
#define MSP_BLOCK_SLOT_LOCAL 0
#endif
__device__ __forceinline__ uint64_t block_slot(uint64_t bk, uint64_t mask) {
  if (MSP_BLOCK_SLOT_LOCAL) return (bk + hash_key(bk >> __popcll(mask))) & mask;
  return hash_key(bk) & mask;
}

__global__ __launch_bounds__(kThreads) void hash_build_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                              uint64_t* __restrict__ table, uint64_t mask) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t bk = keys[i] >> kBlockBits;
  if (i > 0 && (keys[i - 1] >> kBlockBits) == bk) return;  // not the block's first row
  uint32_t occ = 0;
#pragma unroll 8
  for (int k = 0; k < (1 << kBlockBits); ++k) {  // the block's rows are keys[i .. i + 32) with the same block key
    if (i + k >= n) break;
    const uint64_t key = keys[i + k];
    if ((key >> kBlockBits) != bk) break;
    occ |= 1u << (key & ((1u << kBlockBits) - 1));
  }
  uint64_t h = block_slot(bk, mask);
  for (;;) {
    const unsigned long long prev =
        atomicCAS((unsigned long long*)&table[2 * h], (unsigned long long)kEmptyKey, (unsigned long long)bk);
    if (prev == kEmptyKey) {
      table[2 * h + 1] = ((uint64_t)i << 32) | occ;
      return;
    }
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ int32_t block_find(const uint64_t* __restrict__ table, uint64_t mask, uint64_t key) {
  const uint64_t bk = key >> kBlockBits;
  uint64_t h = block_slot(bk, mask);
  for (;;) {
    const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(table + 2 * h);
    if (e.x == bk) {
      const uint32_t occ = (uint32_t)e.y, c = (uint32_t)(key & ((1u << kBlockBits) - 1));
      if (!((occ >> c) & 1u)) return -1;
      return (int32_t)(e.y >> 32) + __popc(occ & ((1u << c) - 1u));
    }
    if (e.x == kEmptyKey) return -1;
    h = (h + 1) & mask;
  }
}

// Every entry of nbr[K][n] written (no memset).  A block covers 1024 consecutive rows of one offset, each thread
// four rows 256 apart: the four key loads and the four slot probes are independent, so a wave has four chains of
// (key -> probe) in flight instead of one (one row per thread was latency-bound: 247 us at level 0,
// profiles/r05/prof_r05final2).  Within each of the four steps a wave's 64 rows are consecutive (coalesced
// stores; their lookups at one offset share a few block slots).  Grid-stride over (offset, row block) with at
// most kMapBlocks blocks; part (nullable): each block's count of present entries (msp_subm_map_counted).
constexpr int kMapRows = 4;
__global__ __launch_bounds__(kThreads) void subm_map_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                            int log2s, int64_t size, int f,
                                                            const uint64_t* __restrict__ table, uint64_t mask,
                                                            int32_t* __restrict__ nbr, int32_t* __restrict__ part) {
  const int K = f * f * f, centre = (K - 1) / 2, h = f / 2;
  const int64_t nrb = (n + (int64_t)kThreads * kMapRows - 1) / ((int64_t)kThreads * kMapRows);
  int c = 0;  // present entries this wave wrote (part only)
  for (int64_t bi = blockIdx.x; bi < nrb * K; bi += gridDim.x) {
    const int o = (int)(bi / nrb);
    const int64_t i0 = (bi - (int64_t)o * nrb) * kThreads * kMapRows + threadIdx.x;
    const int dx = o / (f * f) - h, dy = (o / f) % f - h, dz = o % f - h;
    uint64_t key[kMapRows];
#pragma unroll
    for (int k = 0; k < kMapRows; ++k) {
      const int64_t i = i0 + (int64_t)k * kThreads;
      key[k] = (o != centre && i < n) ? keys[i] : 0;
    }
    int32_t j[kMapRows];
#pragma unroll
    for (int k = 0; k < kMapRows; ++k) {
      const int64_t i = i0 + (int64_t)k * kThreads;
      j[k] = -1;
      if (i < n) {
        if (o == centre) {
          j[k] = (int32_t)i;
        } else {
          int64_t b, x, y, z;
          split_key(key[k], log2s, b, x, y, z);
          const int64_t xx = x + dx, yy = y + dy, zz = z + dz;
          if (xx >= 0 && yy >= 0 && zz >= 0 && xx < size && yy < size && zz < size)
            j[k] = block_find(table, mask, make_key(b, xx, yy, zz, log2s));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kMapRows; ++k) {
      const int64_t i = i0 + (int64_t)k * kThreads;
      if (i < n) nbr[(int64_t)o * n + i] = j[k];
      if (part) c += __popcll(__ballot(j[k] >= 0));
    }
  }
  if (part) {
    __shared__ int wc[kThreads / 64];
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
#pragma unroll
      for (int w = 0; w < kThreads / 64; ++w) t += wc[w];
      part[blockIdx.x] = t;
    }
  }
}

// *total = the sum of part[0 .. nb) (one block, nb <= kMapBlocks: 16 loads per thread; int64, so the order does not
// matter).  Over one count per 256-entry block -- 137 k at level 0 -- this one block took 142 us.
__global__ __launch_bounds__(kThreads) void sum_parts_kernel(const int32_t* __restrict__ part, int64_t nb,
                                                             int64_t* __restrict__ total) {
  __shared__ int64_t ws[kThreads / 64];
  int64_t t = 0;
  for (int64_t i = threadIdx.x; i < nb; i += kThreads) t += part[i];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) t += __shfl_xor(t, d, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t s = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += ws[w];
    *total = s;
  }
}

__global__ __launch_bounds__(kThreads) void down_map_kernel(const uint64_t* __restrict__ keys, int64_t n_fine,
                                                            const int32_t* __restrict__ parent, int log2s,
                                                            int ls, int32_t* __restrict__ down,
                                                            int64_t n_coarse) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n_fine) return;
  int64_t b, x, y, z;
  split_key(keys[i], log2s, b, x, y, z);
  const int64_t m = (1 << ls) - 1;
  const int o = (int)((((x & m) << ls) + (y & m)) << ls) + (int)(z & m);
  down[(int64_t)o * n_coarse + parent[i]] = (int32_t)i;
}

// ---------------------------------------------------------------- pair lists
// Stable per-offset compaction of an offset-major map.  One block handles
// kSegTile consecutive rows of one offset.
__global__ __launch_bounds__(kThreads) void pair_count_kernel(const int32_t* __restrict__ map, int64_t n,
                                                              int64_t nrb, int64_t* __restrict__ counts) {
  const int o = blockIdx.y;
  const int64_t base = (int64_t)blockIdx.x * kSegTile + (int64_t)threadIdx.x * kSegItems;
  const int32_t* row = map + (int64_t)o * n;
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < kSegItems; ++j) {
    const int64_t i = base + j;
    if (i < n) c += row[i] >= 0;
  }
  int64_t tot;
  block_excl_scan<kThreads>(c, &tot);
  if (threadIdx.x == 0) counts[(int64_t)o * nrb + blockIdx.x] = tot;
}

__global__ void pair_starts_kernel(const int64_t* __restrict__ offs, int K, int64_t nrb, const int64_t* total,
                                   int64_t* __restrict__ off_start) {
  const int o = threadIdx.x + blockIdx.x * blockDim.x;
  if (o < K) off_start[o] = offs[(int64_t)o * nrb];
  if (o == K) off_start[K] = *total;
}

__global__ __launch_bounds__(kThreads) void pair_fill_kernel(const int32_t* __restrict__ map, int64_t n,
                                                             int64_t nrb, const int64_t* __restrict__ offs,
                                                             int32_t* __restrict__ pin,
                                                             int32_t* __restrict__ pout) {
  const int o = blockIdx.y;
  const int64_t base = (int64_t)blockIdx.x * kSegTile + (int64_t)threadIdx.x * kSegItems;
  const int32_t* row = map + (int64_t)o * n;
  int32_t v[kSegItems];
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < kSegItems; ++j) {
    const int64_t i = base + j;
    v[j] = (i < n) ? row[i] : -1;
    c += v[j] >= 0;
  }
  int64_t tot;
  int64_t p = block_excl_scan<kThreads>(c, &tot) + offs[(int64_t)o * nrb + blockIdx.x];
#pragma unroll
  for (int j = 0; j < kSegItems; ++j) {
    if (v[j] >= 0) {
      pin[p] = v[j];
      pout[p] = (int32_t)(base + j);
      ++p;
    }
  }
}

// ---------------------------------------------------------------- tile rulebook
// Output tiles of TW*64 rows; one wave per 64-row band, TW waves per tile
// (a block of kThreads holds 4/TW tiles).  For each filter offset every wave
// ballots which of its rows have that neighbour, the TW wave counts are
// combined through LDS, and the present rows are compacted (wave prefix +
// mbcnt) into 16-row chunks that share the offset.
constexpr int kChunk = MSP_CHUNK;

// Phase 1 (both kernels): every wave ballots its 64 rows for all K offsets
// and leaves the per-offset popcounts (and first present input row) in LDS;
// one barrier; then per-tile sums over the TW waves.  K <= 255.
template <int TW>
__global__ __launch_bounds__(kThreads) void tile_count_kernel(const int32_t* __restrict__ map, int K, int64_t n,
                                                              int64_t n_tiles, int64_t* __restrict__ cnt) {
  __shared__ uint8_t pc_s[kThreads / 64][256];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = wave % TW;
  const int64_t t = (int64_t)blockIdx.x * (kThreads / 64 / TW) + wave / TW;
  const int64_t r = t * (64 * TW) + sub * 64 + lane;
  const bool live = t < n_tiles && r < n;

  for (int o = 0; o < K; ++o) {
    const int pc = __popcll(ballot64(live && map[(int64_t)o * n + r] >= 0));
    if (lane == 0) pc_s[wave][o] = (uint8_t)pc;
  }
  if (TW > 1) __syncthreads();
  if (sub != 0 || t >= n_tiles) return;
  int64_t nch = 0;
  for (int o = lane; o < K; o += 64) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < TW; ++w) tot += pc_s[wave + w][o];
    nch += (tot + kChunk - 1) / kChunk;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) nch += __shfl_xor(nch, d, 64);
  if (lane == 0) cnt[t] = nch;  // (the largest: the scan's max_out)
}

template <int TW>
__global__ __launch_bounds__(kThreads) void tile_fill_kernel(const int32_t* __restrict__ map, int K, int64_t n,
                                                             int64_t n_tiles,
                                                             const int64_t* __restrict__ tile_start,
                                                             uint8_t* __restrict__ chunk_off,
                                                             int32_t* __restrict__ chunk_src,
                                                             uint16_t* __restrict__ chunk_row) {
  constexpr int TR = 64 * TW;
  constexpr int TPB = kThreads / 64 / TW;  // tiles per block
  __shared__ uint8_t pc_s[kThreads / 64][256];
  __shared__ int32_t first_s[kThreads / 64][256];
  __shared__ int32_t cst_s[TPB][256];  // first chunk of each offset (relative to the tile)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = wave % TW, tb = wave / TW;
  const int64_t t = (int64_t)blockIdx.x * TPB + tb;
  const int slot = sub * 64 + lane;  // row inside the tile
  const int64_t r = t * TR + slot;
  const bool live = t < n_tiles && r < n;

  for (int o = 0; o < K; ++o) {
    const int32_t v = live ? map[(int64_t)o * n + r] : -1;
    const unsigned long long m = ballot64(v >= 0);
    const int32_t vf = m ? __shfl(v, __ffsll((long long)m) - 1) : -1;
    if (lane == 0) {
      pc_s[wave][o] = (uint8_t)__popcll(m);
      first_s[wave][o] = vf;
    }
  }
  __syncthreads();
  if (sub == 0) {
    // per offset: chunk count, exclusive prefix over offsets (64 at a time),
    // and the tile's first present input row (padding slots repeat it)
    int carry = 0;
    for (int o0 = 0; o0 < K; o0 += 64) {
      const int o = o0 + lane;
      int nchk = 0;
      int32_t vfirst = -1;
      if (o < K) {
        int tot = 0;
#pragma unroll
        for (int w = 0; w < TW; ++w) {
          tot += pc_s[wave + w][o];
          const int32_t f = first_s[wave + w][o];
          if (vfirst < 0) vfirst = f;
        }
        nchk = (tot + kChunk - 1) / kChunk;
      }
      const int incl = wave_incl_scan(nchk);
      if (o < K) {
        cst_s[tb][o] = carry + incl - nchk;
        first_s[wave][o] = vfirst;
      }
      carry += __shfl(incl, 63, 64);
    }
  }
  __syncthreads();
  if (t >= n_tiles) return;
  const int64_t c0 = tile_start[t];
  const int w0 = wave - sub;

  for (int o = 0; o < K; ++o) {
    int before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < TW; ++w) {
      const int p = pc_s[w0 + w][o];
      if (w < sub) before += p;
      tot += p;
    }
    if (tot == 0) continue;  // uniform over the tile
    const int64_t c = c0 + cst_s[tb][o];
    const int nch = (tot + kChunk - 1) / kChunk;
    const int32_t v = live ? map[(int64_t)o * n + r] : -1;
    if (v >= 0) {
      const unsigned long long m = ballot64(true);  // lanes with a neighbour (exec = v >= 0)
      const int pos = before + mbcnt64(m);
      const int64_t e = (c + pos / kChunk) * kChunk + (pos % kChunk);
      chunk_src[e] = v;
      chunk_row[e] = (uint16_t)slot;
    }
    if (slot >= tot && slot < nch * kChunk) {  // padding slots of the last chunk
      const int64_t e = (c + slot / kChunk) * kChunk + (slot % kChunk);
      chunk_src[e] = first_s[w0][o];
      chunk_row[e] = (uint16_t)TR;
    }
    if (slot < nch) chunk_off[c + slot] = (uint8_t)o;
  }
}

__global__ __launch_bounds__(kThreads) void decode_kernel(const uint64_t* __restrict__ keys, int64_t n, int log2s,
                                                          int64_t* __restrict__ coords) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  int64_t b, x, y, z;
  split_key(keys[i], log2s, b, x, y, z);
  coords[4 * i + 0] = x;
  coords[4 * i + 1] = y;
  coords[4 * i + 2] = z;
  coords[4 * i + 3] = b;
}

inline unsigned grid1(int64_t n) { return (unsigned)ceil_div(n > 0 ? n : 1, kThreads); }

}  // namespace msp

using namespace msp;

extern "C" {

int msp_point_keys(const int64_t* coords, int64_t n, int64_t row_stride, int log2_size, int64_t spatial_size,
                   uint64_t* keys, int32_t* vals, int64_t* stats, msp_stream_t stream) {
  MSP_REQUIRE(n >= 0 && row_stride >= 4, "msp_point_keys: bad n/row_stride");
  MSP_REQUIRE(log2_size >= 1 && log2_size <= 20 && (1ll << log2_size) >= spatial_size,
              "msp_point_keys: log2_size %d does not cover spatial_size %lld", log2_size,
              (long long)spatial_size);
  MSP_REQUIRE(n < (1ll << 31), "msp_point_keys: too many points");
  if (n == 0) return MSP_OK;
  point_keys_kernel<<<grid1(n), kThreads, 0, as_stream(stream)>>>(coords, n, row_stride, log2_size,
                                                                   spatial_size, keys, vals, stats);
  return check_launch("msp_point_keys");
}

int msp_batch_starts(const int64_t* coords, int64_t n, int64_t row_stride, int64_t n_batch, int64_t* starts,
                     msp_stream_t stream) {
  MSP_REQUIRE(n >= 0 && row_stride >= 4 && n_batch >= 0, "msp_batch_starts: bad n/row_stride/n_batch");
  MSP_REQUIRE(starts != nullptr, "msp_batch_starts: starts is NULL");
  MSP_REQUIRE(n == 0 || coords != nullptr, "msp_batch_starts: coords is NULL");
  batch_starts_kernel<<<grid1(n_batch + 1), kThreads, 0, as_stream(stream)>>>(coords, n, row_stride, n_batch,
                                                                              starts);
  return check_launch("msp_batch_starts");
}

// ---------------------------------------------------------------- dense row order
// Row order for the dense row-group convolution (msp_conv_nbr): inside each
// window of 2^lw consecutive rows (spatially compact in key order), rows are
// sorted stably by their neighbour mask, so a 16-row group mostly shares its
// offsets (fewer zero rows in the MFMA tiles: at 4096-row windows about 0.74
// of a group's (offset, row) slots carry a rule at level 1 instead of 0.49)
// while the gathers of a window stay local.  Keys (window << K | mask) are
// radix sorted with their row numbers; the neighbour map is then permuted.
static __global__ __launch_bounds__(256) void dense_keys_kernel(const int32_t* __restrict__ nbr, int K, int64_t n,
                                                                int lw, uint64_t* __restrict__ keys,
                                                                int32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t m = 0;
  for (int o = 0; o < K; ++o) m |= (uint64_t)(nbr[(int64_t)o * n + i] >= 0) << o;
  keys[i] = ((uint64_t)(i >> lw) << K) | m;
  vals[i] = (int32_t)i;
}

static __global__ __launch_bounds__(256) void permute_map_kernel(const int32_t* __restrict__ nbr, int K, int64_t n,
                                                                 const int32_t* __restrict__ perm,
                                                                 int32_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int64_t src = perm[j];
  for (int o = 0; o < K; ++o) out[(int64_t)o * n + j] = nbr[(int64_t)o * n + src];
}

static int dense_order_bits(int64_t n, int K, int lw) {
  int wb = 0;
  while (wb < 40 && ((n - 1) >> lw) >> wb) ++wb;
  return K + wb;
}

size_t msp_dense_order_workspace_size(int64_t n, int K, int log2_window) {
  if (n <= 0 || K <= 0 || K > 32 || log2_window < 4 || log2_window > 30) return 0;
  const int end_bit = dense_order_bits(n, K, log2_window);
  auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
  return 2 * r((size_t)n * 8) + r((size_t)n * 4) + r(msp_sort_workspace_size(n, end_bit));
}

int msp_dense_order(const int32_t* nbr, int K, int64_t n, int log2_window, int32_t* perm, int32_t* nbr_perm,
                    void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= 32, "msp_dense_order: K must be in [1, 32] (got %d)", K);
  MSP_REQUIRE(log2_window >= 4 && log2_window <= 30, "msp_dense_order: log2_window must be in [4, 30]");
  MSP_REQUIRE(n >= 0, "msp_dense_order: n must be >= 0");
  if (n == 0) return MSP_OK;
  const size_t need = msp_dense_order_workspace_size(n, K, log2_window);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_dense_order: workspace too small (%zu < %zu)", ws_bytes, need);
  hipStream_t s = as_stream(stream);
  auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
  char* w = static_cast<char*>(ws);
  uint64_t* k_in = reinterpret_cast<uint64_t*>(w);
  uint64_t* k_out = reinterpret_cast<uint64_t*>(w + r((size_t)n * 8));
  int32_t* v_in = reinterpret_cast<int32_t*>(w + 2 * r((size_t)n * 8));
  void* sws = w + 2 * r((size_t)n * 8) + r((size_t)n * 4);
  const int end_bit = dense_order_bits(n, K, log2_window);
  const unsigned nb = (unsigned)ceil_div(n, 256);
  dense_keys_kernel<<<nb, 256, 0, s>>>(nbr, K, n, log2_window, k_in, v_in);
  const int rc = msp_sort_pairs(k_in, k_out, v_in, perm, n, end_bit, sws, msp_sort_workspace_size(n, end_bit), stream);
  if (rc) return rc;
  permute_map_kernel<<<nb, 256, 0, s>>>(nbr, K, n, perm, nbr_perm);
  return check_launch("msp_dense_order");
}

int msp_segment(const uint64_t* sorted_keys, int64_t n, int shift, const int32_t* perm, int32_t* seg_of,
                int32_t* p2v, uint64_t* uniq_keys, int32_t* seg_start, int64_t* n_uniq, void* ws,
                size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(n >= 0 && shift >= 0 && shift < 64, "msp_segment: bad args");
  MSP_REQUIRE((p2v == nullptr) == (perm == nullptr), "msp_segment: perm and p2v go together");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    MSP_HIP(hipMemsetAsync(n_uniq, 0, sizeof(int64_t), s), "msp_segment");
    MSP_HIP(hipMemsetAsync(seg_start, 0, sizeof(int32_t), s), "msp_segment");
    return MSP_OK;
  }
  const int64_t nb = ceil_div(n, kSegTile);
  MSP_REQUIRE(ws_bytes >= (size_t)(nb + 1) * sizeof(int64_t), "msp_segment: workspace too small");
  int64_t* sums = reinterpret_cast<int64_t*>(ws);
  seg_count_kernel<<<nb, kThreads, 0, s>>>(sorted_keys, n, shift, sums);
  int rc = scan_small_inplace(sums, nb, n_uniq, s);
  if (rc) return rc;
  seg_apply_kernel<<<nb, kThreads, 0, s>>>(sorted_keys, n, shift, sums, perm, seg_of, p2v, uniq_keys,
                                           seg_start);
  return check_launch("msp_segment");
}

int64_t msp_hash_capacity(int64_t n) {
  int64_t cap = 1024;
  while (cap < 2 * n) cap <<= 1;
  return cap;
}

int msp_hash_build(const uint64_t* keys, int64_t n, uint64_t* table, int64_t cap, msp_stream_t stream) {
  MSP_REQUIRE(cap >= 2 * n && (cap & (cap - 1)) == 0, "msp_hash_build: capacity must be a power of 2 >= 2n");
  hipStream_t s = as_stream(stream);
  const int rc = fill_bytes(table, 0xFF, (size_t)cap * 16, s, "msp_hash_build");  // every slot empty
  if (rc || n == 0) return rc;
  hash_build_kernel<<<grid1(n), kThreads, 0, s>>>(keys, n, table, (uint64_t)(cap - 1));
  return check_launch("msp_hash_build");
}

// the counted map's grid (one partial count per block, written by every block)
static unsigned subm_map_blocks(int64_t n, int filter_size) {
  const int64_t K = (int64_t)filter_size * filter_size * filter_size;
  return (unsigned)std::min<int64_t>(ceil_div(n, (int64_t)kThreads * kMapRows) * K, kMapBlocks);
}

size_t msp_subm_map_workspace_size(int64_t n, int filter_size) {
  const unsigned nb = n > 0 ? subm_map_blocks(n, filter_size) : 1u;
  return (size_t)(nb > 0 ? nb : 1u) * sizeof(int32_t);
}

int msp_subm_map_counted(const uint64_t* keys, int64_t n, int log2_size, int64_t spatial_size, int filter_size,
                         const uint64_t* table, int64_t cap, int32_t* nbr, int64_t* n_rules, void* ws,
                         size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(filter_size >= 1 && (filter_size & 1) == 1 && filter_size <= 5,
              "msp_subm_map_counted: filter_size must be odd and <= 5 (got %d)", filter_size);
  MSP_REQUIRE((cap & (cap - 1)) == 0, "msp_subm_map_counted: bad capacity");
  MSP_REQUIRE(n_rules && ws && ws_bytes >= msp_subm_map_workspace_size(n, filter_size),
              "msp_subm_map_counted: NULL count or workspace too small");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    MSP_HIP(hipMemsetAsync(n_rules, 0, sizeof(int64_t), s), "msp_subm_map_counted");
    return MSP_OK;
  }
  const unsigned nb = subm_map_blocks(n, filter_size);
  int32_t* part = static_cast<int32_t*>(ws);
  subm_map_kernel<<<nb, kThreads, 0, s>>>(keys, n, log2_size, spatial_size, filter_size, table, (uint64_t)(cap - 1),
                                          nbr, part);
  sum_parts_kernel<<<1, kThreads, 0, s>>>(part, nb, n_rules);
  return check_launch("msp_subm_map_counted");
}

int msp_subm_map(const uint64_t* keys, int64_t n, int log2_size, int64_t spatial_size, int filter_size,
                 const uint64_t* table, int64_t cap, int32_t* nbr, msp_stream_t stream) {
  MSP_REQUIRE(filter_size >= 1 && (filter_size & 1) == 1 && filter_size <= 5,
              "msp_subm_map: filter_size must be odd and <= 5 (got %d)", filter_size);
  MSP_REQUIRE((cap & (cap - 1)) == 0, "msp_subm_map: bad capacity");
  if (n == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  const unsigned nb = subm_map_blocks(n, filter_size);
  subm_map_kernel<<<nb, kThreads, 0, s>>>(keys, n, log2_size, spatial_size, filter_size, table, (uint64_t)(cap - 1),
                                          nbr, nullptr);
  return check_launch("msp_subm_map");
}

int msp_down_map(const uint64_t* fine_keys, int64_t n_fine, const int32_t* parent_of, int log2_size_fine,
                 int log2_stride, int32_t* down, int64_t n_coarse, msp_stream_t stream) {
  MSP_REQUIRE(log2_stride >= 1 && log2_stride <= 2, "msp_down_map: stride must be 2 or 4");
  const int K = 1 << (3 * log2_stride);
  hipStream_t s = as_stream(stream);
  const int rc = fill_bytes(down, 0xFF, (size_t)K * n_coarse * sizeof(int32_t), s, "msp_down_map");
  if (rc) return rc;
  if (n_fine == 0) return MSP_OK;
  down_map_kernel<<<grid1(n_fine), kThreads, 0, s>>>(fine_keys, n_fine, parent_of, log2_size_fine,
                                                     log2_stride, down, n_coarse);
  return check_launch("msp_down_map");
}

int msp_pair_lists(const int32_t* map, int K, int64_t n, int32_t* pair_in, int32_t* pair_out, int64_t cap,
                   int64_t* off_start, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= 65535 && n >= 0, "msp_pair_lists: bad K/n");
  hipStream_t s = as_stream(stream);
  const int64_t nrb = ceil_div(n > 0 ? n : 1, kSegTile);
  const int64_t m = (int64_t)K * nrb;
  // workspace: counts[m] | offs[m] | total | scan ws
  const size_t need = (size_t)(2 * m + 1) * sizeof(int64_t) + scan_ws_bytes(m);
  MSP_REQUIRE(ws_bytes >= need, "msp_pair_lists: workspace too small (%zu < %zu)", ws_bytes, need);
  int64_t* counts = reinterpret_cast<int64_t*>(ws);
  int64_t* offs = counts + m;
  int64_t* total = offs + m;
  void* sws = total + 1;
  dim3 grid((unsigned)nrb, (unsigned)K);
  if (cap <= 0) {  // counting call; the filling call reuses its workspace (block offsets)
    pair_count_kernel<<<grid, kThreads, 0, s>>>(map, n, nrb, counts);
    int rc = scan_exclusive_i64(counts, offs, m, total, sws, scan_ws_bytes(m), s);
    if (rc) return rc;
    pair_starts_kernel<<<(unsigned)ceil_div(K + 1, 256), 256, 0, s>>>(offs, K, nrb, total, off_start);
  } else {
    pair_fill_kernel<<<grid, kThreads, 0, s>>>(map, n, nrb, offs, pair_in, pair_out);
  }
  return check_launch("msp_pair_lists");
}

int msp_tile_rulebook(const int32_t* map, int K, int64_t n, int tile_rows, int64_t* tile_start,
                      uint8_t* chunk_off, int32_t* chunk_src, uint16_t* chunk_row, int64_t chunk_cap, void* ws,
                      size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(K >= 1 && K <= 255 && n >= 0, "msp_tile_rulebook: K must be in [1,255]");
  MSP_REQUIRE(tile_rows == 64 || tile_rows == 128 || tile_rows == 256,
              "msp_tile_rulebook: tile_rows must be 64, 128 or 256 (got %d)", tile_rows);
  hipStream_t s = as_stream(stream);
  const int64_t n_tiles = ceil_div(n, tile_rows);
  const size_t need = (size_t)(n_tiles + 1) * sizeof(int64_t) + scan_ws_bytes(n_tiles);
  MSP_REQUIRE(ws_bytes >= need, "msp_tile_rulebook: workspace too small (%zu < %zu)", ws_bytes, need);
  if (n_tiles == 0) {
    MSP_HIP(hipMemsetAsync(tile_start, 0, 2 * sizeof(int64_t), s), "msp_tile_rulebook");
    return MSP_OK;
  }
  int64_t* cnt = reinterpret_cast<int64_t*>(ws);
  void* sws = cnt + n_tiles + 1;
  const int tw = tile_rows / 64;
  const unsigned g = (unsigned)ceil_div(n_tiles, kThreads / 64 / tw);
  if (chunk_cap <= 0) {  // counting call; the filling call reuses its tile_start
    switch (tw) {
      case 1: tile_count_kernel<1><<<g, kThreads, 0, s>>>(map, K, n, n_tiles, cnt); break;
      case 2: tile_count_kernel<2><<<g, kThreads, 0, s>>>(map, K, n, n_tiles, cnt); break;
      default: tile_count_kernel<4><<<g, kThreads, 0, s>>>(map, K, n, n_tiles, cnt); break;
    }
    const int rc = scan_exclusive_i64(cnt, tile_start, n_tiles, tile_start + n_tiles, sws, scan_ws_bytes(n_tiles),
                                      s, tile_start + n_tiles + 1);
    if (rc) return rc;
  } else {
    switch (tw) {
      case 1:
        tile_fill_kernel<1><<<g, kThreads, 0, s>>>(map, K, n, n_tiles, tile_start, chunk_off, chunk_src, chunk_row);
        break;
      case 2:
        tile_fill_kernel<2><<<g, kThreads, 0, s>>>(map, K, n, n_tiles, tile_start, chunk_off, chunk_src, chunk_row);
        break;
      default:
        tile_fill_kernel<4><<<g, kThreads, 0, s>>>(map, K, n, n_tiles, tile_start, chunk_off, chunk_src, chunk_row);
        break;
    }
  }
  return check_launch("msp_tile_rulebook");
}

int msp_decode_keys(const uint64_t* keys, int64_t n, int log2_size, int64_t* coords, msp_stream_t stream) {
  if (n == 0) return MSP_OK;
  decode_kernel<<<grid1(n), kThreads, 0, as_stream(stream)>>>(keys, n, log2_size, coords);
  return check_launch("msp_decode_keys");
}

}  // extern "C"
