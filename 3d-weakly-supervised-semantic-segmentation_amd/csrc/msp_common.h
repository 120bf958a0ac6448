// Shared helpers for the mi3dsparse HIP library (gfx950 / CDNA4).
//
// Error convention (include/mi3dsparse.h): every entry point returns 0 on
// success or a negative MSP_E* code; the message is kept per thread and read
// back with msp_last_error().  Kernels never abort the process.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>

#include "../../include/mi3dsparse.h"

namespace msp {

void set_error(const char* fmt, ...);

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch error %s", what, hipGetErrorString(e));
    return MSP_EHIP;
  }
  return MSP_OK;
}

#define MSP_REQUIRE(cond, ...)                 \
  do {                                         \
    if (!(cond)) {                             \
      ::msp::set_error(__VA_ARGS__);           \
      return MSP_EINVAL;                       \
    }                                          \
  } while (0)

#define MSP_HIP(call, what)                                                        \
  do {                                                                             \
    hipError_t _e = (call);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::msp::set_error("%s: %s", what, hipGetErrorString(_e));                     \
      return MSP_EHIP;                                                             \
    }                                                                              \
  } while (0)

inline hipStream_t as_stream(msp_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- per-device caches (the library's only process-wide state; include/mi3dsparse.h) -----------------------
// Both are indexed by the current device and held in atomics: several host threads and several devices may call
// the library concurrently.  device_cu_count(): the current device's CU count, read once per device.
// raise_lds_limit(): hipFuncSetAttribute(MaxDynamicSharedMemorySize) for kernel `slot` (a small integer per
// kernel, < 64) on the current device, once per (device, slot); the attribute is idempotent, so two threads
// racing to set it are harmless.
int device_cu_count();
int raise_lds_limit(const void* fn, int bytes, int slot, const char* what);
enum LdsSlot { kLdsNinF32 = 0, kLdsNinX6 = 8 };  // + template variant (NTT 1..8 / NT 1..2)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- Morton (Z-order) keys -------------------------------------------------
// key = batch << (3*S) | interleave(x, y, z), with x in the highest bit of each
// 3-bit group.  With this layout the key of the parent cell under a stride-2^k
// convolution is exactly key >> 3k, so the sorted key order is preserved by
// coarsening and the children of one parent are a contiguous run.  For a
// stride-2 step the child offset index (key & 7) equals SparseConvNet's
// last-axis-fastest filter offset (x&1)*4 + (y&1)*2 + (z&1).
__host__ __device__ inline uint64_t part1by2(uint64_t v) {
  v &= 0x1fffffull;
  v = (v | (v << 32)) & 0x1f00000000ffffull;
  v = (v | (v << 16)) & 0x1f0000ff0000ffull;
  v = (v | (v << 8)) & 0x100f00f00f00f00full;
  v = (v | (v << 4)) & 0x10c30c30c30c30c3ull;
  v = (v | (v << 2)) & 0x1249249249249249ull;
  return v;
}

__host__ __device__ inline uint64_t compact1by2(uint64_t v) {
  v &= 0x1249249249249249ull;
  v = (v ^ (v >> 2)) & 0x10c30c30c30c30c3ull;
  v = (v ^ (v >> 4)) & 0x100f00f00f00f00full;
  v = (v ^ (v >> 8)) & 0x1f0000ff0000ffull;
  v = (v ^ (v >> 16)) & 0x1f00000000ffffull;
  v = (v ^ (v >> 32)) & 0x1fffffull;
  return v;
}

__host__ __device__ inline uint64_t morton3(uint64_t x, uint64_t y, uint64_t z) {
  return (part1by2(x) << 2) | (part1by2(y) << 1) | part1by2(z);
}

__host__ __device__ inline uint64_t make_key(int64_t b, int64_t x, int64_t y, int64_t z, int log2s) {
  return ((uint64_t)b << (3 * log2s)) | morton3((uint64_t)x, (uint64_t)y, (uint64_t)z);
}

__host__ __device__ inline void split_key(uint64_t key, int log2s, int64_t& b, int64_t& x, int64_t& y,
                                          int64_t& z) {
  const uint64_t m = (log2s >= 21) ? ~0ull : ((1ull << (3 * log2s)) - 1);
  const uint64_t mort = key & m;
  b = (int64_t)(key >> (3 * log2s));
  x = (int64_t)compact1by2(mort >> 2);
  y = (int64_t)compact1by2(mort >> 1);
  z = (int64_t)compact1by2(mort);
}

// Open-addressing hash (linear probing) of the neighbour queries (msp_meta.hip: block_slot / block_find).
constexpr uint64_t kEmptyKey = ~0ull;
__host__ __device__ inline uint64_t hash_key(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// wave64 helpers
__device__ inline int lane_id() { return threadIdx.x & 63; }
__device__ inline unsigned long long ballot64(bool p) { return __ballot(p); }
__device__ inline int mbcnt64(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}

// Inclusive scan across a wave64.
template <typename T>
__device__ inline T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Exclusive scan of one value per thread across a block of NT threads
// (NT multiple of 64); returns the exclusive prefix, block total in *total.
template <int NT, typename T>
__device__ inline T block_excl_scan(T v, T* total) {
  __shared__ T wsum[NT / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  T off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    if (w < wave) off += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

// Exclusive scan over int64 in device memory, used by every compaction.
// Workspace: msp_scan_workspace_size(n) bytes.
// max_out (optional): the largest input (the count passes' largest tile).
int scan_exclusive_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* total, void* ws, size_t ws_bytes,
                       hipStream_t s, int64_t* max_out = nullptr);
size_t scan_ws_bytes(int64_t n);
// Exclusive scan of a short array in place with one block; total -> *total.
int scan_small_inplace(int64_t* data, int64_t n, int64_t* total, hipStream_t s);

}  // namespace msp
