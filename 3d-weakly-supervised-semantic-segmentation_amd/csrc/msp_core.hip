// Error state, ABI version and the device-wide exclusive scan that every
// compaction in the library (voxel dedup, rulebooks, pair lists) is built on.
#include "msp_common.h"

#include <atomic>
#include <cstring>

namespace msp {

static thread_local char g_err[512] = "";

constexpr int kMaxDevices = 64;
static std::atomic<int> g_cus[kMaxDevices];
static std::atomic<unsigned long long> g_lds_raised[kMaxDevices];

int device_cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  int n = g_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  g_cus[dev].store(n, std::memory_order_relaxed);
  return n;
}

int raise_lds_limit(const void* fn, int bytes, int slot, const char* what) {
  int dev = 0;
  MSP_HIP(hipGetDevice(&dev), what);
  const unsigned long long bit = 1ull << (slot & 63);
  if (dev >= 0 && dev < kMaxDevices && (g_lds_raised[dev].load(std::memory_order_acquire) & bit)) return MSP_OK;
  MSP_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes), what);
  if (dev >= 0 && dev < kMaxDevices) g_lds_raised[dev].fetch_or(bit, std::memory_order_acq_rel);
  return MSP_OK;
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---- block-level scan helpers (256 threads = 4 waves) ----------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;  // items per thread
constexpr int kScanTile = kScanThreads * kScanItems;

// Largest value over the block (every thread gets it): wave maxima by shuffles, then the four waves' in LDS.
__device__ int64_t block_max_i64(int64_t v) {
  __shared__ int64_t wm[kScanThreads / 64];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const int64_t o = __shfl_xor(v, d, 64);
    v = o > v ? o : v;
  }
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t m = wm[0];
#pragma unroll
  for (int w = 1; w < kScanThreads / 64; ++w) m = wm[w] > m ? wm[w] : m;
  __syncthreads();
  return m;
}

// block_max (optional): the block's largest input, for the scan's max_out (round 5: the count passes' largest
// tile used to need a memset and an atomicMax of their own, ~8 us of side-stream latency per count)
__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(const int64_t* __restrict__ in, int64_t n,
                                                                   int64_t* __restrict__ block_sums,
                                                                   int64_t* __restrict__ block_max) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  int64_t s = 0, mx = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + (int64_t)k * kScanThreads + threadIdx.x;
    if (i < n) {
      s += in[i];
      mx = in[i] > mx ? in[i] : mx;
    }
  }
  int64_t tot;
  block_excl_scan<kScanThreads>(s, &tot);
  if (block_max) mx = block_max_i64(mx);
  if (threadIdx.x == 0) {
    block_sums[blockIdx.x] = tot;
    if (block_max) block_max[blockIdx.x] = mx;
  }
}

// single block: exclusive scan of the block sums in place, total -> *total; max_out (optional) = the largest of
// block_max[0 .. nb)
__global__ __launch_bounds__(kScanThreads) void scan_blocks_kernel(int64_t* __restrict__ sums, int64_t nb,
                                                                   int64_t* __restrict__ total,
                                                                   const int64_t* __restrict__ block_max,
                                                                   int64_t* __restrict__ max_out) {
  int64_t carry = 0, mx = 0;
  for (int64_t base = 0; base < nb; base += kScanThreads) {
    int64_t i = base + threadIdx.x;
    int64_t v = (i < nb) ? sums[i] : 0;
    if (block_max && i < nb) mx = block_max[i] > mx ? block_max[i] : mx;
    int64_t tot;
    int64_t ex = block_excl_scan<kScanThreads>(v, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
  if (max_out) mx = block_max_i64(mx);
  if (threadIdx.x == 0) {
    if (total) *total = carry;
    if (max_out) *max_out = mx;
  }
}

__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(const int64_t* __restrict__ in, int64_t n,
                                                                  const int64_t* __restrict__ block_off,
                                                                  int64_t* __restrict__ out) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  // each thread owns kScanItems consecutive items
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + (int64_t)threadIdx.x * kScanItems + k;
    v[k] = (i < n) ? in[i] : 0;
    s += v[k];
  }
  int64_t tot;
  int64_t ex = block_excl_scan<kScanThreads>(s, &tot) + block_off[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + (int64_t)threadIdx.x * kScanItems + k;
    if (i < n) out[i] = ex;
    ex += v[k];
  }
}

// n <= kScanTile: the whole scan and its total in one launch (most of a metadata build's scans are this small:
// per-tile or per-offset counts of the smaller levels; three dependent launches were ~10 us each on the side
// stream)
__global__ __launch_bounds__(kScanThreads) void scan_one_kernel(const int64_t* __restrict__ in, int64_t n,
                                                                int64_t* __restrict__ out, int64_t* __restrict__ total,
                                                                int64_t* __restrict__ max_out) {
  int64_t v[kScanItems];
  int64_t s = 0, mx = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = (int64_t)threadIdx.x * kScanItems + k;
    v[k] = (i < n) ? in[i] : 0;
    s += v[k];
    mx = v[k] > mx ? v[k] : mx;
  }
  if (max_out) {
    mx = block_max_i64(mx);
    if (threadIdx.x == 0) *max_out = mx;  // (before the in-place writes below: max_out may alias nothing read)
  }
  int64_t tot;
  int64_t ex = block_excl_scan<kScanThreads>(s, &tot);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = (int64_t)threadIdx.x * kScanItems + k;
    if (i < n) out[i] = ex;
    ex += v[k];
  }
  if (threadIdx.x == 0 && total) *total = tot;
}

size_t scan_ws_bytes(int64_t n) { return (size_t)(2 * (ceil_div(n, kScanTile) + 1)) * sizeof(int64_t); }

int scan_exclusive_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* total, void* ws, size_t ws_bytes,
                       hipStream_t s, int64_t* max_out) {
  MSP_REQUIRE(n >= 0, "scan: n < 0");
  MSP_REQUIRE(ws_bytes >= scan_ws_bytes(n), "scan: workspace too small (%zu < %zu)", ws_bytes,
              scan_ws_bytes(n));
  const int64_t nb = ceil_div(n, kScanTile);
  int64_t* sums = reinterpret_cast<int64_t*>(ws);
  int64_t* bmax = max_out ? sums + nb + 1 : nullptr;
  if (nb == 0) {
    if (total) MSP_HIP(hipMemsetAsync(total, 0, sizeof(int64_t), s), "scan: memset");
    if (max_out) MSP_HIP(hipMemsetAsync(max_out, 0, sizeof(int64_t), s), "scan: memset");
    return MSP_OK;
  }
  if (nb == 1) {
    scan_one_kernel<<<1, kScanThreads, 0, s>>>(in, n, out, total, max_out);
    return check_launch("scan_exclusive_i64");
  }
  scan_reduce_kernel<<<nb, kScanThreads, 0, s>>>(in, n, sums, bmax);
  scan_blocks_kernel<<<1, kScanThreads, 0, s>>>(sums, nb, total, bmax, max_out);
  scan_apply_kernel<<<nb, kScanThreads, 0, s>>>(in, n, sums, out);
  return check_launch("scan_exclusive_i64");
}

int scan_small_inplace(int64_t* data, int64_t n, int64_t* total, hipStream_t s) {
  scan_blocks_kernel<<<1, kScanThreads, 0, s>>>(data, n, total, nullptr, nullptr);
  return check_launch("scan_small_inplace");
}

}  // namespace msp

extern "C" {

int msp_abi_version(void) { return 10; }

const char* msp_last_error(void) { return msp::g_err; }

size_t msp_scan_workspace_size(int64_t n) { return msp::scan_ws_bytes(n); }

}  // extern "C"
