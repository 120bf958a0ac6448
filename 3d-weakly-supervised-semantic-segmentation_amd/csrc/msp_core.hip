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

__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(const int64_t* __restrict__ in, int64_t n,
                                                                   int64_t* __restrict__ block_sums) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + (int64_t)k * kScanThreads + threadIdx.x;
    if (i < n) s += in[i];
  }
  int64_t tot;
  block_excl_scan<kScanThreads>(s, &tot);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

// single block: exclusive scan of the block sums in place, total -> *total
__global__ __launch_bounds__(kScanThreads) void scan_blocks_kernel(int64_t* __restrict__ sums, int64_t nb,
                                                                   int64_t* __restrict__ total) {
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += kScanThreads) {
    int64_t i = base + threadIdx.x;
    int64_t v = (i < nb) ? sums[i] : 0;
    int64_t tot;
    int64_t ex = block_excl_scan<kScanThreads>(v, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
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
                                                                int64_t* __restrict__ out, int64_t* __restrict__ total) {
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = (int64_t)threadIdx.x * kScanItems + k;
    v[k] = (i < n) ? in[i] : 0;
    s += v[k];
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

size_t scan_ws_bytes(int64_t n) { return (size_t)(ceil_div(n, kScanTile) + 1) * sizeof(int64_t); }

int scan_exclusive_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* total, void* ws, size_t ws_bytes,
                       hipStream_t s) {
  MSP_REQUIRE(n >= 0, "scan: n < 0");
  MSP_REQUIRE(ws_bytes >= scan_ws_bytes(n), "scan: workspace too small (%zu < %zu)", ws_bytes,
              scan_ws_bytes(n));
  const int64_t nb = ceil_div(n, kScanTile);
  int64_t* sums = reinterpret_cast<int64_t*>(ws);
  if (nb == 0) {
    if (total) MSP_HIP(hipMemsetAsync(total, 0, sizeof(int64_t), s), "scan: memset");
    return MSP_OK;
  }
  if (nb == 1) {
    scan_one_kernel<<<1, kScanThreads, 0, s>>>(in, n, out, total);
    return check_launch("scan_exclusive_i64");
  }
  scan_reduce_kernel<<<nb, kScanThreads, 0, s>>>(in, n, sums);
  scan_blocks_kernel<<<1, kScanThreads, 0, s>>>(sums, nb, total);
  scan_apply_kernel<<<nb, kScanThreads, 0, s>>>(in, n, sums, out);
  return check_launch("scan_exclusive_i64");
}

int scan_small_inplace(int64_t* data, int64_t n, int64_t* total, hipStream_t s) {
  scan_blocks_kernel<<<1, kScanThreads, 0, s>>>(data, n, total);
  return check_launch("scan_small_inplace");
}

}  // namespace msp

extern "C" {

int msp_abi_version(void) { return 8; }

const char* msp_last_error(void) { return msp::g_err; }

size_t msp_scan_workspace_size(int64_t n) { return msp::scan_ws_bytes(n); }

}  // extern "C"
