// NetworkInNetwork dense products (scn.NetworkInNetwork,
// the 2a -> a shortcut of the UNet decoder's first residual block):
//   forward        out[V][c_out] = x[V][c_in] W[c_in][c_out]
//   backward-data  dx[V][c_in]   = dy[V][c_out] W^T
// both as C[M][N] = A[M][K] B[K][N], row-major fp32.  These are tall-skinny
// (M ~ 10^6, K, N <= a few hundred), so the bound is HBM: one read of A, one
// write of C, B (<= 256 KiB) served from L1/L2.  The library GEMMs picked for
// these shapes ran at 2.5-4x the HBM floor (scripts/kbench_nin.py).
//
// Persistent waves (first cut staged A tiles in LDS and read B fragments
// from global per k-step: 1.0-3x of hipBLASLt's time, the B loads exposed).
// A block stages its column chunk of B (K x 16 NTT, row stride 16 NTT + 4:
// the four lane groups q land 16 banks apart) in LDS once; then each wave
// walks 16-row groups g = wave_id, wave_id + n_waves, ... on its own (no
// further barriers).  The contraction index is permuted inside each 16-deep
// k-block so A loads are float4: lane (r, q) loads A[16 g + r][k0 + 4q ..
// 4q + 3] and k-step s of the block uses component s with
// B[k0 + 4q + s][16 t + r] (any k order is the same sum of exact products;
// the k-blocks are accumulated in order).  A runs one k-block ahead in
// registers across group boundaries; rows past M are clamped on load and
// not stored.  f32 MFMA 16x16x4: lane holds C[16 g + 4q + j][n0 + 16 t + r].
// Measured (scripts/kbench_nin.py, profiles/r01/kbench_nin_r01.log): L0/L1
// forward and backward-data 108-122 us against 130-204 us for hipBLASLt
// (4.4-5.1 TB/s at L0); below ~2.6e5 rows the per-block B staging dominates
// and the library GEMM is faster, so ops.nin_gemm routes those shapes there
// (msp_nin_gemm_preferred).  A variant that loads a whole row group ahead
// (KC float4 per lane, two register sets) measured the same.
#include "msp_common.h"

namespace msp {

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NTT>
__global__ __launch_bounds__(256) void nin_gemm_kernel(const float* __restrict__ A, int64_t M, int K,
                                                       const float* __restrict__ B, int N, int n_chunks,
                                                       float* __restrict__ C) {
  extern __shared__ float sb[];  // [K][16 NTT + 4]
  constexpr int NB = 16 * NTT, LDB = NB + 4;
  const int ch = (int)(blockIdx.x % n_chunks);
  const int64_t blk = blockIdx.x / n_chunks, n_blk = gridDim.x / n_chunks;
  const int n0 = ch * NB;
  for (int u = threadIdx.x; u < K * (NB / 4); u += 256) {
    const int k = u / (NB / 4), c4 = u - k * (NB / 4);
    *reinterpret_cast<float4*>(&sb[k * LDB + 4 * c4]) =
        *reinterpret_cast<const float4*>(B + (int64_t)k * N + n0 + 4 * c4);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int64_t G = (M + 15) / 16;
  const int64_t g0 = blk * 4 + wave, gs = n_blk * 4;
  if (g0 >= G) return;  // wave-uniform; no barrier follows
  const int KC = K >> 4;
  auto ld_a = [&](int64_t g, int kc) {
    int64_t row = g * 16 + r;
    row = row < M ? row : M - 1;
    return *reinterpret_cast<const float4*>(A + row * K + 16 * kc + 4 * q);
  };
  const float* bq = sb + 4 * q * LDB + r;
  int64_t g = g0;
  int kc = 0;
  float4 cur = ld_a(g, 0);
  floatx4 acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  while (true) {
    // the next (group, k-block) in this wave's walk, loaded before the MFMAs of the current one
    int64_t gn = g;
    int kn = kc + 1;
    if (kn == KC) {
      kn = 0;
      gn = g + gs;
    }
    const float4 nxt = ld_a(gn < G ? gn : g, kn);
    const float av[4] = {cur.x, cur.y, cur.z, cur.w};
    const float* bk = bq + 16 * kc * LDB;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int t = 0; t < NTT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bk[s * LDB + 16 * t], acc[t], 0, 0, 0);
    }
    if (kn == 0) {  // group done: store its 16 rows
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t row = g * 16 + 4 * q + j;
        if (row < M) {
#pragma unroll
          for (int t = 0; t < NTT; ++t) C[row * N + n0 + 16 * t + r] = acc[t][j];
        }
      }
#pragma unroll
      for (int t = 0; t < NTT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (gn >= G) break;
    }
    g = gn;
    kc = kn;
    cur = nxt;
  }
}

namespace {

constexpr size_t kNinLds = 80 * 1024;

size_t nin_lds(int K, int ntt) { return (size_t)K * (16 * ntt + 4) * sizeof(float); }

int nin_ntt(int K, int N) {  // largest column-tile count <= 8 dividing N / 16 whose B chunk fits the LDS budget
  const int n16 = N / 16;
  for (int d = 8; d >= 1; --d)
    if (n16 % d == 0 && nin_lds(K, d) <= kNinLds) return d;
  return 0;
}

template <int NTT>
int launch_nin(const float* A, int64_t M, int K, const float* B, int N, float* C, hipStream_t s) {
  static bool attr_set = false;  // dynamic LDS above the 64 KiB default
  if (!attr_set) {
    MSP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&nin_gemm_kernel<NTT>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNinLds),
            "msp_nin_gemm: LDS attribute");
    attr_set = true;
  }
  const size_t lds = nin_lds(K, NTT);
  const int n_chunks = N / (16 * NTT);
  const int64_t groups = (M + 15) / 16;
  int64_t blocks = (groups + 3) / 4;
  const int64_t cap = 256 * (lds > 40 * 1024 ? 2 : 4);  // resident blocks per launch (256 CUs)
  if (blocks > cap) blocks = cap;
  const unsigned grid = (unsigned)(blocks * n_chunks);
  nin_gemm_kernel<NTT><<<grid, 256, lds, s>>>(A, M, K, B, N, n_chunks, C);
  return check_launch("msp_nin_gemm");
}

}  // namespace
}  // namespace msp

using namespace msp;

extern "C" {

int msp_nin_gemm_ok(int64_t M, int K, int N) {
  return M >= 0 && K >= 16 && K % 16 == 0 && N >= 16 && N % 16 == 0 && nin_ntt(K, N) > 0 ? 1 : 0;
}

int msp_nin_gemm_preferred(int64_t M, int K, int N) { return msp_nin_gemm_ok(M, K, N) && M >= (1 << 18) ? 1 : 0; }

int msp_nin_gemm(const float* A, int64_t M, int K, const float* B, int N, float* C, msp_stream_t stream) {
  MSP_REQUIRE(msp_nin_gemm_ok(M, K, N), "msp_nin_gemm: needs K %% 16 == 0, N %% 16 == 0 and a 16 x K slice of B within 80 KiB (M=%lld K=%d N=%d)",
              (long long)M, K, N);
  MSP_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0, "msp_nin_gemm: A and B must be 16-byte aligned");
  if (M == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
#define NL(T) \
  if (nin_ntt(K, N) == T) return launch_nin<T>(A, M, K, B, N, C, s);
  NL(1) NL(2) NL(3) NL(4) NL(5) NL(6) NL(7) NL(8)
#undef NL
  return MSP_EINVAL;
}

}  // extern "C"
