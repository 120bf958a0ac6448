// NetworkInNetwork dense products (scn.NetworkInNetwork,
// the 2a -> a shortcut of the UNet decoder's first residual block):
//   forward        out[V][c_out] = x[V][c_in] W[c_in][c_out]
//   backward-data  dx[V][c_in]   = dy[V][c_out] W^T
// both as C[M][N] = A[M][K] B[K][N], row-major fp32.  These are tall-skinny
// (M ~ 10^4 .. 10^6, K, N <= a few hundred): one read of A and one write of C
// bound them, B (<= 0.8 MiB) is served from L2.
//
// Round 3: the products run on bf16 MFMA over exact three-piece splits of
// both operands (the "x6" form of msp_conv_x6.hip, fp32-class error) instead
// of the fp32 MFMA (157 TF/s, 2.6x below the split form's 416.7 TF/s
// fp32-equivalent, which left the 2a -> a shapes at levels 1-3 compute-bound
// and the library GEMM the faster choice below 2^18 rows).  B is split once
// per call into a lane-ordered fragment image (nin_split_kernel); persistent
// blocks of 4 waves copy their 16 NT-column slice of it into LDS once and walk
// 32-row groups of A, splitting each 32-deep k-slice in registers (the next
// slice's A loads in flight) and issuing 2 x 6 NT MFMAs per slice.  From 2^18
// rows the round-1 fp32-MFMA kernel stays: it streams those shapes at 4.4-5.1
// TB/s, where the split form measured 2-22 % slower (scripts/kbench_nin.py,
// profiles/r03/kbench_nin_r03j.log); below, the split form runs level 2's
// 192 -> 96 in 69 us against 83 us (fp32 MFMA) and 66 us (hipBLASLt, which
// the product no longer calls).
#include "msp_x6.h"

namespace msp {

// B[K][N] -> fragment image: unit (((cy * nks + ks) * NT + t) * 3 + p) * 64 + lane, lane = 16 q + r, holds
// piece p of B[32 ks + 8 q .. + 7][16 (cy NT + t) + r] (zero past K)
__global__ __launch_bounds__(256) void nin_split_kernel(const float* __restrict__ B, int K, int N, int NT,
                                                        u32x4* __restrict__ img) {
  const int nks = (K + 31) / 32, n_y = N / (16 * NT);
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (int64_t)n_y * nks * NT * 64) return;
  const int lane = (int)(g & 63), r = lane & 15, q = lane >> 4;
  int64_t rest = g >> 6;
  const int t = (int)(rest % NT);
  rest /= NT;
  const int ks = (int)(rest % nks);
  const int cy = (int)(rest / nks);
  const int n = 16 * (cy * NT + t) + r, k = 32 * ks + 8 * q;
  floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  if (k < K) {  // K % 16 == 0: an octet is all data or all padding
    const float* src = B + (int64_t)k * N + n;
    a = floatx4{src[0], src[N], src[2 * N], src[3 * N]};
    b = floatx4{src[4 * N], src[5 * N], src[6 * N], src[7 * N]};
  }
  u32x4 pc[3];
  split8(a, b, pc);
  u32x4* dst = img + (g >> 6) * 3 * 64 + lane;
#pragma unroll
  for (int p = 0; p < 3; ++p) dst[p * 64] = pc[p];
}

// fp32-MFMA form (round 1), kept for the >= 2^18-row shapes where it streams A closer to the HBM rate: a
// block stages its column chunk of B (K x 16 NTT, row stride 16 NTT + 4) in LDS once and each wave walks 16-row
// groups with the contraction index permuted inside each 16-deep k-block so A loads are float4 (lane (r, q)
// loads A[16 g + r][k0 + 4q .. 4q + 3], k-step s uses component s); A runs one k-block ahead.  f32 MFMA
// 16x16x4: lane holds C[16 g + 4q + j][n0 + 16 t + r].
template <int NTT>
__global__ __launch_bounds__(256) void nin_f32_kernel(const float* __restrict__ A, int64_t M, int K,
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

// Persistent: a block copies its column slice's image (nks x NT x 3 KiB) into LDS once, then its waves walk
// 32-row groups g = block * 4 + wave, + 4 n_blk, ...; each (group, k-slice) step has the next step's A rows in
// flight (across group boundaries) while it splits the current ones and issues 2 x 6 NT MFMAs.
template <int NT>
__global__ __launch_bounds__(256) void nin_x6_kernel(const float* __restrict__ A, int64_t M, int K,
                                                     const u32x4* __restrict__ img, int N, int n_y,
                                                     float* __restrict__ C) {
  extern __shared__ u32x4 wl[];
  const int nks = (K + 31) / 32;
  const int cy = (int)(blockIdx.x % n_y);
  const int64_t blk = blockIdx.x / n_y, n_blk = gridDim.x / n_y;
  {
    const int units = nks * NT * 3 * 64;
    const u32x4* src = img + (int64_t)cy * units;
    for (int u = threadIdx.x; u < units; u += 256) wl[u] = src[u];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int64_t G = (M + 31) / 32, gs = n_blk * 4;
  int64_t g = blk * 4 + wave;
  if (g >= G) return;  // wave-uniform; no barrier follows
  auto ld_a = [&](int64_t gg, int ks, floatx4 (&a)[2][2]) {
    const int k = 32 * ks + 8 * q;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int64_t row = gg * 32 + 16 * h + r;
      row = row < M ? row : M - 1;  // clamped loads, unstored rows
      a[h][0] = a[h][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        const floatx4* p = reinterpret_cast<const floatx4*>(A + row * K + k);
        a[h][0] = p[0];
        a[h][1] = p[1];
      }
    }
  };
  floatx4 acc[2][NT];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[h][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  int ks = 0;
  floatx4 a[2][2];
  ld_a(g, 0, a);
  while (true) {
    int64_t gn = g;
    int kn = ks + 1;
    if (kn == nks) {
      kn = 0;
      gn = g + gs;
    }
    u32x4 xp[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h) split8(a[h][0], a[h][1], xp[h]);
    ld_a(gn < G ? gn : g, kn, a);
    u32x4 w[NT][3];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) w[t][p] = wl[((ks * NT + t) * 3 + p) * 64 + lane];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      floatx4 c[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][2], xp[h][0], floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][1], xp[h][1], c[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], xp[h][2], c[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][1], xp[h][0], c[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], xp[h][1], c[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = mfma_bf16(w[t][0], xp[h][0], c[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[h][t] += c[t];
    }
    if (kn == 0) {  // group done: lane (r, q) holds C[row 32 g + 16 h + r][columns 16 t + 4 q .. + 3] of the slice
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t row = g * 32 + 16 * h + r;
        if (row < M) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
            *reinterpret_cast<floatx4*>(C + row * N + 16 * (cy * NT + t) + 4 * q) = acc[h][t];
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[h][t] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      if (gn >= G) break;
    }
    g = gn;
    ks = kn;
  }
}

namespace {
constexpr size_t kF32Lds = 80 * 1024;

size_t nin_lds(int K, int ntt) { return (size_t)K * (16 * ntt + 4) * sizeof(float); }

int nin_ntt(int K, int N) {  // largest column-tile count <= 8 dividing N / 16 whose B chunk fits the LDS budget
  const int n16 = N / 16;
  for (int d = 8; d >= 1; --d)
    if (n16 % d == 0 && nin_lds(K, d) <= kF32Lds) return d;
  return 0;
}

template <int NTT>
int launch_f32(const float* A, int64_t M, int K, const float* B, int N, float* C, hipStream_t s) {
  // dynamic LDS above the 64 KiB default, once per device
  int rc = raise_lds_limit(reinterpret_cast<const void*>(&nin_f32_kernel<NTT>), (int)kF32Lds, kLdsNinF32 + NTT - 1,
                           "msp_nin_gemm: LDS attribute");
  if (rc) return rc;
  const size_t lds = nin_lds(K, NTT);
  const int n_chunks = N / (16 * NTT);
  const int64_t groups = (M + 15) / 16;
  int64_t blocks = (groups + 3) / 4;
  const int64_t cap = 256 * (lds > 40 * 1024 ? 2 : 4);  // resident blocks per launch (256 CUs)
  if (blocks > cap) blocks = cap;
  const unsigned grid = (unsigned)(blocks * n_chunks);
  nin_f32_kernel<NTT><<<grid, 256, lds, s>>>(A, M, K, B, N, n_chunks, C);
  return check_launch("msp_nin_gemm");
}


constexpr size_t kNinLds = 96 * 1024;

inline int nin_nt(int K, int N) {  // two 16-column tiles per slice unless N is odd in 16s or the image outgrows LDS
  return N % 32 == 0 && (size_t)((K + 31) / 32) * 2 * 3 * 1024 <= kNinLds ? 2 : 1;
}

template <int NT>
int launch_nin(const float* A, int64_t M, int K, const u32x4* img, int N, float* C, hipStream_t s) {
  int rc = raise_lds_limit(reinterpret_cast<const void*>(&nin_x6_kernel<NT>), (int)kNinLds, kLdsNinX6 + NT - 1,
                           "msp_nin_gemm: LDS attribute");
  if (rc) return rc;
  const int n_y = N / (16 * NT), nks = (K + 31) / 32;
  const size_t lds = (size_t)nks * NT * 3 * 1024;
  const int64_t groups = (M + 31) / 32;
  int64_t blocks = (groups + 3) / 4;
  int64_t per_cu = (int64_t)(160 * 1024 / lds);  // resident blocks per CU by LDS, at most 4 (16 waves)
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  const int64_t cap = 256 * per_cu / n_y > 0 ? 256 * per_cu / n_y : 1;  // one resident wave of blocks
  if (blocks > cap) blocks = cap;
  nin_x6_kernel<NT><<<(unsigned)(blocks * n_y), 256, lds, s>>>(A, M, K, img, N, n_y, C);
  return check_launch("msp_nin_gemm");
}
}  // namespace

}  // namespace msp

using namespace msp;

extern "C" {

int msp_nin_gemm_ok(int64_t M, int K, int N) {
  return M >= 0 && K >= 16 && K % 16 == 0 && N >= 16 && N % 16 == 0 && (size_t)((K + 31) / 32) * 3 * 1024 <= kNinLds
             ? 1
             : 0;
}

int msp_nin_gemm_form(int64_t M, int K, int N) {
  if (!msp_nin_gemm_ok(M, K, N)) return 0;
  return M >= (1 << 18) && nin_ntt(K, N) > 0 ? 1 : 2;
}

size_t msp_nin_gemm_workspace_size(int K, int N) {
  return (size_t)(N > 0 ? N / 16 : 0) * (size_t)((K + 31) / 32) * 3 * 64 * 16;
}

int msp_nin_gemm(const float* A, int64_t M, int K, const float* B, int N, float* C, void* ws, size_t ws_bytes,
                 msp_stream_t stream) {
  MSP_REQUIRE(msp_nin_gemm_ok(M, K, N), "msp_nin_gemm: needs K %% 16 == 0 and N %% 16 == 0 (M=%lld K=%d N=%d)",
              (long long)M, K, N);
  MSP_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 && ((uintptr_t)C & 15) == 0,
              "msp_nin_gemm: A, B and C must be 16-byte aligned");
  const size_t need = msp_nin_gemm_workspace_size(K, N);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_nin_gemm: workspace too small (%zu < %zu)", ws_bytes, need);
  if (M == 0) return MSP_OK;
  hipStream_t s = as_stream(stream);
  if (msp_nin_gemm_form(M, K, N) == 1) {  // fp32 form: streams the large shapes closer to the HBM rate
#define NL(T) \
  if (nin_ntt(K, N) == T) return launch_f32<T>(A, M, K, B, N, C, s);
    NL(1) NL(2) NL(3) NL(4) NL(5) NL(6) NL(7) NL(8)
#undef NL
  }
  const int NT = nin_nt(K, N), n_y = N / (16 * NT), nks = (K + 31) / 32;
  u32x4* img = static_cast<u32x4*>(ws);
  const int64_t lanes = (int64_t)n_y * nks * NT * 64;
  nin_split_kernel<<<(unsigned)ceil_div(lanes, 256), 256, 0, s>>>(B, K, N, NT, img);
  const int rc = check_launch("msp_nin_gemm");
  if (rc) return rc;
  return NT == 2 ? launch_nin<2>(A, M, K, img, N, C, s) : launch_nin<1>(A, M, K, img, N, C, s);
}

}  // extern "C"
