// Fused encoder tail for training:
//
//   OutputLayer -> SparseConvBase_.postProcessing
//   (models/SparseConvNet.py:20-26: per-scene torch.mean over the point rows
//    [batch_offsets[b], batch_offsets[b+1]) of the per-point features)
//
// computed straight from the level-0 voxel rows, without materialising the
// (N, C) per-point tensor:
//
//   out[b] = (1 / n_b) * sum over voxels v of scene b of cnt_v * feat[v]
//
// where cnt_v = vstart[v+1] - vstart[v] is the number of points in voxel v
// (every point of v carries feat[v] after the OutputLayer) and n_b the points
// of scene b.  Voxel rows are sorted by Morton key with the batch index in
// the high bits, so each scene is one contiguous voxel range.  The reduction
// is two-stage and fixed-order (pieces of kPiece rows inside one scene, then
// the pieces of a scene in order): bitwise reproducible.
//
// Backward: dfeat[v] = cnt_v / n_b(v) * dout[b(v)].
#include "msp_common.h"

namespace msp {

constexpr int kTT = 256;
constexpr int kPiece = 1024;  // voxel rows per stage-1 block

// vscene[b] = first voxel row of scene b (b in [0, B]), from the sorted keys
__global__ __launch_bounds__(kTT) void scene_ranges_kernel(const uint64_t* __restrict__ keys, int64_t V, int shift,
                                                           int B, int64_t* __restrict__ vscene) {
  const int64_t v = (int64_t)blockIdx.x * kTT + threadIdx.x;
  if (v > V) return;
  const int64_t bv = v < V ? (int64_t)(keys[v] >> shift) : (int64_t)B;
  const int64_t bp = v > 0 ? (int64_t)(keys[v - 1] >> shift) : -1;
  const int64_t hi = bv < B ? bv : B;
  for (int64_t b = bp + 1; b <= hi; ++b) vscene[b] = v;
}

// pstart[b] = first stage-1 piece of scene b (pstart[B] = number of pieces);
// npts[b] = points of scene b (from the voxel point runs)
__global__ __launch_bounds__(kTT) void scene_pieces_kernel(const int64_t* __restrict__ vscene,
                                                           const int32_t* __restrict__ vstart, int B,
                                                           int64_t* __restrict__ pstart, int64_t* __restrict__ npts) {
  if (threadIdx.x != 0) return;
  int64_t acc = 0;
  for (int b = 0; b < B; ++b) {
    pstart[b] = acc;
    const int64_t v0 = vscene[b], v1 = vscene[b + 1];
    acc += (v1 - v0 + kPiece - 1) / kPiece;
    npts[b] = (int64_t)vstart[v1] - (int64_t)vstart[v0];
  }
  pstart[B] = acc;
}

// stage 1: block p sums cnt_v * feat[v] over its piece's rows; thread layout
// rows-in-parallel x channels (C <= 256), or all threads on channels with the
// rows sequential (C > 256, up to 4 channels per thread)
__global__ __launch_bounds__(kTT) void scene_partial_kernel(const float* __restrict__ f, int C,
                                                            const int32_t* __restrict__ vstart,
                                                            const int64_t* __restrict__ vscene,
                                                            const int64_t* __restrict__ pstart, int B,
                                                            float* __restrict__ partial) {
  __shared__ float red[kTT];
  const int64_t p = blockIdx.x;
  if (p >= pstart[B]) return;  // the grid is sized for the worst case
  int lo = 0, hi = B;          // scene b with pstart[b] <= p < pstart[b+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pstart[mid] <= p) lo = mid;
    else hi = mid;
  }
  const int b = lo;
  const int64_t r0 = vscene[b] + (p - pstart[b]) * kPiece;
  const int64_t r1 = min(r0 + kPiece, vscene[b + 1]);
  const int t = threadIdx.x;
  float* dst = partial + p * (int64_t)C;
  if (C <= kTT) {
    const int RG = kTT / C, g = t / C, c = t % C;
    float s = 0.f;
    if (g < RG) {
      for (int64_t v = r0 + g; v < r1; v += RG) s += (float)(vstart[v + 1] - vstart[v]) * f[v * C + c];
    }
    red[t] = s;
    __syncthreads();
    if (t < C) {
      float acc = 0.f;
      for (int k = 0; k < RG; ++k) acc += red[k * C + t];
      dst[t] = acc;
    }
  } else {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t v = r0; v < r1; ++v) {
      const float w = (float)(vstart[v + 1] - vstart[v]);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (t + k * kTT < C) s[k] += w * f[v * C + t + k * kTT];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (t + k * kTT < C) dst[t + k * kTT] = s[k];
  }
}

// stage 2: out[b][c] = (sum of scene b's pieces, in order) / n_b
__global__ __launch_bounds__(kTT) void scene_final_kernel(const float* __restrict__ partial, int C,
                                                          const int64_t* __restrict__ pstart,
                                                          const int64_t* __restrict__ npts, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * kTT + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int64_t p = pstart[b]; p < pstart[b + 1]; ++p) s += partial[p * C + c];
  const int64_t n = npts[b];
  out[(int64_t)b * C + c] = n > 0 ? s / (float)n : 0.f;
}

__global__ __launch_bounds__(kTT) void scene_mean_bwd_kernel(const float* __restrict__ dout, int C,
                                                             const uint64_t* __restrict__ keys, int64_t V, int shift,
                                                             const int32_t* __restrict__ vstart,
                                                             const int64_t* __restrict__ npts,
                                                             float* __restrict__ df) {
  const int64_t n = V * C;
  for (int64_t e = (int64_t)blockIdx.x * kTT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kTT) {
    const int64_t v = e / C;
    const int c = (int)(e % C);
    const int64_t b = (int64_t)(keys[v] >> shift);
    const float w = (float)(vstart[v + 1] - vstart[v]) / (float)npts[b];
    df[e] = w * dout[b * C + c];
  }
}

inline int64_t n_pieces_bound(int64_t V, int B) { return (V + kPiece - 1) / kPiece + B; }

// ---------------------------------------------------------------- eval tail
// Per-point logits of the head's Linear (models/MultiLabelContrastive.py:43-45, 84-101; train.py:106):
// the Linear commutes with the OutputLayer's gather, so it runs on the level-0 voxel rows ((V, C) -> (V, ld)
// on msp_nin_gemm) and each point gathers C_out columns of its voxel's row plus the bias.  Thread per output
// element: the (N, C_out) writes are coalesced, the gathered rows hit L2 (points of a voxel are adjacent).
__global__ __launch_bounds__(kTT) void point_rows_bias_kernel(const float* __restrict__ in, int64_t ld, int C,
                                                              const float* __restrict__ bias,
                                                              const int32_t* __restrict__ p2v, int64_t n,
                                                              float* __restrict__ out) {
  const int64_t total = n * C;
  for (int64_t e = (int64_t)blockIdx.x * kTT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kTT) {
    const int64_t p = e / C;
    const int c = (int)(e - p * C);
    const float v = in[(int64_t)p2v[p] * ld + c];
    out[e] = bias ? v + bias[c] : v;
  }
}

// index_add_ along rows (train.py:107 `store.index_add_(0, point_ids, predictions)`), deterministic and
// bit-equal to the serial CPU loop (for i in order: store[ids[i]] += src[i]): the (id, i) pairs are
// radix sorted stably by id, so each id's rows form one run in ascending i; the thread at a run's first
// position adds the run's rows into the stored value in that order.  Ids outside [0, n_store) carry the key
// n_store and are skipped (the caller validates them).
__global__ __launch_bounds__(kTT) void index_keys_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t n_store,
                                                         uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * kTT + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  keys[i] = (id >= 0 && id < n_store) ? (uint64_t)id : (uint64_t)n_store;
  vals[i] = (int32_t)i;
}

__global__ __launch_bounds__(kTT) void index_add_runs_kernel(float* __restrict__ store, int64_t n_store, int C,
                                                             const uint64_t* __restrict__ keys,
                                                             const int32_t* __restrict__ vals, int64_t n,
                                                             const float* __restrict__ src) {
  const int64_t total = n * C;
  for (int64_t e = (int64_t)blockIdx.x * kTT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kTT) {
    const int64_t j = e / C;
    const int c = (int)(e - j * C);
    const uint64_t k = keys[j];
    if (k >= (uint64_t)n_store || (j > 0 && keys[j - 1] == k)) continue;
    float s = store[(int64_t)k * C + c];
    for (int64_t q = j; q < n && keys[q] == k; ++q) s += src[(int64_t)vals[q] * C + c];
    store[(int64_t)k * C + c] = s;
  }
}

inline unsigned tail_grid(int64_t total) {
  int64_t g = ceil_div(total > 0 ? total : 1, kTT);
  if (g > 65535 * 16) g = 65535 * 16;
  return (unsigned)g;
}

inline int id_bits(int64_t n_store) {
  int b = 1;
  while (b < 63 && (n_store >> b) != 0) ++b;
  return b;
}

inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace msp

using namespace msp;

extern "C" {

size_t msp_scene_mean_workspace_size(int64_t V, int B, int C) {
  return (size_t)(B + 1) * sizeof(int64_t) + (size_t)n_pieces_bound(V, B) * (size_t)C * sizeof(float);
}

int msp_scene_mean_fwd(const float* feats, int C, const uint64_t* keys, int64_t V, int shift,
                       const int32_t* vstart, int B, int64_t* vscene, int64_t* npts, float* out, void* ws,
                       size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && C <= 4 * kTT && B >= 1 && V >= 0 && shift >= 0 && shift < 64,
              "msp_scene_mean_fwd: bad arguments (C=%d B=%d V=%lld)", C, B, (long long)V);
  MSP_REQUIRE(ws_bytes >= msp_scene_mean_workspace_size(V, B, C), "msp_scene_mean_fwd: workspace too small");
  hipStream_t s = as_stream(stream);
  int64_t* pstart = static_cast<int64_t*>(ws);
  float* partial = reinterpret_cast<float*>(pstart + B + 1);
  scene_ranges_kernel<<<(unsigned)ceil_div(V + 1, kTT), kTT, 0, s>>>(keys, V, shift, B, vscene);
  scene_pieces_kernel<<<1, 64, 0, s>>>(vscene, vstart, B, pstart, npts);
  scene_partial_kernel<<<(unsigned)n_pieces_bound(V, B), kTT, 0, s>>>(feats, C, vstart, vscene, pstart, B, partial);
  scene_final_kernel<<<dim3((unsigned)ceil_div(C, kTT), (unsigned)B), kTT, 0, s>>>(partial, C, pstart, npts, out);
  return check_launch("msp_scene_mean_fwd");
}

int msp_scene_mean_bwd(const float* dout, int C, const uint64_t* keys, int64_t V, int shift, const int32_t* vstart,
                       const int64_t* npts, float* dfeats, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && V >= 0, "msp_scene_mean_bwd: bad arguments");
  if (V == 0) return MSP_OK;
  int64_t g = ceil_div(V * C, kTT);
  if (g > 65535 * 16) g = 65535 * 16;
  scene_mean_bwd_kernel<<<(unsigned)g, kTT, 0, as_stream(stream)>>>(dout, C, keys, V, shift, vstart, npts, dfeats);
  return check_launch("msp_scene_mean_bwd");
}

int msp_point_rows_bias(const float* in, int64_t ld, int C, const float* bias, const int32_t* p2v, int64_t n_points,
                        float* out, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && ld >= C && n_points >= 0, "msp_point_rows_bias: bad arguments (C=%d ld=%lld)", C,
              (long long)ld);
  if (n_points == 0) return MSP_OK;
  MSP_REQUIRE(in && p2v && out, "msp_point_rows_bias: NULL pointer");
  point_rows_bias_kernel<<<tail_grid(n_points * C), kTT, 0, as_stream(stream)>>>(in, ld, C, bias, p2v, n_points,
                                                                                 out);
  return check_launch("msp_point_rows_bias");
}

size_t msp_index_add_workspace_size(int64_t n, int64_t n_store) {
  if (n <= 0) return 0;
  return 2 * al256((size_t)n * 8) + 2 * al256((size_t)n * 4) + al256(msp_sort_workspace_size(n, id_bits(n_store)));
}

int msp_index_add_rows(float* store, int64_t n_store, int C, const int64_t* ids, const float* src, int64_t n,
                       void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(C > 0 && n >= 0 && n_store >= 0 && n < (1ll << 31), "msp_index_add_rows: bad arguments");
  if (n == 0 || n_store == 0) return MSP_OK;
  const size_t need = msp_index_add_workspace_size(n, n_store);
  MSP_REQUIRE(ws && ws_bytes >= need, "msp_index_add_rows: workspace too small (%zu < %zu)", ws_bytes, need);
  hipStream_t s = as_stream(stream);
  char* w = static_cast<char*>(ws);
  uint64_t* k_in = reinterpret_cast<uint64_t*>(w);
  uint64_t* k_out = reinterpret_cast<uint64_t*>(w + al256((size_t)n * 8));
  int32_t* v_in = reinterpret_cast<int32_t*>(w + 2 * al256((size_t)n * 8));
  int32_t* v_out = reinterpret_cast<int32_t*>(w + 2 * al256((size_t)n * 8) + al256((size_t)n * 4));
  void* sws = w + 2 * al256((size_t)n * 8) + 2 * al256((size_t)n * 4);
  const int bits = id_bits(n_store);
  index_keys_kernel<<<(unsigned)ceil_div(n, kTT), kTT, 0, s>>>(ids, n, n_store, k_in, v_in);
  int rc = msp_sort_pairs(k_in, k_out, v_in, v_out, n, bits, sws, msp_sort_workspace_size(n, bits), stream);
  if (rc) return rc;
  index_add_runs_kernel<<<tail_grid(n * C), kTT, 0, s>>>(store, n_store, C, k_out, v_out, n, src);
  return check_launch("msp_index_add_rows");
}

}  // extern "C"
