// Batch assembly on the device: the geometric part
// of the reference's DataLoader collate functions
//
//   trainMerge  dataset/data.py:135-238  (random scale/flip/rotation, random
//               offset into [0, full_scale)^3, crop, .long(), batch id in the
//               last column, per-scene colour shift, batch_offsets)
//   valMerge    dataset/data.py:256-310  (same with a centred placement and
//               per-point ids of the kept points)
//
// for B scenes whose raw points are already in HBM.  The random draws are
// data-independent and stay on the host (same numpy draw order as the
// restatement in wsss3d/synthetic.py); everything per point runs here.
//
// Arithmetic follows the numpy restatement operation by operation in fp64
// (no contraction into FMAs): t = ((a0*r0j + a1*r1j) + a2*r2j) + c1j + c2j,
// per-scene min/max of t, the offset formula of the mode, p = t + offset,
// keep = 0 <= p < full_scale, coordinate = trunc(p).  min/max are exact, so
// the atomic combination is order-independent; the compaction keeps the
// point order (block prefix sums), so the output is deterministic.
#include "msp_common.h"

#include <climits>

#pragma clang fp contract(off)

namespace msp {

constexpr int kMT = 256;
constexpr int kMIt = 4;  // points per thread
constexpr int kMPB = kMT * kMIt;

struct MergeParams {
  const double* rot;   // [B][9]  row-major 3x3 (points are row vectors: t = a . rot)
  const double* c1;    // [B][3]
  const double* c2;    // [B][3]
  const double* u1;    // [B][3]  the two rand(3) draws of the offset
  const double* u2;    // [B][3]
  const float* shift;  // [B][3]  colour shift
};

// order-preserving map of doubles onto int64 (for atomic min / max)
__device__ inline long long ord_of(double d) {
  long long i = __double_as_longlong(d);
  return i >= 0 ? i : (i ^ 0x7fffffffffffffffll);
}
__host__ __device__ inline double dbl_of(long long i) {
  const long long j = i >= 0 ? i : (i ^ 0x7fffffffffffffffll);
#ifdef __HIP_DEVICE_COMPILE__
  return __longlong_as_double(j);
#else
  double d;
  __builtin_memcpy(&d, &j, sizeof d);
  return d;
#endif
}

__device__ inline void transform(const float* __restrict__ xyz, int64_t i, const double* r, const double* c1,
                                 const double* c2, double (&t)[3]) {
  const double a0 = (double)xyz[3 * i], a1 = (double)xyz[3 * i + 1], a2 = (double)xyz[3 * i + 2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    double v = __dadd_rn(__dadd_rn(__dmul_rn(a0, r[j]), __dmul_rn(a1, r[3 + j])), __dmul_rn(a2, r[6 + j]));
    v = __dadd_rn(v, c1[j]);
    t[j] = __dadd_rn(v, c2[j]);
  }
}

__global__ __launch_bounds__(kMT) void merge_minmax_kernel(const float* __restrict__ xyz,
                                                           const int64_t* __restrict__ sstart, MergeParams P,
                                                           long long* __restrict__ mm /*[B][6]*/) {
  __shared__ long long red[6][kMT / 64];
  const int b = blockIdx.y;
  const int64_t s0 = sstart[b], s1 = sstart[b + 1];
  long long lo[3] = {LLONG_MAX, LLONG_MAX, LLONG_MAX}, hi[3] = {LLONG_MIN, LLONG_MIN, LLONG_MIN};
  for (int k = 0; k < kMIt; ++k) {
    const int64_t i = s0 + (int64_t)blockIdx.x * kMPB + k * kMT + threadIdx.x;
    if (i < s1) {
      double t[3];
      transform(xyz, i, P.rot + 9 * b, P.c1 + 3 * b, P.c2 + 3 * b, t);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        lo[j] = min(lo[j], ord_of(t[j]));
        hi[j] = max(hi[j], ord_of(t[j]));
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      lo[j] = min(lo[j], (long long)__shfl_xor(lo[j], d, 64));
      hi[j] = max(hi[j], (long long)__shfl_xor(hi[j], d, 64));
    }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int j = 0; j < 3; ++j) {
      red[j][wave] = lo[j];
      red[3 + j][wave] = hi[j];
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int j = threadIdx.x;
    long long v = red[j][0];
    for (int w = 1; w < kMT / 64; ++w) v = j < 3 ? min(v, red[j][w]) : max(v, red[j][w]);
    if (j < 3) atomicMin(&mm[6 * b + j], v);
    else atomicMax(&mm[6 * b + j], v);
  }
}

// offset[b] per the mode's formula (numpy evaluation order)
//   train (data.py:176-178): -m + clip(fs - (M - m) - 0.001, 0) * u1 + clip(fs - (M - m) + 0.001, None, 0) * u2
//   val   (data.py:273-275): -m + clip(fs - M + m - 0.001, 0) * u1 + clip(fs - M + m + 0.001, None, 0) * u2
__global__ void merge_offset_kernel(const long long* __restrict__ mm, int B, double fs, int mode, MergeParams P,
                                    double* __restrict__ offset) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 3 * B) return;
  const int b = e / 3, j = e % 3;
  const double m = dbl_of(mm[6 * b + j]), M = dbl_of(mm[6 * b + 3 + j]);
  double q1, q2;
  if (mode == 0) {
    const double len = __dadd_rn(M, -m);
    q1 = __dadd_rn(__dadd_rn(fs, -len), -0.001);
    q2 = __dadd_rn(__dadd_rn(fs, -len), 0.001);
  } else {
    const double g = __dadd_rn(__dadd_rn(fs, -M), m);
    q1 = __dadd_rn(g, -0.001);
    q2 = __dadd_rn(g, 0.001);
  }
  q1 = q1 > 0.0 ? q1 : 0.0;
  q2 = q2 < 0.0 ? q2 : 0.0;
  offset[e] = __dadd_rn(__dadd_rn(-m, __dmul_rn(q1, P.u1[e])), __dmul_rn(q2, P.u2[e]));
}

__device__ inline bool kept(const float* __restrict__ xyz, int64_t i, int b, const MergeParams& P,
                            const double* __restrict__ offset, double fs, double (&p)[3]) {
  double t[3];
  transform(xyz, i, P.rot + 9 * b, P.c1 + 3 * b, P.c2 + 3 * b, t);
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    p[j] = __dadd_rn(t[j], offset[3 * b + j]);
    ok = ok && p[j] >= 0.0 && p[j] < fs;
  }
  return ok;
}

// counts[b * nbx + bx] = kept points of block (b, bx)
__global__ __launch_bounds__(kMT) void merge_count_kernel(const float* __restrict__ xyz,
                                                          const int64_t* __restrict__ sstart, MergeParams P,
                                                          const double* __restrict__ offset, double fs,
                                                          int64_t* __restrict__ counts) {
  const int b = blockIdx.y;
  const int64_t s0 = sstart[b], s1 = sstart[b + 1];
  int64_t c = 0;
  for (int k = 0; k < kMIt; ++k) {
    const int64_t i = s0 + (int64_t)blockIdx.x * kMPB + k * kMT + threadIdx.x;
    double p[3];
    if (i < s1 && kept(xyz, i, b, P, offset, fs, p)) ++c;
  }
  int64_t tot;
  block_excl_scan<kMT>(c, &tot);
  if (threadIdx.x == 0) counts[(int64_t)b * gridDim.x + blockIdx.x] = tot;
}

// stable compaction: output position = block start + prefix of the kept
// points in point order (thread-major inside each of the kMIt sweeps)
__global__ __launch_bounds__(kMT) void merge_write_kernel(const float* __restrict__ xyz,
                                                          const float* __restrict__ rgb,
                                                          const int64_t* __restrict__ lab_in,
                                                          const int64_t* __restrict__ sstart, MergeParams P,
                                                          const double* __restrict__ offset, double fs,
                                                          const int64_t* __restrict__ starts,
                                                          int64_t* __restrict__ coords, float* __restrict__ feats,
                                                          int64_t* __restrict__ lab_out, int64_t* __restrict__ ids,
                                                          int64_t id_base, unsigned* __restrict__ label_mask) {
  const int b = blockIdx.y;
  const int64_t s0 = sstart[b], s1 = sstart[b + 1];
  int64_t pos = starts[(int64_t)b * gridDim.x + blockIdx.x];
  unsigned mask = 0;
  for (int k = 0; k < kMIt; ++k) {
    const int64_t i = s0 + (int64_t)blockIdx.x * kMPB + k * kMT + threadIdx.x;
    double p[3];
    const bool keep = i < s1 && kept(xyz, i, b, P, offset, fs, p);
    int64_t tot;
    const int64_t e = pos + block_excl_scan<kMT>((int64_t)keep, &tot);
    if (keep) {
      coords[4 * e + 0] = (int64_t)p[0];  // trunc toward zero (p >= 0): torch .long()
      coords[4 * e + 1] = (int64_t)p[1];
      coords[4 * e + 2] = (int64_t)p[2];
      coords[4 * e + 3] = b;
#pragma unroll
      for (int j = 0; j < 3; ++j) feats[3 * e + j] = rgb[3 * i + j] + P.shift[3 * b + j];
      const int64_t l = lab_in[i];
      lab_out[e] = l;
      if (l >= 0 && l < 32) mask |= 1u << l;
      if (ids) ids[e] = id_base + i;
    }
    pos += tot;
  }
  // scene label presence (data.py:188-191): OR is order-independent
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mask |= (unsigned)__shfl_xor((int)mask, d, 64);
  if ((threadIdx.x & 63) == 0 && mask) atomicOr(&label_mask[b], mask);
}

__global__ void merge_init_kernel(long long* __restrict__ mm, unsigned* __restrict__ label_mask, int B) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < 6 * B) mm[e] = (e % 6) < 3 ? LLONG_MAX : LLONG_MIN;  // identities of min (lo) and max (hi)
  if (e < B) label_mask[e] = 0u;
}

__global__ void merge_finish_kernel(const int64_t* __restrict__ starts, int nbx, int B,
                                    const int64_t* __restrict__ total, const unsigned* __restrict__ label_mask,
                                    int n_classes, int64_t* __restrict__ batch_offsets,
                                    float* __restrict__ scene_labels) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e <= B) batch_offsets[e] = e < B ? starts[(int64_t)e * nbx] : *total;
  if (e < B * n_classes) {
    const int b = e / n_classes, c = e % n_classes;
    scene_labels[e] = (label_mask[b] >> c) & 1u ? 1.f : 0.f;
  }
}

}  // namespace msp

using namespace msp;

extern "C" {

size_t msp_merge_workspace_size(int B, int64_t max_scene_points) {
  const int64_t nbx = ceil_div(max_scene_points > 0 ? max_scene_points : 1, kMPB);
  const int64_t m = (int64_t)B * nbx;
  return (size_t)B * 6 * sizeof(long long) + (size_t)B * 3 * sizeof(double) + (size_t)B * sizeof(unsigned) + 8 +
         (size_t)(2 * m + 1) * sizeof(int64_t) + scan_ws_bytes(m);
}

int msp_merge(const float* xyz, const float* rgb, const int64_t* labels, const int64_t* scene_start, int B,
              int64_t max_scene_points, int mode, double full_scale, const double* rot, const double* c1,
              const double* c2, const double* u1, const double* u2, const float* shift, int n_classes,
              int64_t* coords, float* feats, int64_t* labels_out, int64_t* point_ids, int64_t point_id_base,
              int64_t* batch_offsets, float* scene_labels, void* ws, size_t ws_bytes, msp_stream_t stream) {
  MSP_REQUIRE(B >= 1 && max_scene_points >= 0 && (mode == 0 || mode == 1) && full_scale > 0 && n_classes >= 0 &&
                  n_classes <= 32,
              "msp_merge: bad arguments (B=%d mode=%d n_classes=%d)", B, mode, n_classes);
  MSP_REQUIRE(ws_bytes >= msp_merge_workspace_size(B, max_scene_points), "msp_merge: workspace too small");
  hipStream_t s = as_stream(stream);
  const int64_t nbx = ceil_div(max_scene_points > 0 ? max_scene_points : 1, kMPB);
  const int64_t m = (int64_t)B * nbx;
  char* w = static_cast<char*>(ws);
  long long* mm = reinterpret_cast<long long*>(w);
  w += (size_t)B * 6 * sizeof(long long);
  double* offset = reinterpret_cast<double*>(w);
  w += (size_t)B * 3 * sizeof(double);
  unsigned* label_mask = reinterpret_cast<unsigned*>(w);
  w += ((size_t)B * sizeof(unsigned) + 7) / 8 * 8;
  int64_t* counts = reinterpret_cast<int64_t*>(w);
  int64_t* starts = counts + m;
  int64_t* total = starts + m;
  void* sws = total + 1;
  merge_init_kernel<<<(unsigned)ceil_div(6 * B, 256), 256, 0, s>>>(mm, label_mask, B);
  MergeParams P{rot, c1, c2, u1, u2, shift};
  const dim3 grid((unsigned)nbx, (unsigned)B);
  merge_minmax_kernel<<<grid, kMT, 0, s>>>(xyz, scene_start, P, mm);
  merge_offset_kernel<<<(unsigned)ceil_div(3 * B, 64), 64, 0, s>>>(mm, B, full_scale, mode, P, offset);
  merge_count_kernel<<<grid, kMT, 0, s>>>(xyz, scene_start, P, offset, full_scale, counts);
  int rc = scan_exclusive_i64(counts, starts, m, total, sws, scan_ws_bytes(m), s);
  if (rc) return rc;
  merge_write_kernel<<<grid, kMT, 0, s>>>(xyz, rgb, labels, scene_start, P, offset, full_scale, starts, coords, feats,
                                          labels_out, point_ids, point_id_base, label_mask);
  const int nf = (B + 1) > B * n_classes ? B + 1 : B * n_classes;
  merge_finish_kernel<<<(unsigned)ceil_div(nf, 256), 256, 0, s>>>(starts, (int)nbx, B, total, label_mask,
                                                                  n_classes, batch_offsets, scene_labels);
  return check_launch("msp_merge");
}

}  // extern "C"
