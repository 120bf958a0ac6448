/*
 * mi3dsparse — C ABI of the MI355X-native sparse 3D convolution library.
 *
 * This header is the drop-in boundary that replaces SparseConvNet's pybind11
 * extension `sparseconvnet.SCN` (SCN 0.2 dev, `requirements.txt:2`,
 * `env_list.txt:246`; not vendored under the reference) for the calls that the
 * reference's encoders make through the `scn.*` module API
 * (`models/SparseConvNet.py:57-229`).  The Python namespace
 * `sparseconvnet` shipped with this library binds these symbols with ctypes;
 * INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain pointers + sizes.  All pointers are device pointers unless a
 *     parameter is documented as host.  Integer maps are int32, keys uint64,
 *     features float32 row-major [rows][channels].
 *   - All buffers, including workspaces, are allocated by the caller; sizes are
 *     queried with the *_workspace_size functions.  The library never
 *     allocates or frees device memory and holds no global device state.
 *   - Every kernel is enqueued on the caller's stream; no entry point
 *     synchronises the device.  Counts the caller needs on the host are written
 *     to small device buffers that the caller copies back.
 *   - Return 0 on success, a negative MSP_E* code on failure; the message is
 *     thread-local and read with msp_last_error().
 *   - Stateless and reentrant: no entry point reads or writes process-global
 *     state beyond two per-device caches -- each device's CU count and which
 *     kernels have had their dynamic-LDS limit raised on it -- held in atomics
 *     indexed by device id (safe from several threads and on several devices);
 *     every exported symbol is declared here (tests/test_abi.py checks the .so's
 *     dynamic symbol table against this header).
 *   - Offset-major maps: a neighbour / child map with K filter offsets over n
 *     rows is stored [K][n] (entry -1 = absent).  Filter offsets follow SCN's
 *     last-axis-fastest order: o = ((dx*f) + dy)*f + dz over the f^3 box.
 */
#ifndef MI3DSPARSE_H
#define MI3DSPARSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* msp_stream_t; /* hipStream_t */

#define MSP_OK 0
#define MSP_EINVAL (-1)
#define MSP_EHIP (-2)
#define MSP_ENOSPACE (-3)

#define MSP_TILE_ROWS 64 /* rows of a per-wave tile (tile_rows = 64)         */
#define MSP_CHUNK 16     /* rows per MFMA chunk in rulebooks                  */

int msp_abi_version(void);
const char* msp_last_error(void);

/* ---------------- metadata: voxel indexing (replaces SCN InputLayer rules,
 * `scn.InputLayer(3, full_scale, mode=4)`, models/SparseConvNet.py:61,77,94,147,200;
 * modes documented at Function_test.py:35-44) ------------------------------ */

/* coords: n rows of `row_stride` int64, [x, y, z, batch] (batch column last,
 * dataset/data.py:198).  Writes Morton keys and vals[i] = i.  stats[0] =
 * number of rows outside [0, spatial_size)^3 or with negative batch id,
 * stats[1] = max batch id, stats[2] = number of rows whose batch id is below
 * the previous row's (0: batch column non-decreasing).  stats[3] must be
 * zeroed by the caller. */
int msp_point_keys(const int64_t* coords, int64_t n, int64_t row_stride, int log2_size, int64_t spatial_size,
                   uint64_t* keys, int32_t* vals, int64_t* stats, msp_stream_t stream);

/* Scene boundaries of a non-decreasing batch column (msp_point_keys stats[2]
 * == 0): starts[b] = first row whose batch id is >= b, for b = 0..n_batch
 * (n_batch + 1 entries; starts[n_batch] = n when n_batch > max batch id).  The
 * caller reads them back together with the voxel count, so checking that the
 * reference's batch_offsets (dataset/data.py:142,209) are exactly the batch-id
 * ranges (the fused per-scene mean, models/SparseConvNet.py:20-26) needs no
 * extra device-to-host read. */
int msp_batch_starts(const int64_t* coords, int64_t n, int64_t row_stride, int64_t n_batch, int64_t* starts,
                     msp_stream_t stream);

size_t msp_sort_workspace_size(int64_t n, int end_bit);
/* Stable LSD radix sort of (key, value) pairs on bits [0, end_bit). */
int msp_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in, int32_t* vals_out,
                   int64_t n, int end_bit, void* ws, size_t ws_bytes, msp_stream_t stream);

size_t msp_scan_workspace_size(int64_t n);
/* Group a sorted key array by (key >> shift).  seg_of[i] = group of row i;
 * uniq_keys[g] = key>>shift of group g; seg_start[g] = first row of group g and
 * seg_start[G] = n (capacity n+1); n_uniq[0] = G (device int64).  If perm and
 * p2v are non-NULL, also p2v[perm[i]] = seg_of[i] (point -> voxel map). */
int msp_segment(const uint64_t* sorted_keys, int64_t n, int shift, const int32_t* perm, int32_t* seg_of,
                int32_t* p2v, uint64_t* uniq_keys, int32_t* seg_start, int64_t* n_uniq, void* ws,
                size_t ws_bytes, msp_stream_t stream);

/* ---------------- metadata: hash grid + rulebooks (replaces SCN Metadata's
 * submanifold / strided rulebooks) ----------------- */
int64_t msp_hash_capacity(int64_t n);
/* Block hash of a level's keys: open-addressing table of cap 16-byte slots
 * (table = 2*cap uint64, one probe = one load), one slot per occupied block of
 * 32 consecutive Morton codes: {key >> 5, (first row << 32) | occupancy mask}.
 * msp_hash_build empties every slot first (0xFF bytes); keys unique and
 * sorted ascending (a level's keys are), so a block's rows are contiguous. */
int msp_hash_build(const uint64_t* keys, int64_t n, uint64_t* table, int64_t cap, msp_stream_t stream);
/* Submanifold neighbour map nbr[K][n], K = filter_size^3 (odd filter_size),
 * every entry written (-1: no neighbour); table / cap from msp_hash_build. */
int msp_subm_map(const uint64_t* keys, int64_t n, int log2_size, int64_t spatial_size, int filter_size,
                 const uint64_t* table, int64_t cap, int32_t* nbr, msp_stream_t stream);
/* msp_subm_map + the number of present entries (the rulebook size, centre
 * included) into n_rules (device int64), counted as the map is written;
 * workspace msp_subm_map_workspace_size(n, filter_size) bytes. */
size_t msp_subm_map_workspace_size(int64_t n, int filter_size);
int msp_subm_map_counted(const uint64_t* keys, int64_t n, int log2_size, int64_t spatial_size, int filter_size,
                         const uint64_t* table, int64_t cap, int32_t* nbr, int64_t* n_rules, void* ws,
                         size_t ws_bytes, msp_stream_t stream);
/* Strided (size == stride == 2^log2_stride) child map: down[K][n_coarse],
 * K = 8^log2_stride, down[o][parent_of[i]] = i for every fine row i. */
int msp_down_map(const uint64_t* fine_keys, int64_t n_fine, const int32_t* parent_of, int log2_size_fine,
                 int log2_stride, int32_t* down, int64_t n_coarse, msp_stream_t stream);
/* Per-offset pair lists of an offset-major map: for o in [0,K), for every row
 * r with map[o][r] >= 0 (ascending r): (pair_in, pair_out) = (map[o][r], r).
 * off_start[K+1] (device int64) gets the list starts.  Pass cap = 0 to only
 * count (off_start[K] = total), then call again with cap >= total and the same
 * off_start and workspace (the filling call reuses the counting call's block
 * offsets instead of recounting). */
int msp_pair_lists(const int32_t* map, int K, int64_t n, int32_t* pair_in, int32_t* pair_out, int64_t cap,
                   int64_t* off_start, void* ws, size_t ws_bytes, msp_stream_t stream);
/* Output-tile rulebook for msp_conv_tile: rows are cut into tiles of
 * tile_rows (64, 128 or 256); inside a tile the present (row, offset) pairs of
 * each offset are compacted (wavefront ballot + prefix sum across the tile's
 * waves) into chunks of MSP_CHUNK, chunks sorted by offset.
 * tile_start[n_tiles+2] (device int64; tile_start[n_tiles+1] = the largest
 * chunk count of one tile), chunk_off[c] = offset, chunk_src[c*16+j]
 * = input row, chunk_row[c*16+j] = row inside the tile.  Padding slots of a
 * chunk have chunk_row = tile_rows and repeat a present input row of the same
 * tile and offset (so every gather stays in bounds).
 * Count-then-fill like msp_pair_lists (total chunks = tile_start[n_tiles]); the
 * filling call reuses tile_start from the counting call. */
int msp_tile_rulebook(const int32_t* map, int K, int64_t n, int tile_rows, int64_t* tile_start,
                      uint8_t* chunk_off, int32_t* chunk_src, uint16_t* chunk_row, int64_t chunk_cap, void* ws,
                      size_t ws_bytes, msp_stream_t stream);
/* Tile-local rulebook of a submanifold neighbour map (msp_conv_local):
 * rows are cut into tiles of tile_rows (64, 128 or 256); per tile t the
 * distinct input rows its neighbour entries name are listed in ascending order
 * at u_rows[u_start[t] .. u_start[t+1]); perm[t*T + i] is the tile's i-th row
 * (rows grouped inside the tile so that each 16-row group's rows share
 * offsets: greedy, by fewest offsets added to the group's union; -1 past n)
 * and lidx[o][t*T + i] (uint16, [K][n_tiles*T]) the position in the tile's
 * list of that row's neighbour at offset o (0xFFFF: none).  K <= 32.
 * wave_off (nullable; written for tile_rows = 128 and K <= 27, n_tiles x 64
 * bytes): msp_conv_local's offset lists -- for row half h (16-row groups h,
 * h+2, h+4, h+6) and wave c < 4, wave_off[t*64 + h*32 + c*8 + k] = the k-th
 * offset that wave walks (0xFF: none), every offset some row of the half has
 * listed once, dealt longest-first onto the least-loaded wave.
 * Count-then-fill like msp_pair_lists: the counting call (u_cap = 0) writes
 * u_start[0..n_tiles] (u_start[n_tiles] = total) and u_start[n_tiles+1] = the
 * largest tile's count; the filling call (u_cap >= total) reuses u_start.
 * A filling call with lidx = perm = NULL writes the lists only (u_rows: all
 * msp_conv_wgrad_chunk needs; no row grouping, the bulk of the fill). 
 * Workspace: msp_tile_local_workspace_size. */
size_t msp_tile_local_workspace_size(int64_t n, int tile_rows);
int msp_tile_local(const int32_t* nbr, int K, int64_t n, int tile_rows, int64_t* u_start, int32_t* u_rows,
                   int64_t u_cap, uint16_t* lidx, int32_t* perm, uint8_t* wave_off, void* ws, size_t ws_bytes,
                   msp_stream_t stream);
/* Decode keys back to (x, y, z, batch) int64 rows (SparseToDense, locations). */
int msp_decode_keys(const uint64_t* keys, int64_t n, int log2_size, int64_t* coords, msp_stream_t stream);

/* ---------------- sparse convolution (replaces SCN SubmanifoldConvolution /
 * Convolution / Deconvolution updateOutput + backward) */

/* Output-stationary gather-MFMA convolution over a tile rulebook built with
 * tile_rows = 128 (msp_conv_tile_rows):
 *   out[r, :] = sum over chunks of r's tile: sum_j W'[o]^T x[src_j, :]
 * wt is [K][c_out][c_in] (k contiguous).  flip bit 0: offset o reads
 * wt[K-1-o] (submanifold backward-data with the forward weight layout);
 * bit 1 (128-row tiles): wt is given as [K][c_in][c_out] instead, the
 * module's own layout, so the forward needs no transposed copy.
 * c_in % 16 == 0, c_out % 16 == 0.  Every output row is written.  Narrow
 * outputs (c_out <= 32, c_in <= 64) run per-wave tiles, wider ones a tile
 * shared by the 4 waves of a block; the contraction
 * runs on bf16 MFMA over exact three-piece bf16 splits of both fp32 operands
 * (six piece products, fp32 accumulation: fp32-class error, checked against
 * fp64 in tests/test_gpu_ops.py); the split weights and, on small grids, the
 * partial sums of an offset split (added in a fixed order) live in the
 * workspace: ws_bytes >= msp_conv_tile_workspace_size(n_rows, K, c_in,
 * c_out, tile_rows).  msp_conv_tile_rows gives the tile height the library
 * is tuned for. */
int msp_conv_tile_rows(int64_t n_rows, int c_in, int c_out);
/* Contraction form msp_conv_tile runs for these sizes: 1 = per-wave split-bf16
 * tile (conv_x6r: c_out <= 32, c_in <= 64), 2 = shared split-bf16 tile (conv_x6d,
 * split over offsets on small grids), 0 = nothing to do (or tile_rows != 128). */
int msp_conv_tile_form(int64_t n_rows, int c_in, int c_out, int tile_rows);

/* Tile-local submanifold convolution (replaces the gather forms where
 * msp_conv_local_preferred says so): out[perm row] = sum_o W'[o]^T x[nbr(row, o)]
 * over a msp_tile_local rulebook with tile_rows = 128 (K <= 27).  Each tile's
 * distinct input rows are staged in LDS once per 32 input channels and split
 * into exact bf16 pieces once; the rules read them from LDS.  flip and the
 * weight layouts as msp_conv_tile (bit 0: offset K-1-o, bit 1: wt is
 * [K][c_in][c_out], else [K][c_out][c_in]).  wave_off: msp_tile_local's
 * offset lists of the same rulebook (NULL: offsets dealt round-robin, o = c +
 * 4 j to wave c of each row half).  Workspace: msp_conv_local_workspace_size
 * (the split weight image). */
int msp_conv_local_preferred(int64_t n_rows, int c_in, int c_out);

size_t msp_conv_local_workspace_size(int K, int c_in, int c_out);
int msp_conv_local(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                   const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows, const int32_t* perm,
                   const uint8_t* wave_off, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                   msp_stream_t stream);
/* Submanifold weight gradient over a 128-row tile rulebook (msp_tile_rulebook, tile_rows = 128) and the
 * tile-local rulebook of the same map (msp_tile_local, tile_rows = 128): dW[o][ci][co] = sum over the rules
 * (i, j) of offset o of x[i][ci] dy[j][co] (the forward's [K][c_in][c_out] layout).  msp_wgrad_chunk_index
 * writes per chunk entry e chunk_lr[e] = (position of its input row in its tile's u_rows list) | (row in the
 * tile, 128 for a padding slot) << 16.  msp_conv_wgrad_chunk stages per tile the listed x rows and the 128 dy
 * rows in LDS once per 32 x 32 channel slice (exact bf16 pieces); the rulebook's chunks are the MFMA k-steps.
 * A tile lists at most msp_wgrad_chunk_cap() rows in LDS: a rule whose input row lies past the cap is marked
 * 0xFFFF and contributes nothing to msp_conv_wgrad_chunk; n_far (device int64, nullable) receives the number of
 * such rules (0 when every tile's list, msp_tile_local's largest count u_start[n_tiles + 1], is within the cap).
 * Their products are added afterwards (round 4): msp_wgrad_far_list writes those n_far chunk entries sorted by
 * (offset, entry) -- far_key[k] = offset << 40 | entry, far_tile[k] = the entry's tile; workspace
 * msp_wgrad_far_workspace_size(n_far) -- and msp_conv_wgrad_far adds, after msp_conv_wgrad_chunk filled dw,
 * dw[o][ci][co] += the far rules' x[i][ci] dy[j][co] of offset o, fp64 sums in list order.  K <= 27, channels in
 * multiples of 32 (msp_wgrad_chunk_ok; msp_wgrad_chunk_preferred: the shapes the library takes it for).
 * Blocks run n_ranges contiguous tile ranges (msp_wgrad_chunk_ranges) per slice; slab holds n_ranges x K x
 * c_in x c_out floats of partial sums, added in range order into dw. */
/* Per-step split-weight images (round 3).  msp_conv_tile, msp_conv_local and msp_conv_nbr split their fp32
 * weights into an exact bf16-piece image in the workspace on every call; flip bit 2 (value 4) tells them the
 * workspace ALREADY holds that image (they skip the split).  msp_conv_weight_image describes the image a call with
 * these arguments makes (entry 0: msp_conv_tile with tile_rows 128, 1: msp_conv_local, 2: msp_conv_nbr) -- every
 * field but wt and img, which the caller fills; bytes = the workspace size the call needs.  A training step can
 * then split every layer's images in ONE launch: msp_split_weight_images over a device array of n descriptors and
 * their units' exclusive prefix sums unit_start[0..n] (total_units = unit_start[n]), after the weights last
 * changed and before the convolutions that use them. */
typedef struct {
  const float* wt; /* weights as the convolution is called with them */
  void* img;       /* caller-owned buffer of >= bytes */
  int64_t units;   /* work items of the image */
  int64_t bytes;   /* workspace bytes the call needs (image first) */
  int32_t kind;    /* 1: per-step slices (msp_conv_tile / msp_conv_nbr), 2: lane-ordered (msp_conv_local) */
  int32_t K, c_in, c_out;
  int32_t p;    /* kind 1: columns per slice; kind 2: 16-column tiles per block */
  int32_t wlay; /* 1: wt is [K][c_in][c_out], 0: [K][c_out][c_in] (flip bit 1) */
} msp_weight_image;
int msp_conv_weight_image(int entry, int64_t n_rows, int K, int c_in, int c_out, int flip, msp_weight_image* d);
int msp_split_weight_images(const msp_weight_image* descs, int n, const int64_t* unit_start, int64_t total_units,
                            msp_stream_t stream);
int64_t msp_wgrad_chunk_cap(void);
int msp_wgrad_chunk_ok(int64_t n_rows, int K, int c_in, int c_out);
int msp_wgrad_chunk_preferred(int64_t n_rows, int K, int c_in, int c_out);
int64_t msp_wgrad_chunk_ranges(int64_t n_rows, int c_in, int c_out);
int msp_wgrad_chunk_index(const int64_t* tile_start, const int32_t* chunk_src, const uint16_t* chunk_row,
                          int64_t n_rows, const int64_t* u_start, const int32_t* u_rows, uint32_t* chunk_lr,
                          int64_t* n_far, msp_stream_t stream);
/* The same index (tile_start[n_tiles + 2], chunk_off, chunk_lr as above, tiles of 128 rows) built from a FULL
 * tile-local rulebook of the map (msp_tile_local with lidx / perm, tile_rows = 128) instead of the tile rulebook:
 * per tile and offset the present lidx entries, in natural row order, in 16-entry chunks, offsets
 * ascending; padding slots are (0 | 128 << 16).  Count-then-fill like msp_tile_rulebook (chunk_cap = 0: count,
 * tile_start[n_tiles] = total chunks, tile_start[n_tiles + 1] = the largest tile's; then fill with chunk_cap >=
 * total and the same workspace, msp_tile_local_workspace_size(n, 128) bytes).  Every position must be within
 * msp_wgrad_chunk_cap() (u_start[n_tiles + 1] <= cap): no far rules. */
int msp_local_chunk_index(const uint16_t* lidx, const int32_t* perm, int K, int64_t n, int64_t* tile_start,
                          uint8_t* chunk_off, uint32_t* chunk_lr, int64_t chunk_cap, void* ws, size_t ws_bytes,
                          msp_stream_t stream);
int msp_conv_wgrad_chunk(const float* x, int c_in, const float* dy, int c_out, int K, int tile_rows,
                         const int64_t* tile_start, const uint8_t* chunk_off, const uint32_t* chunk_lr,
                         const int64_t* u_start, const int32_t* u_rows, int64_t n_rows, int64_t n_ranges,
                         float* slab, float* dw, msp_stream_t stream);
size_t msp_wgrad_far_workspace_size(int64_t n_far);
int msp_wgrad_far_list(const int64_t* tile_start, const uint8_t* chunk_off, const uint32_t* chunk_lr,
                       int64_t n_rows, int64_t n_far, int64_t* far_key, int32_t* far_tile, void* ws,
                       size_t ws_bytes, msp_stream_t stream);
int msp_conv_wgrad_far(const float* x, int c_in, const float* dy, int c_out, int K, const int32_t* chunk_src,
                       const uint16_t* chunk_row, const int64_t* far_key, const int32_t* far_tile, int64_t n_far,
                       float* dw, msp_stream_t stream);
size_t msp_conv_tile_workspace_size(int64_t n_rows, int K, int c_in, int c_out, int tile_rows);
int msp_conv_tile(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                  const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                  const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                  msp_stream_t stream);
/* Dense row-group form of the submanifold convolution, straight from the
 * neighbour map nbr[K][n_rows] (int32, -1 absent, row stride n_rows): same
 * sum as msp_conv_tile over that map's tile rulebook (same flip bits and weight
 * layouts), with every 16 consecutive output rows computed together over all
 * K offsets (absent neighbours contribute zero, a group with none of an
 * offset skips it) and accumulated in registers: no tile rulebook needed.
 * Same split-bf16 arithmetic and error class as msp_conv_tile.
 * msp_conv_nbr_preferred says for which shapes the library runs it (the
 * large levels, c_out >= 64); ws_bytes >= msp_conv_nbr_workspace_size. */
/* With perm non-NULL, position j of the groups is output row perm[j] and
 * nbr holds the permuted map (nbr[o][j] = neighbour of row perm[j]), as
 * msp_dense_order makes them: rows with similar neighbour masks share a
 * group, so fewer MFMA rows are zero. */
int msp_conv_nbr_preferred(int64_t n_rows, int c_in, int c_out);
size_t msp_conv_nbr_workspace_size(int K, int c_in, int c_out);
int msp_conv_nbr(const float* x, int c_in, const float* wt, int K, int flip, int c_out, const int32_t* nbr,
                 const int32_t* perm, int64_t n_rows, float* out, void* ws, size_t ws_bytes, msp_stream_t stream);
/* Row order for msp_conv_nbr: inside each window of 2^log2_window
 * consecutive rows, rows sorted stably by their neighbour mask (K <= 32):
 * perm[j] = row at position j, nbr_perm[o][j] = nbr[o][perm[j]] (both [n] /
 * [K][n], caller-owned); ws_bytes >= msp_dense_order_workspace_size. */
size_t msp_dense_order_workspace_size(int64_t n, int K, int log2_window);
int msp_dense_order(const int32_t* nbr, int K, int64_t n, int log2_window, int32_t* perm, int32_t* nbr_perm,
                    void* ws, size_t ws_bytes, msp_stream_t stream);
/* One contribution per output row (deconvolution forward, strided
 * convolution backward-data): out[pair_out[p]] = W'[o]^T x[pair_in[p]] for the
 * pairs of offset o.  chunk_start[K+1] (device) = prefix sums of
 * ceil(n_o / 16); n_chunks = chunk_start[K]. */
int msp_conv_pairs(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* pair_in,
                   const int32_t* pair_out, const int64_t* off_start, const int64_t* chunk_start,
                   int64_t n_chunks, float* out, msp_stream_t stream);
/* msp_conv_pairs_x6 (round 6, ABI 10): the same on the split-bf16 MFMAs (fp32-class, as the other x6 forms) with
 * wt given as [K][c_out][c_in]; ws (>= msp_conv_pairs_x6_workspace_size bytes) receives the call's weight image. */
size_t msp_conv_pairs_x6_workspace_size(int K, int c_in, int c_out);
int msp_conv_pairs_x6(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* pair_in,
                      const int32_t* pair_out, const int64_t* off_start, const int64_t* chunk_start, int64_t n_chunks,
                      float* out, void* ws, size_t ws_bytes, msp_stream_t stream);
/* Weight gradient dW[o] (c_in x c_out) = sum over pairs of offset o of
 * x[pair_in]^T dy[pair_out].  Each offset's pair list (sorted by one side's
 * row) is cut into n_pieces equal pieces; piece j of every offset covers
 * about the same row band, and the K pieces of a band run together so the
 * band's rows are read from L2 once.  Piece (j, o) writes its partial tile to
 * slab[n_pieces][K][c_in][c_out]; a second kernel reduces the pieces in a
 * fixed order (deterministic) into dw[K][c_in][c_out].  msp_wgrad_pieces
 * gives the piece count the library is tuned for (about 4096 blocks). */
int64_t msp_wgrad_pieces(int64_t total_pairs, int K, int c_in, int c_out);
int msp_conv_wgrad(const float* x, int c_in, const float* dy, int c_out, const int32_t* pair_in,
                   const int32_t* pair_out, const int64_t* off_start, int K, int64_t n_pieces, float* slab,
                   float* dw, msp_stream_t stream);
/* Submanifold convolution of a narrow input (the first layer's colour channels, models/SparseConvNet.py:62:
 * SubmanifoldConvolution(3, m, 3, False)) straight from the neighbour map nbr[K][n_rows] (int32, -1 absent):
 * out[i][c] = sum_o sum_k x[nbr[o][i]][k] wt[o][k][c], x [n][c_in] and wt [K][c_in][c_out] unpadded (the
 * module's layout), fp32 fmaf per term, offsets then channels in order.  msp_conv_wgrad_narrow_in: dw[o][k][c] =
 * sum over rows i with a neighbour at offset o of x[nbr[o][i]][k] dy[i][c]; n_parts blocks each write a partial
 * to slab[n_parts][K][c_in][c_out], added in part order into dw (msp_conv_wgrad_narrow_parts: the count the
 * library is tuned for).  Shapes: msp_conv_narrow_in_ok (K <= 27, c_in <= 4, c_out in {16, 32, 64}).  Replaces
 * the padded 16-channel path of msp_conv_tile / msp_conv_wgrad for that layer. */
int msp_conv_narrow_in_ok(int K, int c_in, int c_out);
int msp_conv_narrow_in(const float* x, int c_in, const float* wt, int K, int c_out, const int32_t* nbr,
                       int64_t n_rows, float* out, msp_stream_t stream);
int64_t msp_conv_wgrad_narrow_parts(int64_t n_rows, int K, int c_in, int c_out);
int msp_conv_wgrad_narrow_in(const float* x, int c_in, const float* dy, int c_out, const int32_t* nbr, int K,
                             int64_t n_rows, int64_t n_parts, float* slab, float* dw, msp_stream_t stream);

/* ---------------- batch norm + (leaky) ReLU (replaces SCN BatchNormalization
 * with leakiness; scn.BatchNormReLU / BatchNormLeakyReLU).
 * Per-channel statistics are one float array stats[5][C]: mean_hi, mean_lo
 * (the fp64 mean as an fp32 pair), invstd, scale = weight*invstd,
 * shift = bias; y = leaky_relu(((x - mean_hi) - mean_lo) * scale + shift). */
/* Partial-sum buffers hold (msp_bn_partials(V, C) + 1) * 2 * C doubles. */
int64_t msp_bn_partials(int64_t V, int C);
int msp_bn_stats(const float* x, int64_t V, int C, double* partial, msp_stream_t stream);
/* train: batch statistics from partial, running stats updated; eval: running
 * statistics.  weight/bias may be NULL (non-affine). */
int msp_bn_finalize(const double* partial, int64_t V, int C, double eps, double momentum, int train,
                    float* running_mean, float* running_var, const float* weight, const float* bias,
                    float* stats, msp_stream_t stream);
int msp_bn_apply(const float* x, int64_t V, int C, const float* stats, float leak, float* y, msp_stream_t stream);
int msp_bn_bwd_stats(const float* x, const float* dy, int64_t V, int C, const float* stats, float leak,
                     double* partial, msp_stream_t stream);
int msp_bn_bwd_apply(const float* x, const float* dy, int64_t V, int C, const double* partial, const float* stats,
                     const float* weight, float leak, int train, float* dx, float* dweight, float* dbias,
                     msp_stream_t stream);
/* Residual fusions (SCN's ConcatTable(shortcut, BN...) / AddTable pair,
 * networkArchitectures.py res blocks; the reference leaves these to autograd
 * and a separate add).  msp_bn_bwd_apply_add: as msp_bn_bwd_apply, plus
 * dx += addend (the shortcut's gradient of x, one fp32 add as autograd's
 * accumulation would do); addend may be NULL, must not alias dx.
 * msp_add_bn_stats: sum = a + b and the msp_bn_stats partials of sum in one
 * pass (identical partials to msp_bn_stats on sum). */
int msp_bn_bwd_apply_add(const float* x, const float* dy, int64_t V, int C, const double* partial,
                         const float* stats, const float* weight, float leak, int train, const float* addend,
                         float* dx, float* dweight, float* dbias, msp_stream_t stream);
int msp_add_bn_stats(const float* a, const float* b, int64_t V, int C, float* sum, double* partial,
                     msp_stream_t stream);
/* msp_bn_bwd_apply_split (ABI 10): msp_bn_bwd_apply_add with dx written as two tensors, columns [0, ca) to dxa
 * [V][ca] and [ca, C) to dxb [V][C - ca] -- where x was a JoinTable's output ([a | b], msp_join_cols), these are
 * the gradients of a and b, and no msp_split_cols pass follows (the UNet decoder's join -> BN fork).  Same
 * arithmetic per element as msp_bn_bwd_apply_add; 0 < ca < C; dxa, dxb non-NULL and aliasing nothing. */
int msp_bn_bwd_apply_split(const float* x, const float* dy, int64_t V, int C, const double* partial,
                           const float* stats, const float* weight, float leak, int train, const float* addend,
                           int ca, float* dxa, float* dxb, float* dweight, float* dbias, msp_stream_t stream);
/* Channel join (SCN JoinTable, the UNet / FCN skip joins: identity branch first, then the upsampled deeper
 * level): out[v] = [a[v] | b[v]], a [V][ca], b [V][cb], out [V][ca + cb].  With partial
 * non-NULL also the msp_bn_stats partials of out (identical to msp_bn_stats on it), for the BatchNormalization
 * the join feeds.  msp_split_cols is its backward: in [V][ca + cb] -> a [V][ca], b [V][cb] (either may be
 * NULL). */
int msp_join_cols(const float* a, int ca, const float* b, int cb, int64_t V, float* out, double* partial,
                  msp_stream_t stream);
/* BatchNormalization statistics from a convolution's epilogue (round 6; the BN -> SubM -> BN -> SubM chains of
 * models/SparseConvNet.py:63-69).  msp_conv_local_bn / msp_conv_tile_bn are msp_conv_local / msp_conv_tile plus,
 * when epi is non-NULL, per-channel fp64 sums of the rows they write, one slot per 128-row tile, into the
 * channel-major buffer epi->partial[2][C][P] (C = c_out, P = msp_conv_bn_parts(n_rows); the buffer holds
 * 2 * C * (P + 1) doubles, the tail for msp_bn_bwd_apply_cm's totals):
 *   epi->x == NULL (forward): (sum v, sum v^2) of the output rows v -- msp_bn_stats' sums of the output, for the
 *     BatchNormalization the convolution feeds (msp_bn_finalize_cm);
 *   epi->x != NULL (backward-data): the output is dy, the gradient of the output of the BatchNormalization whose
 *     input rows are epi->x [n_rows][C] and statistics epi->stats [5][C] (leakiness epi->leak) -- the sums of
 *     msp_bn_bwd_stats, (sum dz, sum dz * xhat), for msp_bn_bwd_apply_cm.
 * Sums within a tile are taken in a fixed order and the tiles are added in tile order: deterministic.  The
 * epilogue is available where msp_conv_tile_form(...) == 1 (per-wave tiles) and on every msp_conv_local call;
 * msp_conv_tile_bn with epi on another form returns MSP_EINVAL. */
typedef struct {
  double* partial;
  const float* x;
  const float* stats;
  float leak;
} msp_bn_epilogue;
int64_t msp_conv_bn_parts(int64_t n_rows);
int msp_conv_local_bn(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                      const uint16_t* lidx, const int64_t* u_start, const int32_t* u_rows, const int32_t* perm,
                      const uint8_t* wave_off, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                      const msp_bn_epilogue* epi, msp_stream_t stream);
int msp_conv_tile_bn(const float* x, int c_in, const float* wt, int K, int flip, int c_out, int tile_rows,
                     const int64_t* tile_start, const uint8_t* chunk_off, const int32_t* chunk_src,
                     const uint16_t* chunk_row, int64_t n_rows, float* out, void* ws, size_t ws_bytes,
                     const msp_bn_epilogue* epi, msp_stream_t stream);
/* msp_bn_finalize / msp_bn_bwd_apply_add over a channel-major partial buffer [2][C][P] (+ [2][C] tail) of P
 * slots, as the epilogue above writes it. */
int msp_bn_finalize_cm(const double* partial, int64_t P, int64_t V, int C, double eps, double momentum, int train,
                       float* running_mean, float* running_var, const float* weight, const float* bias,
                       float* stats, msp_stream_t stream);
int msp_bn_bwd_apply_cm(const float* x, const float* dy, int64_t V, int C, const double* partial, int64_t P,
                        const float* stats, const float* weight, float leak, int train, const float* addend,
                        float* dx, float* dweight, float* dbias, msp_stream_t stream);
int msp_split_cols(const float* in, int64_t V, int ca, int cb, float* a, float* b, msp_stream_t stream);

/* ---------------- NetworkInNetwork products (replaces SCN's NetworkInNetwork
 * forward / backward-data, scn.NetworkInNetwork in the UNet/FCN residual
 * shortcuts): C[M][N] = A[M][K] B[K][N], row-major fp32.
 * Forward: A = x, B = W[c_in][c_out]; backward-data: A = dy, B = W^T.  Below
 * 2^18 rows bf16 MFMA over exact three-piece splits of both operands (six
 * piece products, fp32 accumulation), from 2^18 rows fp32 MFMA: fp32-class
 * error either way, checked against fp64 in tests/test_gpu_ops.py.
 * msp_nin_gemm_ok: K % 16 == 0, N % 16 == 0, K <= 1024; A, B and C 16-byte
 * aligned.  Workspace (B's split fragment image):
 * msp_nin_gemm_workspace_size(K, N) bytes. */
int msp_nin_gemm_ok(int64_t M, int K, int N);
/* the form msp_nin_gemm runs: 1 = fp32 MFMA, 2 = split-bf16 MFMA, 0 = unsupported shape */
int msp_nin_gemm_form(int64_t M, int K, int N);
size_t msp_nin_gemm_workspace_size(int K, int N);
int msp_nin_gemm(const float* A, int64_t M, int K, const float* B, int N, float* C, void* ws, size_t ws_bytes,
                 msp_stream_t stream);

/* ---------------- input / output / pooling layers */
/* mode-4 average: out[v] = mean of feats[perm[j]] for j in [vstart[v], vstart[v+1]) */
int msp_input_avg_fwd(const float* feats, int C, const int32_t* perm, const int32_t* vstart, int64_t V,
                      float* out, msp_stream_t stream);
int msp_input_avg_bwd(const float* dout, int C, const int32_t* p2v, const int32_t* vstart, int64_t n_points,
                      float* dfeats, msp_stream_t stream);
int msp_output_fwd(const float* in, int C, const int32_t* p2v, int64_t n_points, float* out, msp_stream_t stream);
int msp_output_bwd(const float* dout, int C, const int32_t* perm, const int32_t* vstart, int64_t V, float* din,
                   msp_stream_t stream);
/* out[i] = in[parent_of[i]] */
int msp_unpool_fwd(const float* in, int C, const int32_t* parent_of, int64_t n_fine, float* out,
                   msp_stream_t stream);
/* din[p] = sum of dout over children [child_start[p], child_start[p+1]) */
int msp_unpool_bwd(const float* dout, int C, const int32_t* child_start, int64_t n_coarse, float* din,
                   msp_stream_t stream);
int msp_maxpool_fwd(const float* in, int C, const int32_t* child_start, int64_t n_coarse, float* out,
                    int32_t* argmax, msp_stream_t stream);
/* din must be zeroed by the caller */
int msp_maxpool_bwd(const float* dout, int C, const int32_t* argmax, int64_t n_coarse, float* din,
                    msp_stream_t stream);

/* ---------------- fused encoder tail (training): OutputLayer + per-scene
 * mean of the per-point features, SparseConvBase_.postProcessing
 * (models/SparseConvNet.py:20-26), from the level-0 voxel rows without the
 * (N, C) per-point tensor.  keys: the level's sorted keys, shift = 3*log2 of
 * its spatial size (batch = key >> shift), vstart[V+1]: point runs of the
 * voxels (InputLayer).  Writes vscene[B+1] (voxel range of each scene),
 * npts[B] (points per scene) and out[B][C] = mean over the scene's points;
 * 1 <= C <= 1024.  Fixed-order two-stage reduction (deterministic). */
size_t msp_scene_mean_workspace_size(int64_t V, int B, int C);
int msp_scene_mean_fwd(const float* feats, int C, const uint64_t* keys, int64_t V, int shift,
                       const int32_t* vstart, int B, int64_t* vscene, int64_t* npts, float* out, void* ws,
                       size_t ws_bytes, msp_stream_t stream);
/* dfeats[v] = (cnt_v / npts[b(v)]) * dout[b(v)] */
int msp_scene_mean_bwd(const float* dout, int C, const uint64_t* keys, int64_t V, int shift, const int32_t* vstart,
                       const int64_t* npts, float* dfeats, msp_stream_t stream);

/* ---------------- fused encoder tail (eval / per-point logits): the head's Linear
 * (models/MultiLabelContrastive.py:43-45 `self.linear(self.pc_encoder(x))`, :84-101; train.py:106) commutes
 * with the OutputLayer's gather, so the caller applies it to the level-0 voxel rows ((V, C) @ W^T on
 * msp_nin_gemm -> in, row stride ld) and this gathers the C output columns per point plus the bias:
 * out[p][c] = in[p2v[p] * ld + c] + bias[c] (bias may be NULL).  The (N, C_embed) per-point feature tensor
 * is never formed. */
int msp_point_rows_bias(const float* in, int64_t ld, int C, const float* bias, const int32_t* p2v, int64_t n_points,
                        float* out, msp_stream_t stream);
/* store[ids[i]][:] += src[i][:] for i = 0..n-1 (train.py:107 `store.index_add_(0, point_ids, predictions)`),
 * bit-equal to the serial loop in i order for any ids (repeated ids included): pairs (id, i) are radix sorted
 * stably by id and each id's run is added into the stored row in ascending i.  Ids outside [0, n_store) are
 * skipped (the caller validates them).  store [n_store][C], src [n][C] float32; ids int64 (device).
 * ws_bytes >= msp_index_add_workspace_size(n, n_store). */
size_t msp_index_add_workspace_size(int64_t n, int64_t n_store);
int msp_index_add_rows(float* store, int64_t n_store, int C, const int64_t* ids, const float* src, int64_t n,
                       void* ws, size_t ws_bytes, msp_stream_t stream);

/* ---------------- batch assembly on the device:
 * the per-point part of trainMerge (mode 0, dataset/data.py:135-238) and
 * valMerge (mode 1, :256-310) for B scenes already in HBM.  Scene b is points
 * [scene_start[b], scene_start[b+1]) of xyz/rgb (f32, 3 per point) and labels
 * (int64).  Per scene (device arrays, the host's random draws): rot[b][9]
 * (t = a . rot), c1[b][3], c2[b][3] (added to t in that order), u1/u2[b][3]
 * (the offset's two rand(3)), shift[b][3] (f32 colour shift).  fp64
 * arithmetic in a fixed order without FMA contraction; then the mode's
 * offset formula, the crop to [0, full_scale)^3 and trunc() -> coords
 * (N,4) int64 [x,y,z,b] in point order, feats = rgb + shift, labels_out,
 * point_ids (mode 1, may be NULL) = point_id_base + input index,
 * batch_offsets[B+1] (device) and scene_labels[B][n_classes] (1 where a kept
 * point has that label; n_classes <= 32).  Outputs are sized for all points
 * (capacity scene_start[B]); the kept count is batch_offsets[B]. */
size_t msp_merge_workspace_size(int B, int64_t max_scene_points);
int msp_merge(const float* xyz, const float* rgb, const int64_t* labels, const int64_t* scene_start, int B,
              int64_t max_scene_points, int mode, double full_scale, const double* rot, const double* c1,
              const double* c2, const double* u1, const double* u2, const float* shift, int n_classes,
              int64_t* coords, float* feats, int64_t* labels_out, int64_t* point_ids, int64_t point_id_base,
              int64_t* batch_offsets, float* scene_labels, void* ws, size_t ws_bytes, msp_stream_t stream);

/* The training step's optimizer (round 6, ABI 10): torch.optim.Adam (the reference's train.py:39, Adam(lr=1e-3);
 * amsgrad off) over up to MSP_ADAM_MAX_TENSORS parameter tensors in one launch.  table: device array of n
 * msp_adam_tensor (param, exp_avg, exp_avg_sq: fp32, n floats each, contiguous); chunk_start: device exclusive
 * prefix sums [n + 1] of msp_adam_chunks(table[i].n) (n_chunks = chunk_start[n]); grads: HOST array of n device
 * gradient pointers (NULL: that tensor is skipped this step), passed to the kernel by value, so a captured graph
 * keeps the step's own; step: device float step count, incremented first when bump != 0 (the first call of an
 * optimizer step), then read as t.  Per element (fp32; 1 - b1, 1 - b2 and the bias corrections formed in double,
 * as torch's fused Adam takes its scalars): g += wd * p; m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2;
 * p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps). */
#define MSP_ADAM_MAX_TENSORS 256
typedef struct {
  float* param;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
} msp_adam_tensor;
int64_t msp_adam_chunks(int64_t n);
int msp_adam_step(const msp_adam_tensor* table, const int64_t* chunk_start, const float* const* grads, int n,
                  int64_t n_chunks, float* step, int bump, double lr, double beta1, double beta2, double eps,
                  double weight_decay, msp_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MI3DSPARSE_H */
