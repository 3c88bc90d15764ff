/*
 * ngnn.h — C ABI of the MI355X-native GraphSAGE / GCN aggregation path.
 *
 * The reference (hhilsber/noise-GNN) is pure Python: its hot path is
 * SAGE.forward -> PyG SAGEConv.forward (src/models/layers/sage.py:30-40,
 * conv call at :34) and SimpleGCN.forward -> PyG GCNConv.forward
 * (src/models/layers/convolution.py:29-35, call at :31).  PyG 2.5.1 [ext]
 * implements each conv as index_select (gather) + scatter_add_/scatter_reduce_
 * (scatter) + Linear.  The reference has no FFI of its own; the entry points
 * below are what a ctypes binding of those PyG internals would bind, and are
 * what noise-gnn_amd/ngnn/_lib.py binds (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless stated; the caller owns every
 *     buffer (PyTorch caching-allocator tensors).  The library never
 *     allocates, frees or retains pointers beyond the call.
 *   - Every call is asynchronous and stream-ordered on `stream`
 *     (a hipStream_t passed as void*; NULL = the legacy default stream).
 *   - Return 0 on success, a negative NGNN_E_* for argument errors (nothing
 *     is launched), or a positive hipError_t from a failed launch.
 *   - Index arrays are int32 internally (N, E < 2^31), rows of feature
 *     matrices are addressed with an explicit leading dimension (elements).
 *   - No global mutable state: re-entrant, safe from any host thread.
 */
#ifndef NGNN_H
#define NGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGNN_ABI_VERSION 21

/* error codes (negative); positive values are hipError_t */
#define NGNN_OK 0
#define NGNN_E_ARG (-1)        /* null pointer / negative size / bad enum   */
#define NGNN_E_DTYPE (-2)      /* unsupported dtype                          */
#define NGNN_E_SHAPE (-3)      /* F / leading dimension / size out of range  */
#define NGNN_E_ALIGN (-4)      /* pointer alignment not supported            */
#define NGNN_E_RANGE (-5)      /* N or E does not fit int32                  */
#define NGNN_E_WORKSPACE (-6)  /* workspace too small                        */

/* reductions: PyG `aggr` names (utils/scatter.py [ext]) */
#define NGNN_REDUCE_SUM 0  /* GCNConv aggr='add'                             */
#define NGNN_REDUCE_MEAN 1 /* SAGEConv default aggr='mean' (sage.py:16-19)   */
#define NGNN_REDUCE_MAX 2  /* SAGEConv(aggr='max'): build extension          */
/* math-mode flag OR-ed into ngnn_sage_fwd_raw's `reduce`: the root term
 * x . W_r^T on exact fp32 MFMA (v_mfma_f32_16x16x4_f32, a fmaf chain) instead
 * of the default fp32-accurate 3 x bf16 split. */
#define NGNN_MATH_EXACT_F32 0x100
/* flag OR-ed into ngnn_sage_fwd_raw's `reduce` (MEAN / SUM, no ReLU, no
 * dropout, agg_out == NULL: an output layer): aggregate the neighbour term in
 * the F_out-wide space -- z = x W_l^T for every row in the same launch as the
 * root term (ws holds z: n_rows x ceil16(F_out) floats), then out[d] +=
 * mean/sum_{j -> d} z[j] for the rows below n_edge_rows.  Equal to
 * W_l . mean(x_j) up to fp32 rounding (the aggregation is linear); the
 * K-wide gather becomes an F_out-wide one.  Other cases run the fused path. */
#define NGNN_FWD_NARROW 0x200
/* flag OR-ed into ngnn_sage_fwd_raw's `reduce`: x (and x_dev's rows) are
 * bf16 [*, ldx] (ldx in elements, a multiple of 4; 16-B aligned base).  The
 * rows are read as bf16 -- half the bytes of the fp32 layout -- and widened
 * exactly: the split-bf16 root term needs one part (3 products), the gather
 * sums in fp32.  Outputs (unless NGNN_OUT_BF16), z and agg_out stay fp32.  Not
 * with NGNN_MATH_EXACT_F32 (NGNN_E_SHAPE: convert x and call again). */
#define NGNN_X_BF16 0x400
/* flag OR-ed into ngnn_sage_fwd_raw's `reduce`: the weights (W_r, and W_l of
 * NGNN_FWD_NARROW) hold bf16-exact values -- a bf16 model's parameters
 * (sage.py:40 under model.to(torch.bfloat16)) widened to fp32.  The split-bf16
 * root term then needs ONE weight part (its other two parts are zero): the
 * LDS image is a third of the size (wider column slices, fewer re-reads of x)
 * and each 32-deep chunk issues 3 MFMAs (1 with NGNN_X_BF16) instead of 6.
 * The result is bitwise the one without the flag on such weights (the
 * skipped products are exact zeros); weights that are not bf16-exact are
 * rounded to bf16.  MEAN / SUM only (NGNN_E_SHAPE otherwise: call without). */
#define NGNN_W_BF16 0x800
/* flag OR-ed into ngnn_sage_fwd_raw's `reduce`: `ws` already holds
 * ngnn_pack_weight(wl) (a producer packed this step's W_l: the graph slot's
 * load, ngnn_slot_load's pack job), so a layer whose W_l streams from L2
 * issues no pack launch of its own; ignored when W_l is staged in LDS. */
#define NGNN_WL_PREPACKED 0x1000
/* flag OR-ed into ngnn_sage_fwd_raw's `reduce`: `out` holds bf16 [n_rows,
 * ldo] (ldo in elements, a multiple of 4; 8-B aligned), each output rounded to
 * nearest even after bias, ReLU and dropout -- a bf16 model's hidden
 * activations, which the reference's bf16 layer stores in bf16 too.  Whole
 * 16-column output tiles only; not with NGNN_FWD_NARROW or the wide path
 * (NGNN_E_SHAPE: call without and convert). */
#define NGNN_OUT_BF16 0x2000

/* dtypes */
#define NGNN_F32 0
#define NGNN_BF16 1

int ngnn_abi_version(void);
const char *ngnn_strerror(int rc);

/* ------------------------------------------------------------------ edges
 * Validate a PyG edge_index [2,E] int64 (row 0 = source, row 1 = target,
 * flow source_to_target) before any kernel indexes with it.
 * status (device int32[4], caller zeroes it):
 *   [0] != 0  some source id outside [0, n_src)
 *   [1] != 0  some target id outside [0, n_dst)
 *   [2] != 0  targets are NOT non-decreasing (needs the sorting CSR path)
 *   [3] != 0  sources are NOT non-decreasing
 * Replaces PyG's implicit index checks in index_select / scatter [ext]
 * (reached from sage.py:34 / convolution.py:31). */
int ngnn_edge_probe(const int64_t *edge_index, int64_t E, int64_t n_src, int64_t n_dst,
                    int32_t *status, void *stream);

/* Workspace bytes ngnn_csr_build needs for the unsorted path. */
size_t ngnn_csr_workspace_bytes(int64_t E, int64_t n_rows);

/* Group the E edges by `keys` (int64, values in [0,n_rows)) into CSR:
 *   rowptr[n_rows+1] (int32), col[E] = vals in grouped order (int32),
 *   eid[E] = original edge position (int32, nullable).
 * Grouping is STABLE (edge order kept inside a row), so per-row reductions
 * run in the same order as PyG's CPU scatter_add_ / index_add_.
 * keys_sorted=1 claims keys are non-decreasing (fast path, no workspace);
 * keys_sorted=0 uses a stable radix sort in `ws`.
 * Forward CSR: keys = edge_index[1] (targets), vals = edge_index[0].
 * Transposed CSR for the backward gather: keys = edge_index[0], vals = edge_index[1]. */
int ngnn_csr_build(const int64_t *keys, const int64_t *vals, int64_t E, int64_t n_rows,
                   int keys_sorted, int32_t *rowptr, int32_t *col, int32_t *eid,
                   void *ws, size_t ws_bytes, void *stream);

/* ------------------------------------------------------------ aggregation
 * out[i, :F] = reduce_{e in rowptr[i]..rowptr[i+1]} x[col[e], :F]
 * SUM : edge-order fp32 sum; MEAN: sum / max(deg,1) (IEEE division);
 * MAX : NaN-propagating max, empty rows -> 0 (scatter_reduce amax,
 *       include_self=False on a zero tensor).
 * Replaces PyG MessagePassing.propagate (gather x_j + utils.scatter) [ext].
 * dtype NGNN_BF16: x holds bf16 rows (F, ldx multiples of 4; 8-B aligned),
 * widened exactly; out stays fp32. */
int ngnn_seg_agg_fwd(const void *x, int64_t ldx, int64_t F, const int32_t *rowptr,
                     const int32_t *col, int64_t n_dst, int reduce, int dtype,
                     void *out, int64_t ldo, void *stream);

/* grad_x[j, :F] = sum over edges e with source j (transposed CSR, edge
 * order) of  SUM : g[dst_e]   MEAN: g[dst_e] / max(deg(dst_e),1)
 *            MAX : [x[j]==agg[dst_e]] * g[dst_e] / ties(dst_e)
 * where ties = #tied sources + [agg == 0] (torch scatter_reduce amax
 * backward, FunctionsManual.cpp [ext]).  grad_x is fully overwritten
 * (rows with no out-edges get 0).  For MAX, `ws` must hold n_dst*F floats
 * (ngnn_seg_agg_bwd_workspace_bytes) and x/agg/rowptr/col (forward CSR)
 * are required; for SUM/MEAN they may be NULL except rowptr (degrees). */
size_t ngnn_seg_agg_bwd_workspace_bytes(int64_t n_dst, int64_t F, int reduce);
int ngnn_seg_agg_bwd(const void *grad_out, int64_t ldg, int64_t F,
                     const int32_t *rowptr, const int32_t *col, int64_t n_dst,
                     const int32_t *rowptr_t, const int32_t *col_t, int64_t n_src,
                     int reduce, int dtype, const void *x, int64_t ldx,
                     const void *agg, int64_t lda, void *grad_x, int64_t ldgx,
                     void *ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------- sampling
 * One hop of uniform neighbour sampling without replacement (PyG
 * NeighborLoader / pyg-lib neighbor_sample semantics [ext], constructed at
 * pipeline.py:75-83): for frontier node v (global id) with in-degree d,
 * take min(d, fanout) distinct in-neighbours from graph CSR
 * (g_rowptr int64[N+1], g_col int32[nnz]) in Floyd order.
 *   out_nbr[i*fanout + k] = global neighbour id (or -1 past the count),
 *   out_cnt[i]            = number taken.
 * Deterministic in (seed, frontier position). */
int ngnn_sample_hop(const int64_t *g_rowptr, const int32_t *g_col, const int64_t *frontier,
                    int64_t n_frontier, int fanout, uint64_t seed, int64_t *out_nbr,
                    int32_t *out_cnt, void *stream);

/* ------------------------------------------------- whole-block sampling
 * The whole NeighborLoader mini-batch on the device: every hop of
 * ngnn_sample_hop's sampler (hop h uses seed*1000003 + h), the relabelling
 * of sampled global ids to block-local ids and the block's edge list --
 * what PyG's NeighborLoader (pipeline.py:75-83, pyg-lib neighbor_sample
 * [ext]) builds in its worker process plus the batch.to(device) of
 * pipeline.py:153.  Local ids: seeds first (seeds must be distinct), then
 * each hop's newly reached nodes in order of first appearance in the hop's
 * (frontier position, draw) sequence.  Edges: row 0 = local source (the
 * sampled neighbour), row 1 = local target, grouped by target in frontier
 * order (targets non-decreasing).
 *
 * Two calls.  ngnn_sample_block runs the hops and writes
 * counts (device int32[4]) = {n_nodes, n_edges, n_active, 0}, n_active =
 * rows that received in-edges (the frontiers of hops < last); the caller
 * reads them (one device->host copy), allocates the outputs and calls
 * ngnn_sample_block_finish with the same fanouts / seeds count / workspace,
 * which writes n_id int64[n_nodes], edge_index int64[2, n_edges]
 * (contiguous), optionally y = y_all[n_id] and x = x_all[n_id] (fp32 rows),
 * and restores node_map.
 *   node_map: int32[2 * n_graph], caller-owned, all -1 before the first call
 *             and again after every finish (one map per stream at a time).
 *   ws:       ngnn_sample_block_workspace_bytes(batch, fanouts, n_hops);
 *             holds the block between the two calls.
 *   fanouts:  HOST int32[n_hops], each 0..64.
 * ABI 18: n_active (counts[2]) and, nullable as a pair, csr_rowptr
 * int32[n_nodes + 1] / csr_col int32[n_edges]: the block's target-grouped
 * CSR (edge order kept inside a row; col = the local sources), taken from the
 * relabelling itself, so a consumer of the block builds none.  The hops run
 * as three launches each (one lane per draw: draws + claims; first-
 * appearance counts; the relabelling writes) and the outputs, x rows
 * included, as one.
 * ABI 19: counts_dev (nullable): the counts array ngnn_sample_block wrote,
 * read on the DEVICE -- no host read-back: n_nodes / n_edges / n_active are
 * then the capacities the outputs are sized for (the plan's n_cap / e_cap
 * at most) and bound the device counts; the first counts[0] rows / counts[1]
 * edges are written.  edge_index's row stride is n_edges in both modes (the
 * capacity here).  With ngnn_slot_load's counts_dev this is NeighborLoader's
 * sync-free pipeline (no host wait per batch). */
size_t ngnn_sample_block_workspace_bytes(int64_t batch, const int32_t *fanouts, int n_hops);
int ngnn_sample_block(const int64_t *g_rowptr, const int32_t *g_col, int64_t n_graph,
                      const int64_t *seeds, int64_t n_seeds, const int32_t *fanouts, int n_hops,
                      uint64_t seed, int32_t *node_map, void *ws, size_t ws_bytes,
                      int32_t *counts, void *stream);
int ngnn_sample_block_finish(const int32_t *fanouts, int n_hops, int64_t n_seeds,
                             int64_t n_nodes, int64_t n_edges, int32_t *node_map,
                             int64_t n_graph, const void *ws, size_t ws_bytes, int64_t *n_id,
                             int64_t *edge_index, const int64_t *y_all, int64_t *y,
                             const float *x_all, int64_t ldx, int64_t F, float *x, int64_t ldo,
                             int64_t n_active, int32_t *csr_rowptr, int32_t *csr_col,
                             const int32_t *counts_dev, void *stream);

/* ------------------------------------------------------ co-teaching loss
 * CTLoss.forward (src/utils/losses.py:19-49) without its two host argsorts:
 * for models m = 1, 2 with logits y_m [B, C] (row stride ld_m) and noisy
 * labels y_noise int64[B]:
 *   l_m[r]       = cross_entropy(y_m[r], y_noise[r])  (0 if ignore_index)
 *   ind_m_sorted = argsort(l_m) ascending, ties by row index, NaN last
 *                  (np.argsort(loss_m) of losses.py:22,26)
 *   out[0] = mean_{r in ind_2_sorted[:R]} l_1[r]   (loss_1_update, :44)
 *   out[1] = mean_{r in ind_1_sorted[:R]} l_2[r]   (loss_2_update, :45)
 *   out[2] = sum noise_or_not[ind[ind_1_sorted[:R]]] / R  (pure_ratio_1, :33)
 *   out[3] = same for model 2 (NaN when noise_or_not is NULL)
 * with R = num_remember (losses.py:31), ind = the batch's n_id (NULL = row
 * ids), noise_or_not bool (uint8) [n_noise]; an index outside it sets *err
 * (device int, caller-zeroed) and contributes nothing.  B <= 8192.
 * ngnn_ct_loss_bwd: d y_m = grad_m / #valid (softmax - onehot) on the rows
 * the other model kept, 0 on every other row of [0, B) -- the autograd of
 * out[m-1]; model = 0 or 1.  ws: ngnn_ct_loss_workspace_bytes(B), kept
 * between the forward and both backwards. */
size_t ngnn_ct_loss_workspace_bytes(int64_t B);
int ngnn_ct_loss_fwd(const float *y1, int64_t ld1, const float *y2, int64_t ld2, int64_t B,
                     int64_t C, const int64_t *y_noise, int64_t ignore_index, int64_t num_remember,
                     const int64_t *ind, const uint8_t *noise_or_not, int64_t n_noise, float *out,
                     int64_t *ind1_sorted, int64_t *ind2_sorted, void *ws, size_t ws_bytes,
                     int *err, void *stream);
int ngnn_ct_loss_bwd(int model, const float *y, int64_t ld, int64_t B, int64_t C,
                     const int64_t *y_noise, int64_t ignore_index, const void *ws,
                     const float *grad, float *dy, int64_t ldd, void *stream);

/* ------------------------------------------------------- fused SAGE layer
 * One SAGEConv layer of SAGE.forward (sage.py:33-39) in one launch:
 *   out[r] = act( b + x[r] . W_r^T + [deg(r)>0] agg(r) . W_l^T ),   r < n_rows
 * agg(r) = reduce over the CSR row r of x (MEAN / SUM / MAX as in
 * ngnn_seg_agg_fwd, bit-identical); act = optional ReLU then optional
 * dropout with keep probability 1-p_drop and scale 1/(1-p_drop), drawn from a
 * counter-based hash of (seed, r, c) (no mask tensor; backward uses out > 0).
 * W_l / W_r are the PyG Linear weights [Fo, K] packed by ngnn_pack_weight;
 * wl_packed may be NULL (no neighbour term; rowptr/col may then be NULL).
 * bias may be NULL.  x, out fp32 (outputs wider than 512 columns run as
 * several launches of 512-column slices); exact fp32 MFMA
 * (v_mfma_f32_16x16x4_f32).  Optional modes:
 *   n_rows_dev  device int: rows = min(n_rows, *n_rows_dev) (rows past it are
 *               not written) -- bounds that only the device knows;
 *   agg_out     [n_rows, ld_agg]: workgroups whose 64 rows have in-edges also
 *               store those rows' aggregate (saved for the backward);
 *   xmask       stage x * (xmask > 0 ? xscale : 0) instead of x (ReLU/dropout
 *               backward fused into a dgrad GEMM's input);
 *   seed_dev    device uint64 XORed into `seed` when the kernel starts, so a
 *               captured HIP graph draws a fresh dropout mask per replay (the
 *               graph increments it); NULL = the host seed alone.
 * Replaces PyG SAGEConv.forward [ext] + relu + F.dropout. */
size_t ngnn_pack_weight_bytes(int64_t Fo, int64_t K);
int ngnn_pack_weight(const float *w, int64_t ldw, int64_t Fo, int64_t K, void *packed,
                     void *stream);
/* Pack M[Fo][K] = rows [0,rows0) from w0, rows [rows0,Fo) from w1 (either
 * read transposed: M[n][k] = src[k][n]).  The backward packs
 * [W_l^T ; W_r^T] for its dgrad GEMM. */
int ngnn_pack_weight_ex(const float *w0, const float *w1, int64_t ldw, int64_t rows0, int64_t Fo,
                        int64_t K, int transposed, void *packed, void *stream);
int ngnn_sage_fwd(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                  const int32_t *n_rows_dev, const int32_t *rowptr, const int32_t *col, int reduce,
                  const void *wl_packed, const void *wr_packed, const float *bias, int64_t Fo,
                  float *out, int64_t ldo, int relu, float p_drop, uint64_t seed,
                  const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, const float *xmask,
                  int64_t ldm, float xscale, void *stream);

/* Same layer with the RAW PyG Linear weights (W_l, W_r: [Fo, K] row-major,
 * row stride ldw) through the row-tile kernel (ngnn_sage_rt.hip, the model's
 * path).  Root term x . W_r^T: by default fp32-accurate 3 x bf16 split MFMA
 * (each operand split v = v1 + v2 + v3 in bf16, the six products down to
 * 2^-18 of the leading one accumulated in fp32; error below the fp32
 * rounding of the reference GEMM); `reduce | NGNN_MATH_EXACT_F32` runs it on
 * exact fp32 MFMA.  The W_r image is built in LDS from these rows in the
 * kernel prologue (no pack launch); W_l (fp32, neighbour term of rows with
 * in-edges) shares the LDS when it fits, else it is packed into ws (one
 * launch) and streamed from L2.  Returns NGNN_E_SHAPE, launching nothing,
 * for shapes outside that kernel's envelope (K % 4 != 0, unaligned rows, W_r
 * slice too large for LDS, buffers >= 2 GiB): the caller then packs and calls
 * ngnn_sage_fwd.  x_dev (nullable): a device word holding x's address, read
 * at run time instead of x (a HIP-graph slot whose batch stays where the
 * loader put it; 16-B aligned, row stride ldx, rows < *n_rows_dev).
 * xrow / xrow_dev (nullable; the device word overrides): the fused
 * NeighborLoader feature gather -- logical row r of the layer input is row
 * xrow[r] (int64, the block's n_id) of x, the HBM-resident feature table of
 * x_rows rows (< 3.75 GiB), so x[n_id] is never materialised (pipeline.py:153
 * copies it per batch).  Root rows and gathered neighbour rows both go
 * through it; outputs and agg_out stay in block order.  col_x (nullable,
 * with xrow): col with every entry already mapped through xrow (the slot
 * load writes it), so the neighbour gather makes no dependent index load.
 * wr == NULL: no root term (GCNConv's form, see ngnn_gcn_agg_fwd; raw
 * weights only, not with NGNN_FWD_NARROW).
 * n_edge_rows / n_edge_rows_dev (device int, nullable, min'd with the
 * host value): rows at or past it have no in-edges (NGNN_FWD_NARROW's
 * gather stops there, and the row-tile kernel runs the tiles past it on its
 * root-term-only loop; NeighborLoader numbers the rows that receive edges
 * first).  Pass n_rows when unknown.
 * Wide layers (ngnn_sage_wide_preferred: K % 4 != 0, or F_out needing more
 * than four LDS column slices -- Amazon-Computers' 767 -> 512 layer) with
 * plain fp32 rows run as an aggregate launch over rows < n_edge_rows (into
 * agg_out, else ws) + a 2-D tiled exact-fp32 MFMA dual GEMM (ngnn_wide.hip).
 * ws: ngnn_sage_fwd_raw_workspace_bytes(K, Fo, n_rows) bytes (calls sharing
 * a ws must be stream-ordered); its last 160 KiB hold the launch's prebuilt
 * split-bf16 root image (k_x3_image) when the rest still fits the z rows /
 * packed W_l -- a smaller ws makes every workgroup build the image itself. */
size_t ngnn_sage_fwd_raw_workspace_bytes(int64_t K, int64_t Fo, int64_t n_rows);
/* 1 when ngnn_sage_fwd_raw runs a [K -> Fo] layer on the wide path (exact:
 * the NGNN_MATH_EXACT_F32 mode), else 0. */
int ngnn_sage_wide_preferred(int64_t K, int64_t Fo, int exact);
int ngnn_sage_fwd_raw(const float *x, const float *const *x_dev, const int64_t *xrow,
                      const int64_t *const *xrow_dev, int64_t x_rows, int64_t ldx, int64_t K,
                      int64_t n_rows, const int32_t *n_rows_dev, int64_t n_edge_rows,
                      const int32_t *n_edge_rows_dev, const int32_t *rowptr,
                      const int32_t *col, const int32_t *col_x,
                      int reduce, const float *wl, const float *wr, int64_t ldw, const float *bias,
                      int64_t Fo, float *out, int64_t ldo, int relu, float p_drop, uint64_t seed,
                      const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, void *ws,
                      size_t ws_bytes, void *stream);

/* Two-layer SAGE forward of the headline shape in three launches
 * (ngnn_fwd2.hip): sage.py:33-39 for
 * SAGE(K0, 256, F1, num_layers=2) -- conv0 -> relu -> dropout -> conv1 --
 * replacing two ngnn_sage_fwd_raw calls (the second with NGNN_FWD_NARROW).
 * Shape envelope (ngnn_sage2_supported): 96 < K0 <= 128, K0 % 4 == 0, hidden
 * H == 256, 32 < F1 <= 48, reduce MEAN or SUM.  Weights are the raw PyG
 * Linear matrices (lin_l / lin_r of each conv, rows of ldw0 / ldw1 floats).
 *   h   [n_rows, ldh]  = dropout(relu(b0 + x W_r0^T + agg(x) W_l0^T)); only
 *        rows < min(h_rows, *h_rows_dev) are written (the rows a bounded
 *        backward reads: pass n_rows to write all);
 *   agg0 [n_rows, ld_agg] = the layer-0 neighbour aggregate of the rows of
 *        the 16-row tiles below n_edge_rows (the backward's saved aggregate;
 *        bit-identical to ngnn_seg_agg_fwd);
 *   out [n_rows, F1]   = b1 + h W_r1^T + agg(h) W_l1^T (logits, every row;
 *        rows packed: ldo == F1, out 16-B aligned -- a 16-row tile of out is
 *        one contiguous block, stored as 16-B pieces).
 * Rows at or past min(n_edge_rows, *n_edge_rows_dev) must have no in-edges
 * (NeighborLoader numbers the rows that receive edges first; pass n_rows
 * when unknown).  x_dev (nullable): device word holding x's address (graph
 * slot), x then unused.  xrow / xrow_dev / x_rows / col_x: the fused
 * x[n_id] gather, as ngnn_sage_fwd_raw's (x is the x_rows-row feature table,
 * col_x = n_id[col]).  wr0 (nullable, ABI 17): no layer-0 root term --
 * SimpleGCN's GCNConv(normalize=False), aggregate first: x is then read
 * only through the neighbour aggregate (not with xrow / xrow_dev); pass a
 * zero W_r1 for its output layer.  Arithmetic: H2 (two fp16 parts per operand after
 * power-of-two scaling, three MFMA products), inside the fp32 parity bars.
 * stages: NGNN_SAGE2_ALL, or a subset in order (per-launch timing; the
 * workspace carries nb and z between stages): EDGE the aggregate + nb of
 * the rows with in-edges, MAIN every row's layer 0 + layer-1 products,
 * NARROW the z aggregate into out; PREP is accepted and does nothing (the
 * kernels load their weight slices themselves).
 * head (nullable, ABI 15): the seed-row cross entropy of the training step
 * (pipeline.py:158, F.cross_entropy(out[:B], y[:B]) -- ngnn_seed_xent_fwd_grad's
 * contract) computed by the NARROW launch from the logits it finishes, plus
 * the first step of the backward (see ngnn_xent_head).
 * ws: ngnn_sage2_workspace_bytes(K0, F1, n_rows), 256-B aligned. */
/* The loss head of ngnn_sage2_fwd (ABI 15).  For the logit rows d < B:
 *   loss   = sum_{d < B, y[d] != ignore_index} (lse(out[d]) - out[d][y[d]]) / count
 *   count  = #{d < B : y[d] != ignore_index}   (an out-of-range label: NaN loss)
 *   dy[d]  = (softmax(out[d]) - onehot(y[d])) / count   (0 for an ignored row)
 *            -- d loss / d out at unit scale, rows >= B not written;
 *   g[s]  += dy[d] (/ deg(d) for MEAN) for every edge s -> d, d < B (float
 *            atomics; exact zeros skipped): the narrow scatter ngnn_sage2_bwd
 *            runs first, already done -- pass g as its g_pre.  g [n_rows rows,
 *            C4 = ceil4(F1) floats]: its rows < min(g_rows, *g_rows_dev) are
 *            zeroed by the EDGE launch of the same call (so a head whose
 *            backward never runs leaves nothing behind); nullable (no scatter).
 * ws: ngnn_xent_head_workspace_bytes(B) bytes, 16-B aligned, zero-filled
 * before its first use (it is zero again on return).  The loss sum is in a
 * fixed order (deterministic); needs the EDGE and NARROW stages in one call
 * or in order, F1 <= 64.
 * src_count (nullable, ABI 17): 2 g_rows + 1 int32, zero-filled before its
 * first use and then owned by the head: the EDGE launch counts every source's
 * edges into rows d < B (two count arrays alternating per call, the word past
 * them selects one), so a source with a single such edge takes ONE plain row
 * store of dy[d] (/ deg(d)) instead of F1 float atomics.  Counts left over
 * from a call whose NARROW stage did not finish only ever over-count (the
 * scatter then stays atomic): any call order is safe. */
typedef struct ngnn_xent_head {
    const int64_t *y;
    int64_t B;
    int64_t ignore_index;
    float *loss, *count;
    float *dy;
    int64_t ldd;
    float *g;
    int64_t g_rows;
    const int32_t *g_rows_dev;
    void *ws;
    size_t ws_bytes;
    int32_t *src_count;
} ngnn_xent_head;
size_t ngnn_xent_head_workspace_bytes(int64_t B);
#define NGNN_SAGE2_PREP 1
#define NGNN_SAGE2_EDGE 2
#define NGNN_SAGE2_MAIN 4
#define NGNN_SAGE2_NARROW 8
#define NGNN_SAGE2_ALL 15
int ngnn_sage2_supported(int64_t K0, int64_t H, int64_t F1, int reduce);
size_t ngnn_sage2_workspace_bytes(int64_t K0, int64_t F1, int64_t n_rows);
int ngnn_sage2_fwd(const float *x, const float *const *x_dev, const int64_t *xrow,
                   const int64_t *const *xrow_dev, int64_t x_rows, int64_t ldx, int64_t K0,
                   int64_t n_rows, const int32_t *n_rows_dev, int64_t n_edge_rows,
                   const int32_t *n_edge_rows_dev, const int32_t *rowptr, const int32_t *col,
                   const int32_t *col_x, int reduce, const float *wl0, const float *bl0, const float *wr0,
                   int64_t ldw0, int64_t H, const float *wl1, const float *bl1,
                   const float *wr1, int64_t ldw1, int64_t F1, float p_drop, uint64_t seed,
                   const uint64_t *seed_dev, float *h, int64_t ldh, int64_t h_rows,
                   const int32_t *h_rows_dev, float *agg0, int64_t ld_agg, float *out,
                   int64_t ldo, const ngnn_xent_head *head, int stages, void *ws, size_t ws_bytes,
                   void *stream);

/* Every weight gradient of the two-layer stack above in three launches
 * (ngnn_bwd2.hip): the backward of sage.py:33-39 under
 * loss.backward() when the loss reads logit rows < *r_ptr (the seed rows,
 * pipeline.py:155-160), replacing ngnn_seg_agg_fwd + two ngnn_sage_wgrad +
 * ngnn_sage_dgrad_lowdim.  With g[s] = sum over edges s -> d (d < R) of
 * dy[d] (/ deg(d) for MEAN), over rows < R' = max(R, *rnext_ptr):
 *   dW_l1 = g^T h, dW_r1 = dy^T h, db1 = sum dy            ([F1, 256], [F1])
 *   dz0 = (dy W_r1 + g W_l1) * [h > 0] * yscale            (on chip only)
 *   dW_l0 = dz0^T agg0, dW_r0 = dz0^T x, db0 = sum dz0     ([256, K0], [256])
 * dy [*, ldy] (rows < R read), h [*, ldh] / agg0 [*, ld_agg] the forward's
 * (rows < R' read; an edgeless row's aggregate counts as 0), x / x_dev /
 * xrow / xrow_dev / x_rows as ngnn_sage2_fwd's (row r of layer 0's input).
 * Arithmetic (round 5): H2 -- two fp16 parts per operand after a
 * power-of-two scaling per 32-row chunk, three MFMA products per product
 * (relative ~2^-22), fp32 accumulation -- inside the fp32 weight-gradient
 * bars (1e-5 of each tensor's max).  F1 <= 48, 0 < K0 <= 128, K0 % 4 == 0; weights [F1, 256] rows of
 * ldw1 floats.  ws: ngnn_sage2_bwd_workspace_bytes(n_rows, K0, F1), 256-B
 * aligned, ZERO-FILLED before its first use (g's part is zero again on
 * return; its offset depends on K0 and F1 only, so a zeroed workspace may be
 * grown for more rows).  Float atomics
 * build g: not bitwise reproducible run to run (as the reference's CUDA
 * index_add_).  g_pre (nullable, ABI 15): g already built (ngnn_sage2_fwd's
 * loss head, [n_rows, ceil4(F1)]): no scatter launch, g read from it.
 * adam (nullable, ABI 15): the optimizer step folded into the reduction --
 * every parameter updated from its gradient as ngnn_adam_step would (same
 * arithmetic, the same device step count advanced once); the gradients are
 * still written.  For a training step whose gradients need no exchange
 * (one rank) and whose optimizer holds exactly these six tensors. */
typedef struct ngnn_adam_fold {
    /* in the order dW_l1, db1, dW_r1, dW_l0, db0, dW_r0 (the gradient order) */
    float *param[6], *exp_avg[6], *exp_avg_sq[6];
    float *step; /* the device step count (advanced once, then read) */
    float lr, beta1, beta2, eps, weight_decay;
    /* ABI 20 (nullable): ngnn_slot_load's contract gate and the slot's r_next
     * word -- a step whose block broke the slot's contract updates no
     * parameter and leaves the step count (the gradients are still written) */
    const uint64_t *gate;
    const int64_t *gate_gen;
} ngnn_adam_fold;
size_t ngnn_sage2_bwd_workspace_bytes(int64_t n_rows, int64_t K0, int64_t F1);
int ngnn_sage2_bwd(const float *dy, int64_t ldy, int64_t F1, const float *wl1, const float *wr1,
                   int64_t ldw1, const float *h, int64_t ldh, float yscale, const float *x,
                   const float *const *x_dev, const int64_t *xrow, const int64_t *const *xrow_dev,
                   int64_t x_rows, int64_t ldx, int64_t K0, const float *agg0, int64_t ld_agg,
                   const int32_t *rowptr, const int32_t *col, int64_t n_rows, const int32_t *r_ptr,
                   const int32_t *rnext_ptr, int reduce, float *dwl1, float *dbl1, float *dwr1,
                   float *dwl0, float *dbl0, float *dwr0, const float *g_pre, const ngnn_adam_fold *adam,
                   void *ws, size_t ws_bytes, void *stream);

/* GCNConv(normalize=False) layer (convolution.py:19-35; PyG GCNConv [ext]):
 * out = act(A (x W^T) + b), A the target-grouped sum over in-edges.  The
 * fused path runs it as SAGE with W_r = 0 (linear aggregation: A x W^T ==
 * (A x) W^T up to fp32 rounding): aggregate-first through
 * ngnn_sage_fwd_raw(wr = NULL, wl = W, reduce = SUM) when F_in <= F_out,
 * else transform-first: z = x W^T through ngnn_sage_fwd_raw(wl = NULL, wr =
 * W, bias = NULL) into z [n_rows, ldz], then this launch:
 *   out[d] = act(sum_{e into d, edge order} z[col[e]] + b)   for every row
 *   d < min(n_rows, *n_rows_dev) (act = ReLU + quad-hash dropout as the
 *   row-tile epilogue; rows without in-edges get act(b)).
 * ldz >= ceil4(Fo), z 16-B aligned. */
int ngnn_gcn_agg_fwd(const float *z, int64_t ldz, int64_t Fo, const int32_t *rowptr,
                     const int32_t *col, int64_t n_rows, const int32_t *n_rows_dev,
                     const float *bias, int relu, float p_drop, uint64_t seed,
                     const uint64_t *seed_dev, float *out, int64_t ldo, void *stream);

/* ------------------------------------------ backward receptive-field bounds
 * ngnn_row_extent: out[0] = max(out[0], 1 + last row of g[n_rows, F] holding a
 * nonzero (or NaN)).  The reference's loss reads only the seed rows
 * (pipeline.py:155 slices [:batch_size]), so the output gradient is zero past
 * them and every backward product can stop at that row.
 * ngnn_block_prefix_stats: R = *r_ptr (device);  *r_next = max(*r_next, R,
 * 1 + max col[0..rowptr[R]))  = rows of the input gradient that can be
 * nonzero;  *nnz_out = rowptr[R] (nullable).  E bounds the sweep. */
int ngnn_row_extent(const float *g, int64_t ld, int64_t n_rows, int64_t F, int32_t *out,
                    void *stream);
int ngnn_block_prefix_stats(const int32_t *rowptr, const int32_t *col, const int32_t *r_ptr,
                            int32_t *nnz_out, int32_t *r_next, int64_t E, void *stream);

/* ------------------------------------------------- fused SAGE layer backward
 * Weight gradients over rows r < R = *r_ptr (device):
 *   dz = dy (* [y > 0] * yscale when y != NULL: ReLU+dropout backward)
 *   dW_r = dz^T h,  dW_l = dz^T agg (agg: the forward's saved aggregate; rows
 *   with no in-edges read as 0),  db = sum_r dz.
 * fp32 MFMA over 64-row chunks, per-slice partials in ws, fixed-order
 * reduction => deterministic.  Outputs are overwritten.
 * Replaces autograd of lin_l / lin_r (PyG Linear [ext]) in SAGEConv. */
size_t ngnn_sage_wgrad_workspace_bytes(int64_t Fo, int64_t K);
/* h_dev (nullable): device word holding h's address, read at run time (as
 * ngnn_sage_fwd_raw's x_dev). */
/* h_idx / h_idx_dev (nullable; the device word overrides): row r of h is
 * row h_idx[r] of h, a table of h_rows rows (< 2 GiB) -- layer 0 under the
 * fused x[n_id] gather (see ngnn_sage_fwd_raw's xrow).  bf16_flags: bit 0
 * (NGNN_WG_H_BF16) h holds bf16 (a bf16 model's layer input, as
 * ngnn_sage_fwd_raw's NGNN_X_BF16; K and ldh multiples of 4); bit 1
 * (NGNN_WG_Y_BF16) the mask rows y hold bf16 (a bf16 model's hidden
 * activations, NGNN_OUT_BF16); both widened exactly when staged. */
#define NGNN_WG_H_BF16 1
#define NGNN_WG_Y_BF16 2
int ngnn_sage_wgrad(const float *dy, int64_t ldy, const float *y, int64_t ldyy, float yscale,
                    const float *h, const float *const *h_dev, const int64_t *h_idx,
                    const int64_t *const *h_idx_dev, int64_t h_rows, int bf16_flags, int64_t ldh,
                    const float *agg, int64_t ld_agg, const int32_t *rowptr, int64_t n_rows,
                    const int32_t *r_ptr,
                    int64_t Fo, int64_t K, float *dwl, float *dbl, float *dwr, void *ws,
                    size_t ws_bytes, void *stream);
/* Input gradient of one layer, rows j < Rn = *rnext_ptr (R = *r_ptr):
 *   dh[j] = [j < R] droot[j] + sum over edges e with source j and target
 *           d = col_t[e] < R (transposed CSR, edge order) of
 *           MEAN: dagg[d] / deg(d)   SUM: dagg[d]
 *           MAX : [h[j] == agg[d]] * dagg[d] / ties(d)   (torch amax rule)
 * droot = dz W_r and dagg = dz W_l come from the dgrad GEMM (ngnn_sage_fwd
 * with packed [W_l^T ; W_r^T]).  Rows >= Rn are zeroed if zero_tail, else
 * left untouched.  MAX needs ws of n_rows*K floats
 * (ngnn_sage_dgrad_workspace_bytes).  Replaces autograd of index_select +
 * scatter (PyG propagate [ext]). */
size_t ngnn_sage_dgrad_workspace_bytes(int64_t n_rows, int64_t K, int reduce);
int ngnn_sage_dgrad_gather(const float *dagg, int64_t ld_dagg, const float *droot,
                           int64_t ld_droot, const int32_t *rowptr, const int32_t *col,
                           const int32_t *rowptr_t, const int32_t *col_t, int64_t n_rows,
                           const int32_t *r_ptr, const int32_t *rnext_ptr, int64_t K, int reduce,
                           const float *h, int64_t ldh, const float *agg, int64_t ld_agg,
                           float *dh, int64_t ldd, int zero_tail, void *ws, size_t ws_bytes,
                           void *stream);
/* Same result through float atomics instead of the source-grouped CSR (no
 * per-batch sort): dh[j] = [j < R] droot[j] for j < Rn, then every edge
 * (j -> d), d < R, adds its term into dh[j] (one 256-B atomic wave-instruction
 * per edge and 64 columns).  Summation order is not fixed (as with the
 * reference's CUDA index_add_); the gather variant is the deterministic one.
 * rowptr/col: target-grouped CSR. */
int ngnn_sage_dgrad_scatter(const float *dagg, int64_t ld_dagg, const float *droot,
                            int64_t ld_droot, const int32_t *rowptr, const int32_t *col,
                            int64_t n_rows, const int32_t *r_ptr, const int32_t *rnext_ptr,
                            int64_t K, int reduce, const float *h, int64_t ldh, const float *agg,
                            int64_t ld_agg, float *dh, int64_t ldd, int zero_tail, void *stream);
/* The whole atomic input-gradient path of one layer in two launches, no dgrad
 * GEMM: zero dh rows < Rn, then one wave per target row d < R computes
 * dz[d] = dy[d] (* [y>0] * yscale), dz[d] W_r (atomically into dh[d]) and
 * dz[d] W_l (scaled as in ngnn_sage_dgrad_gather, atomically into every
 * in-neighbour's row).  wl / wr: the raw PyG weights [Fo, K].  Fo <= 512. */
int ngnn_sage_dgrad_fused(const float *dy, int64_t ldy, const float *y, int64_t ldyy,
                          float yscale, const float *wl, const float *wr, int64_t Fo, int64_t K,
                          const int32_t *rowptr, const int32_t *col, int64_t n_rows,
                          const int32_t *r_ptr, const int32_t *rnext_ptr, int reduce,
                          const float *h, int64_t ldh, const float *agg, int64_t ld_agg,
                          float *dh, int64_t ldd, int zero_tail, void *stream);

/* Input gradient for MEAN / SUM when Fo < K, aggregating in the narrow
 * space (the aggregation is linear):
 *   g[j]  = sum over edges (j -> d), d < R, of dz[d] (MEAN: / deg(d))
 *           (Fo-wide float atomics; dz = dy (* [y > 0] * yscale))
 *   dh[j] = [j < R] dz[j] W_r + g[j] W_l   for j < Rn    (one MFMA pass)
 * = ngnn_sage_dgrad_fused's result up to fp32 summation order, with Fo/K of
 * its atomics and no zero-fill of dh.  wl / wr: raw PyG weights [Fo, K],
 * row stride ldw.  ws: ngnn_sage_dgrad_lowdim_workspace_bytes(n_rows, Fo, K)
 * bytes, 16-B aligned, ZERO-FILLED before its first use and dedicated to one
 * (Fo, K) pair: [packed W image | g], g = [n_rows][Fo rounded up to 4]
 * floats; every call leaves g zero again.  Rows >= Rn of dh are zeroed if zero_tail, else untouched.
 * NGNN_E_SHAPE when the weight image does not fit the LDS budget (callers
 * use ngnn_sage_dgrad_fused then).  Replaces autograd of lin_l + propagate
 * (sage.py:34, PyG SAGEConv [ext]). */
size_t ngnn_sage_dgrad_lowdim_workspace_bytes(int64_t n_rows, int64_t Fo, int64_t K);
int ngnn_sage_dgrad_lowdim(const float *dy, int64_t ldy, const float *y, int64_t ldyy,
                           float yscale, const float *wl, const float *wr, int64_t ldw, int64_t Fo,
                           int64_t K, const int32_t *rowptr, const int32_t *col, int64_t n_rows,
                           const int32_t *r_ptr, const int32_t *rnext_ptr, int reduce, float *dh,
                           int64_t ldd, int zero_tail, void *ws, size_t ws_bytes, void *stream);

/* ------------------------------------------------------ seed-row loss
 * Mean cross entropy of the first B rows of logits [*, C] (row stride ld)
 * against labels y[0..B), rows whose label == ignore_index excluded (torch
 * reduction='mean' semantics):  loss = sum (lse(x_r) - x_r[y_r]) / count.
 * Writes *loss and *count (device floats).  Deterministic.  The backward
 * writes dlogits rows < B = g (softmax(x_r) - onehot(y_r)) / count with
 * g = *grad_scale (0 for ignored rows) and leaves rows >= B untouched.
 * Replaces F.cross_entropy(out[:batch_size], y[:batch_size]) in the
 * reference's training loop (pipeline.py:158) and its autograd. */
size_t ngnn_seed_xent_workspace_bytes(int64_t B);
/* ws: ngnn_seed_xent_workspace_bytes(B), 16-B aligned (row losses; calls
 * sharing a ws must be stream-ordered).  The backward takes the same ws
 * (reserved) and recomputes the row log-sum-exps. */
int ngnn_seed_xent_fwd(const float *logits, int64_t ld, int64_t B, int64_t C, const int64_t *y,
                       int64_t ignore_index, float *loss, float *count, void *ws,
                       size_t ws_bytes, void *stream);
/* Forward and the unit-scale input gradient in ONE launch (the captured
 * training step's loss.backward(1)): writes *loss, *count and dlogits rows
 * < B = (softmax(x_r) - onehot(y_r)) / count (zeros for ignored rows); rows >=
 * B untouched.  The loss sum is the last workgroup's fixed-order sum of the
 * workgroups' partial sums (device ticket in ws, zero on entry, reset on exit):
 * deterministic.  ws as ngnn_seed_xent_fwd (zero-filled once).  Replaces
 * F.cross_entropy(out[:bs], y[:bs]) + its backward (pipeline.py:158,167). */
int ngnn_seed_xent_fwd_grad(const float *logits, int64_t ld, int64_t B, int64_t C,
                            const int64_t *y, int64_t ignore_index, float *loss, float *count,
                            float *dlogits, int64_t ldd, void *ws, size_t ws_bytes, void *stream);
int ngnn_seed_xent_bwd(const float *logits, int64_t ld, int64_t B, int64_t C, const int64_t *y,
                       int64_t ignore_index, const void *ws, const float *grad_scale,
                       const float *count, float *dlogits, int64_t ldd, void *stream);

/* ------------------------------------------------------------- optimiser
 * Adam step over n_tensors parameter tensors (host arrays of device
 * pointers; grads, exp_avgs, exp_avg_sqs like params, numels their sizes),
 * torch.optim.Adam's rule (amsgrad/maximize off, optional L2 weight decay),
 * with the step count a device float that this call advances (so a captured
 * HIP graph replays correctly).  ticket (nullable): 1024 device uint32 (ABI
 * 21; 64 in ABI 17-20, one before), zero before the first call, that the
 * update's workgroups count themselves on in two levels (each group's word
 * on a 128-B line of its own); the last one advances *step and every
 * word is zero again on return (one launch per call instead of an update +
 * increment pair; up to 16 tensors).  dtypes (host, nullable
 * = all NGNN_F32): per tensor NGNN_F32 or NGNN_BF16 (params and grads in that
 * dtype; exp_avgs / exp_avg_sqs always fp32).  Replaces the reference's
 * torch.optim.Adam(...).step() (model.py:66-69). */
/* dst[i] = bf16(src[i]) (round to nearest even, NaN kept) for i < n: a bf16
 * model's fp32 logits handed back in bf16 (Tensor.to(torch.bfloat16), the
 * `SAGE.forward` return dtype of a bf16 model).  src 16-B, dst 8-B aligned. */
int ngnn_cast_f32_bf16(const float *src, void *dst, int64_t n, void *stream);
/* The same over rows < min(n_rows, *n_rows_dev) of row_elems contiguous
 * elements each (n_rows_dev nullable): a graph slot's logits, cast for the
 * block's real rows only (ABI 15). */
int ngnn_cast_f32_bf16_rows(const float *src, void *dst, int64_t n_rows, int64_t row_elems,
                            const int32_t *n_rows_dev, void *stream);
/* n <= 16 tensors cast in one launch: to_bf16 = 0: dst[k][i] = float(src[k]
 * [i]) (bf16 -> fp32, exact); 1: dst[k][i] = bf16(src[k][i]) (round to
 * nearest even, NaN kept), i < numels[k] -- a bf16 model's parameters widened
 * for the fused kernels and their fp32 gradients narrowed back (Tensor.float()
 * and its autograd backward, one ATen copy kernel per tensor). */
int ngnn_cast_tensors(int n, const void *const *src, void *const *dst, const int64_t *numels,
                      int to_bf16, void *stream);
/* ABI 18: n <= 16 tensors of mixed dtypes in one launch: dst[k][i] =
 * cast(src[k][i]) / divisor (src_dtypes / dst_dtypes: host arrays of NGNN_F32
 * or NGNN_BF16 per tensor; bf16 -> fp32 exact, fp32 -> bf16 round to nearest
 * even; divisor 1: no division, otherwise the IEEE quotient as Tensor.div_;
 * src[k] == dst[k] allowed when the dtypes agree: in place) -- the
 * data-parallel gradient bucket's pack (each parameter's gradient into the
 * flat fp32 bucket) and unpack (bucket / world back into bf16 gradients and
 * in place into the fp32 ones that are bucket views): the copies and the
 * div_ of DistributedDataParallel's bucket path (pipeline.py:167-169 under
 * seed-sharded DP) as one launch each way. */
int ngnn_cast_tensors_ex(int n, const void *const *src, void *const *dst, const int64_t *numels,
                         const int32_t *src_dtypes, const int32_t *dst_dtypes, float divisor,
                         void *stream);
/* dst[r, :F] = float(src[r, :F]) (bf16 -> fp32, exact) for rows r <
 * min(n_rows, *n_rows_dev) (n_rows_dev nullable): the rows of a bf16 model's
 * activations a backward kernel reads as an fp32 mask. */
int ngnn_widen_bf16_rows(const void *src, int64_t lds, int64_t F, int64_t n_rows,
                         const int32_t *n_rows_dev, float *dst, int64_t ldd, void *stream);
/* gate / gate_gen (ABI 20, nullable): as ngnn_adam_fold's -- the step of a
 * block that broke the graph slot's contract updates nothing. */
int ngnn_adam_step(int n_tensors, float *const *params, const float *const *grads,
                   float *const *exp_avgs, float *const *exp_avg_sqs, const int64_t *numels,
                   const int32_t *dtypes, float *step, uint32_t *ticket, float lr, float beta1, float beta2, float eps,
                   float weight_decay, const uint64_t *gate, const int64_t *gate_gen, void *stream);

/* ------------------------------------------------------ HIP-graph slot
 * Fill the static slot a captured training step reads (ngnn/graphs.py) with
 * one NeighborLoader block, in one launch: x rows [0, N) (slot rows past N
 * untouched), edge_index [2, E] (row stride ld_ei) plus padding self-loops
 * on rows N + floor(j (n_cap - N) / (e_cap - E)) for slot edges E + j, the
 * first B labels, and *n_valid = N.  Padding needs N < n_cap when E < e_cap.
 * Optional (NULL to skip): slot_rowptr [n_cap + 1] / slot_col [e_cap] int32
 * = the target-grouped CSR of the padded edges (both or neither; targets
 * must be non-decreasing, NeighborLoader's order), and *seed_state advanced
 * by one splitmix64 step (the dropout seed of the captured step).  x_dev
 * (nullable): zero-copy -- store x's address there instead of copying the
 * rows (slot_x may then be NULL; x 16-B aligned with ldx == ld_slot).
 * r_next (nullable, 8-B aligned): its low 32 bits become max(B, 1 + max
 * source of the edges into rows < B) -- ngnn_block_prefix_stats for R = B,
 * the input-gradient row bound of the top layer's backward (computed here
 * so the captured step has no bound launch).  Kept by a 64-bit atomicMax of
 * (gen << 32 | value): gen must grow with every load (no reset launch).
 * n_edge_rows (nullable): 1 + the last target (0 without edges) = the split
 * of ngnn_sage_fwd_raw's n_edge_rows_dev.
 * slot_ei may be NULL when the CSR is written (a captured step that reads
 * only the CSR).
 * pack_dst (nullable): a pack job in the same launch -- pack_dst =
 * ngnn_pack_weight(pack_w [pack_fo, pack_k], row stride pack_ldw), the
 * current values of a weight the captured step's forward then reads with
 * NGNN_WL_PREPACKED (no pack launch inside the step; read at load time, so
 * parameters changed between steps are picked up).
 * err (nullable; may be host memory the device can write, e.g. pinned):
 * bits OR-ed in (never cleared here) when the block breaks the slot's
 * contract -- NGNN_SLOT_UNSORTED: a target smaller than the one before it;
 * NGNN_SLOT_RANGE: a source or target outside [0, N).  The CSR of such a
 * block is wrong, but no consumer of the slot reads or writes out of bounds:
 * a source outside [0, N) is stored as row 0 (slot_ei, slot_col, slot_colx
 * and the r_next bound; ABI 18), a target only selects which rowptr entries
 * (clamped to [0, n_cap]) its edge lands under.  E > 0 needs N >= 1.  The
 * caller checks the word without a device sync (ABI 16: replaces a host
 * read-back of the targets).
 * gate (ABI 20, nullable, 8-B aligned device word): (gen << 32 | bits) of the
 * newest load that broke the contract, by a 64-bit atomicMax -- the device
 * copy of err that ngnn_adam_fold / ngnn_adam_step read to skip that step's
 * update (no reset launch: the generation tells this load's bits from an
 * older load's).
 * counts_dev (ABI 19, nullable): device int32 {N', E', ...} -- the block's
 * row and edge counts are min(N', N) / min(E', E), read on the device (N / E
 * are then bounds: the capacity-sized buffers a sync-free sampler wrote;
 * ld_ei >= E still holds).
 * Replaces the host-side batch hand-over of pipeline.py:152-160 (batch.x,
 * batch.edge_index, batch.y[:batch_size]) for graph replay. */
#define NGNN_SLOT_UNSORTED 1
#define NGNN_SLOT_RANGE 2
int ngnn_slot_load(const float *x, int64_t ldx, int64_t N, int64_t F, const int64_t *edge_index,
                   int64_t ld_ei, int64_t E, const int64_t *y, int64_t B, float *slot_x,
                   int64_t ld_slot, int64_t n_cap, int64_t *slot_ei, int64_t e_cap,
                   int64_t *slot_y, int32_t *n_valid, int32_t *slot_rowptr, int32_t *slot_col,
                   uint64_t *seed_state, const float **x_dev, int64_t *r_next, uint32_t gen,
                   int32_t *n_edge_rows, const int64_t *xrow, const int64_t **xrow_dev,
                   int32_t *slot_colx, const float *pack_w, int64_t pack_ldw, int64_t pack_fo,
                   int64_t pack_k, float *pack_dst, int32_t *err, const int32_t *counts_dev,
                   uint64_t *gate, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NGNN_H */
