/*
 * ppnp_amd.h -- C ABI of the MI355X (gfx950) APPNP propagation path.
 *
 * This is the drop-in boundary for the propagation hot path of bkj/ppnp.  The reference
 * has no FFI of its own (it is pure Python); each entry point below names the reference
 * interface it replaces (file:line under the reference checkout):
 *
 *   appnp_graph_create*   helpers.py:58-66   calc_A_hat(adj, mode)   (host scipy, fp64)
 *                         helpers.py:68-71   compute_ppr(...)         (dense O(N^3) inverse)
 *   appnp_propagate       model.py:63        self.ppr[idx] @ self.encoder(X)  -- the dense
 *                                            PPR product becomes K fused CSR SpMM+AXPBY
 *                                            launches  Z <- (1-a) A_hat Z + a H
 *   appnp_propagate_bwd   model.py:63        autograd of the same product (dH = J^T dZ)
 *   appnp_step            one iteration; used by the row-partitioned multi-GPU driver
 *   appnp_step_split      the same on the split layout (whole-line main columns + the
 *                         L2-blocked remainder pass) of a row-partitioned graph
 *   appnp_dist_*          the row partition's whole K loop (SURVEY.md 8(b) appnp_dist_create)
 *   appnp_standardize     ppnp/data/sparsegraph.py:191-222  SparseGraph.standardize
 *                         (unweighted, undirected, no self loops, largest CC)
 *   appnp_spmm            model.py:36-38,47  Dropout + X @ W1 of the encoder on a CSR X
 *                         (main.py:91 densifies X; 1.76 % dense on Cora-ML)
 *
 * Conventions
 *   - Every function returns 0 (APPNP_OK) or a negative errno-style code; nothing throws or
 *     aborts across the ABI.  appnp_strerror() names a code.
 *   - All array arguments are DEVICE pointers on the current HIP device; the caller owns H,
 *     Z, dZ, dH and the workspace; the graph handle owns its device CSR.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).  appnp_propagate,
 *     appnp_propagate_bwd and appnp_step are asynchronous and stream-ordered: no host sync,
 *     no allocation (graph-capturable).  appnp_graph_create* allocates and synchronises.
 *   - Dense matrices are row-major with a leading dimension `ld` in ELEMENTS (ld >= f).
 *   - A handle is not thread-safe; distinct handles are independent.
 */
#ifndef PPNP_AMD_H
#define PPNP_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 6): appnp_dist_workspace_bytes reserves staging for a misaligned H / Z (a larger
 * workspace than version 1 asked for); the pipelined row steps (appnp_graph_shard_offsets,
 * appnp_step_shards, appnp_step_split_shards, appnp_dist_set_broadcast); the per-launch timer
 * brackets each launch (start and end events) and has the kinds APPNP_KT_LOCAL / _REMOTE /
 * _XCHG; appnp_tuning_overrides / appnp_tuning_names. */
#define PPNP_AMD_ABI_VERSION 2

typedef struct appnp_graph appnp_graph;

enum appnp_status {
  APPNP_OK = 0,
  APPNP_EDEVICE = -5,   /* HIP runtime / kernel launch failure            */
  APPNP_ENOMEM = -12,   /* device allocation failed                       */
  APPNP_EINVAL = -22,   /* bad argument (shape, pointer, ld, alignment)   */
  APPNP_ERANGE = -34,   /* size exceeds the int32 CSR index range         */
  APPNP_ENOTSUP = -95   /* valid request this build does not implement    */
};

/* helpers.py:61-66: 'sym' = D^-1/2 (A+I) D^-1/2, 'rw' = D^-1 (A+I) */
enum appnp_norm { APPNP_NORM_SYM = 0, APPNP_NORM_RW = 1 };

/* OR into `mode` of appnp_graph_create: also build A_hat^T (full graphs only) so that
 * appnp_propagate_bwd works for 'rw' and for directed graphs.  Not needed (and not built)
 * for 'sym' on an undirected graph, where A_hat^T == A_hat. */
#define APPNP_GRAPH_TRANSPOSE 0x100

/* OR into `mode`: also keep a copy of A_hat regrouped by source block (2^15 source rows per
 * block; full graphs only).  appnp_propagate then takes the last 1-4 columns of fp32 rows
 * with F = 32q + r (e.g. F = 100) out of the random gather and forms their product in one
 * persistent, L2-resident pass per iteration, so a gathered row costs q cache lines instead
 * of q + 1.  Costs 8 bytes per nonzero (4 on an unweighted graph without self loops, whose
 * entries need no values, plus 8 bytes per node) plus one int32 per (block, 640-row group) of
 * device memory (segments padded to 64 entries).  Best-effort: when the copy cannot be built (too many blocks, device memory), the
 * graph is still created and gathers whole rows; appnp_graph_source_blocks tells. */
#define APPNP_GRAPH_SOURCE_BLOCKS 0x200

/* OR into `mode` instead of (or with) APPNP_GRAPH_SOURCE_BLOCKS: the source-blocked copy for a
 * remainder of up to 8 (W8) or 16 (W16) columns: fp32 rows of F = 32q + r features with
 * r <= 8 on a W8 copy (a wider remainder beside a main part costs as much as its extra line,
 * measured), and narrow rows F <= 8 / 16 whole (for example F = 40 = 32 + 8, or the 12-13-column
 * slabs of an 8-rank column layout of F = 100).  A W16 copy serves narrow rows only: beside a
 * main part its 4 row passes cost more than the extra line (F = 100 / 36 measured), so such
 * rows stay whole on it.  The pass then gives 2 / 4 lanes to each
 * entry and holds 320 / 160 rows per wave group, so a graph may need 2 / 4 row passes per
 * launch.  Same memory as APPNP_GRAPH_SOURCE_BLOCKS (segments padded to 32 / 16 entries). */
#define APPNP_GRAPH_SB_W8 0x400
#define APPNP_GRAPH_SB_W16 0x800

/* storage type of H / Z (accumulation is always fp32) */
enum appnp_dtype { APPNP_F32 = 0, APPNP_BF16 = 1 };

int appnp_abi_version(void);
/* Provenance of this build: "src=<digest of the .hip and .h files of ppnp_amd/csrc and of this
 * header (srcdigest.py)>;abi=..;arch=<the Makefile's ARCH, gfx950>;compiler=..;built=..".
 * bench.py prints it next to the digest of the tree it runs in, so a library built from other
 * sources shows. */
const char* appnp_build_info(void);
const char* appnp_strerror(int code);

/*
 * Build A_hat on the device from the CSR of A (helpers.py:58-66).
 *   indptr[n+1], indices[nnz]: int32 CSR of A, columns strictly increasing in each row
 *                              (scipy canonical form); device pointers.
 *   vals[nnz]: fp32 edge weights, or NULL for an unweighted graph (all ones).
 *   A may or may not contain diagonal entries: A+I merges them (a_ii + 1), exactly as
 *   `adj + sp.eye(n)` does, and entries whose merged value is 0 are dropped.
 * Degrees are fp64 weighted row sums of A+I; A_hat values are computed in fp64 and rounded
 * once to fp32, so they equal float32(calc_A_hat(adj, mode).data) bit for bit.
 */
int appnp_graph_create(const int32_t* indptr, const int32_t* indices, const float* vals,
                       int64_t n, int64_t nnz, int mode, void* stream, appnp_graph** out);

/*
 * Device-side SparseGraph.standardize (ppnp/data/sparsegraph.py:191-222): unweighted,
 * undirected (pattern of A + A^T), no self loops and, if select_lcc, only the largest
 * connected component with nodes renumbered in increasing order (create_subgraph,
 * sparsegraph.py:300-352).  Input: CSR of the raw adjacency (device; vals may be NULL;
 * explicit zero weights count as absent).  Output: a handle owning the standardized int32
 * CSR (sorted columns) and node_map[n_out] (int64 input node id of each kept node), which
 * subsets attributes/labels exactly as the reference does.  Allocates and synchronises.
 * Ties for the largest component go to the one with the largest smallest node index (the
 * reference's np.argsort(sizes)[::-1][:1] is not stable, so its own tie order depends on the
 * numpy build; real datasets have a unique largest component).
 */
typedef struct appnp_csr appnp_csr;
int appnp_standardize(const int32_t* indptr, const int32_t* indices, const float* vals,
                      int64_t n, int64_t nnz, int select_lcc, void* stream, appnp_csr** out);
int appnp_csr_info(const appnp_csr* c, int64_t* n, int64_t* nnz, int64_t* n_in);
int appnp_csr_copy(const appnp_csr* c, int32_t* indptr, int32_t* indices, int64_t* node_map,
                   void* stream);
void appnp_csr_destroy(appnp_csr* c);

/* Transpose of a CSR (rows x cols) as a canonical CSR (cols x rows, columns = input rows in
 * increasing order), values carried when vals != NULL.  appnp_csr_info reports n = cols,
 * n_in = rows; appnp_csr_copy gives indptr/indices (node_map unused); appnp_csr_values the
 * values.  Allocates and synchronises. */
int appnp_csr_transpose(const int32_t* indptr, const int32_t* indices, const float* vals,
                        int64_t rows, int64_t cols, int64_t nnz, void* stream, appnp_csr** out);
int appnp_csr_values(const appnp_csr* c, float* data, void* stream);

/*
 * General sparse x dense product on the same fused kernel family (fp32):
 *   C[rows, f] = (M o A) B,   A: CSR rows x cols (vals NULL = all ones), B: cols x f (ld_b)
 * with optional entry dropout M (keep iff 24-bit hash of (seed, 0, i, j) >= p * 2^24, kept
 * entries scaled by 1/(1-p)); transposed_key != 0 keys entry (i, j) as (j, i), so the product
 * with A^T (appnp_csr_transpose) replays the mask of A -- the backward of a dropout SpMM.
 * Used for the sparse encoder input (model.py:36-38, 47 on a CSR X; main.py:91 densifies X).
 */
int appnp_spmm(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t rows,
               int64_t cols, const float* B, int64_t ld_b, float* C, int64_t ld_c, int64_t f,
               float p_drop, uint64_t seed, int transposed_key, void* stream);

/*
 * Same as appnp_graph_create, but keeps only rows [row_lo, row_hi) of A_hat (global column indices); degrees of
 * all n nodes are still computed from the full A.  Used for the row-partitioned multi-GPU
 * path: rank r owns rows [row_lo, row_hi).  With split_local != 0 the rows are also stored
 * as two CSRs -- columns inside [row_lo,row_hi) ("local") and outside ("remote") -- so the
 * local product can overlap the all-gather of the remote rows.
 */
int appnp_graph_create_rows(const int32_t* indptr, const int32_t* indices, const float* vals,
                            int64_t n, int64_t nnz, int mode, int64_t row_lo, int64_t row_hi,
                            int split_local, void* stream, appnp_graph** out);

void appnp_graph_destroy(appnp_graph* g);

/* n (global nodes), rows held [row_lo,row_hi), nnz of the held A_hat rows, symmetric flag
 * (1 if A's pattern and weights are symmetric, so A_hat^T == A_hat for 'sym'). */
int appnp_graph_info(const appnp_graph* g, int64_t* n, int64_t* row_lo, int64_t* row_hi,
                     int64_t* nnz_hat, int* mode, int* symmetric);

/* Read-only device views of the held A_hat CSR (row_ptr is local: row_ptr[0] == 0). */
int appnp_graph_csr(const appnp_graph* g, const int32_t** row_ptr, const int32_t** col,
                    const float** val);

/* Stream-ordered copy of the held A_hat CSR and of dinv into caller-owned device buffers
 * (row_ptr[rows+1], col[nnz_hat], val[nnz_hat], dinv[n]); any pointer may be NULL. */
int appnp_graph_copy_csr(const appnp_graph* g, int32_t* row_ptr, int32_t* col, float* val,
                         double* dinv, void* stream);

/* Device bytes of the source-blocked copy (APPNP_GRAPH_SOURCE_BLOCKS); 0 if not built. */
int appnp_graph_source_blocks(const appnp_graph* g, int64_t* bytes);

/* Device view of the fp64 inverse-degree vector (1/sqrt(D) for sym, 1/D for rw), length n. */
int appnp_graph_dinv(const appnp_graph* g, const double** dinv);

/* Bytes of workspace appnp_propagate / appnp_propagate_bwd need for this shape.  The
 * workspace holds the ping-pong iterates with its own line-aligned leading dimension, or the
 * two buffers of the split layout ([n, fs] + [n, width of the source-blocked copy]), whichever
 * is larger (`ld` is accepted for ABI stability and ignored). */
size_t appnp_workspace_bytes(const appnp_graph* g, int64_t f, int64_t ld, int dtype);

/* The column split appnp_propagate uses for this shape when H and Z are 16-B aligned with
 * leading dimensions that are multiples of 4 floats (K >= 2): columns [0, *fs) gather whole cache
 * lines and [*fs, F) run the persistent L2-blocked remainder pass.  fp32 rows of F = 32q + r
 * features take it on a graph built with a source-blocked copy, above 2^16 nodes and without
 * gather locality: r <= 4 on an APPNP_GRAPH_SOURCE_BLOCKS copy, r <= 8 on an APPNP_GRAPH_SB_W8
 * copy (wider remainders beside a main part keep whole rows, and so does every F > 32 on an
 * APPNP_GRAPH_SB_W16 copy).  *fs = 0 when rows are
 * gathered whole, and also for narrow rows, which run wholly in the pass (see below).
 * Informational: appnp_propagate decides by itself, on the same rule. */
int appnp_propagate_split_point(const appnp_graph* g, int64_t f, int dtype, int64_t* fs);

/* The remainder columns of that split: *r = F - fs columns run the L2-blocked pass -- 1-4 on an
 * APPNP_GRAPH_SOURCE_BLOCKS copy, up to 8 on a W8 copy -- and narrow rows F <= 4 / 8 / 16
 * (the copy's width) run wholly in the pass, *r = F with *fs = 0.  *r = 0 when rows are
 * gathered whole. */
int appnp_propagate_remainder_cols(const appnp_graph* g, int64_t f, int dtype, int64_t* r);

/* The source-blocked copy as built: *width remainder columns per row (4, 8, 16; 0 = not built),
 * *entries regrouped entries including padding, *value_free = 1 when entries carry no values
 * (unit graph: A_hat_ij = dl_i dr_j), *row_passes row-group passes per launch, and *launches the
 * remainder-pass launches enqueued on this graph so far (which path a propagation took). */
int appnp_graph_source_block_layout(const appnp_graph* g, int* width, int64_t* entries,
                                    int* value_free, int* row_passes, int64_t* launches);

/*
 * Z = APPNP_K(H):  Z_0 = H;  Z_{k+1} = (1-alpha) (M_k o A_hat) Z_k + alpha H,  k < K.
 *   H, Z: n x f, leading dims ld_h / ld_z, `dtype` storage; must not alias.
 *   p_drop in [0,1): edge dropout; M_k keeps edge (i,j) at step k iff the 24-bit counter
 *   hash of (seed, k, i, j) >= p_drop * 2^24, and scales kept edges by 1/(1-p_drop).
 *   p_drop = 0 is eval mode (the reference's semantics).
 *   ws: appnp_workspace_bytes() bytes (may be NULL when that is 0).
 * One fused kernel launch per iteration.  With split rows (appnp_propagate_remainder_cols >
 * 0) an iteration is that launch on the first fs columns (none for narrow rows) plus ONE
 * persistent launch of the L2-blocked remainder pass over every source block, and H is first
 * copied into the workspace's split layout.  All launches are stream-ordered on `stream`;
 * nothing is allocated or synchronised.  Requires a full (non-partitioned) graph.
 */
int appnp_propagate(const appnp_graph* g, const void* H, int64_t ld_h, void* Z, int64_t ld_z,
                    int64_t f, int dtype, int K, float alpha, float p_drop, uint64_t seed,
                    void* ws, size_t ws_bytes, void* stream);

/*
 * dH = J^T dZ for the map H -> Z of appnp_propagate with the same (K, alpha, p_drop, seed).
 * Uses A_hat^T: A_hat itself for 'sym' on an undirected graph, otherwise the transpose built
 * at creation with APPNP_GRAPH_TRANSPOSE; APPNP_ENOTSUP if neither is available.  On a
 * self-adjoint A_hat it uses the same column split as appnp_propagate.
 */
int appnp_propagate_bwd(const appnp_graph* g, const void* dZ, int64_t ld_dz, void* dH,
                        int64_t ld_dh, int64_t f, int dtype, int K, float alpha, float p_drop,
                        uint64_t seed, void* ws, size_t ws_bytes, void* stream);

/*
 * One iteration on the held rows:  Zout[i-row_lo] = (1-alpha) sum_j (M_k o A_hat)_ij Zin[j]
 *                                                   + alpha H[i-row_lo],  i in [row_lo,row_hi)
 *   Zin: all n rows (global row index), Zout/H: the held rows only.
 *   part selects which stored CSR is applied:
 *     APPNP_PART_ALL     the held rows' full CSR (epilogue as above)
 *     APPNP_PART_LOCAL   local-column CSR only:  P[i] = (1-alpha) sum_local ...   (P = Zout, fp32)
 *     APPNP_PART_REMOTE  remote-column CSR, finishing: Zout = (1-alpha) sum_remote + P + alpha H
 *                        (P passed as `partial`, fp32, ld = ld_partial)
 */
enum appnp_part { APPNP_PART_ALL = 0, APPNP_PART_LOCAL = 1, APPNP_PART_REMOTE = 2 };

int appnp_step(const appnp_graph* g, int part, const void* Zin, int64_t ld_in, const void* H,
               int64_t ld_h, void* Zout, int64_t ld_out, const float* partial,
               int64_t ld_partial, int64_t f, int dtype, int k, float alpha, float p_drop,
               uint64_t seed, void* stream);

/*
 * Split rows on the held rows of a row-partitioned graph (appnp_graph_create_rows with a
 * source-blocked copy, APPNP_GRAPH_SOURCE_BLOCKS / _SB_W8 / _SB_W16; fp32; the split rule of
 * appnp_propagate_remainder_cols).  The iterate is kept as two FULL-HEIGHT parts (every rank's
 * rows, global row index): main [rows_total, fs] (fs = F - r columns, whole cache lines per
 * gathered row) and rem [rows_total, rem_width] (the r remainder columns, zero padded; on a unit
 * graph scaled by the column scale of A_hat, which only these functions read and write).  Each
 * rank writes its held rows of both parts; an exchange (all-gather) fills the others.  All
 * buffers 16-B aligned, leading dimensions multiples of 4 floats.
 *
 * appnp_split_layout  *fs and *rem_width of that layout for F; APPNP_ENOTSUP when F does not
 *                     split on this graph (then use appnp_step).
 * appnp_split_copy    the held rows of H (ld_h) into rows [row_lo, row_hi) of main and rem: the
 *                     Z_0 parts.  main may be NULL when fs = 0.
 * appnp_step_split    one iteration of the held rows from all rows of zin_main / zin_rem:
 *                     into rows [row_lo, row_hi) of zout_main / zout_rem, or, when Z != NULL,
 *                     into the held rows of Z (ld_z, all F columns: the last iteration).  part
 *                     as for appnp_step, on the main columns: ALL (then the remainder pass),
 *                     LOCAL (local-column product of the main part into the fp32 `partial`
 *                     [held rows, fs], ld_partial; zin_rem is not read, so it may still be in
 *                     flight), REMOTE (remote columns + partial + alpha H, then the remainder
 *                     pass).  LOCAL / REMOTE need split_local.  Stream-ordered, no allocation.
 * the north_star's row partition gathers q lines per nonzero for F = 32q + r
 * instead of q + 1, as the single-GPU appnp_propagate does.
 */
int appnp_split_layout(const appnp_graph* g, int64_t f, int64_t* fs, int64_t* rem_width);
int appnp_split_copy(const appnp_graph* g, const float* H, int64_t ld_h, int64_t f, float* main,
                     float* rem, void* stream);
int appnp_step_split(const appnp_graph* g, int part, const float* zin_main, const float* zin_rem,
                     const float* H, int64_t ld_h, float* zout_main, float* zout_rem, float* Z,
                     int64_t ld_z, float* partial, int64_t ld_partial, int64_t f, int k,
                     float alpha, float p_drop, uint64_t seed, void* stream);

/*
 * Pipelined row steps.  A row rank's product split by
 * SOURCE SHARD: with the held rows' entries grouped by the shard of their column (rank s of P
 * holds rows [s S, (s+1) S)), the product over the shards that have already arrived can run while
 * the others are still in flight, one launch per group of shards, so only the last group's share
 * of the compute is left after the exchange ends.
 *
 * appnp_graph_shard_offsets  build the held rows' shard offsets (nshards = P, shard_rows = S,
 *                            P S >= n; (P + 1) x rows int32 of device memory).  Allocates and
 *                            synchronises; idempotent for the same P and S.
 * appnp_step_shards          one iteration's product over the entries of the held rows whose
 *                            column lies in shards [s_lo, s_hi) (fp32):
 *                              APPNP_SHARDS_FIRST  partial  = (1-alpha) sum
 *                              APPNP_SHARDS_ACC    partial += (1-alpha) sum
 *                              APPNP_SHARDS_LAST   Zout     = (1-alpha) sum + partial + alpha H
 *                              APPNP_SHARDS_ONLY   Zout     = (1-alpha) sum + alpha H
 *                            Zin: all n rows (only the range's rows are read); partial [held rows,
 *                            f] fp32.  Summing every shard once, in any grouping, gives the
 *                            appnp_step result up to fp32 summation order.
 * appnp_step_split_shards    the same on the split layout of appnp_step_split: the main columns
 *                            take the shard range and mode; LAST / ONLY then run the remainder
 *                            pass (which needs every row of zin_rem) and write zout_* or Z.
 * Stream-ordered, no allocation; the dropout hash is the same as appnp_step's.
 */
enum appnp_shard_mode {
  APPNP_SHARDS_FIRST = 0,
  APPNP_SHARDS_ACC = 1,
  APPNP_SHARDS_LAST = 2,
  APPNP_SHARDS_ONLY = 3
};
int appnp_graph_shard_offsets(appnp_graph* g, int nshards, int64_t shard_rows, void* stream);
int appnp_step_shards(const appnp_graph* g, int s_lo, int s_hi, int mode, const float* Zin,
                      int64_t ld_in, const float* H, int64_t ld_h, float* Zout, int64_t ld_out,
                      float* partial, int64_t ld_partial, int64_t f, int k, float alpha,
                      float p_drop, uint64_t seed, void* stream);
int appnp_step_split_shards(const appnp_graph* g, int s_lo, int s_hi, int mode,
                            const float* zin_main, const float* zin_rem, const float* H,
                            int64_t ld_h, float* zout_main, float* zout_rem, float* Z,
                            int64_t ld_z, float* partial, int64_t ld_partial, int64_t f, int k,
                            float alpha, float p_drop, uint64_t seed, void* stream);

/*
 * A captured propagation plan: the K launches of appnp_propagate for FIXED buffers (H, Z, ws)
 * and parameters, recorded once into a hipGraph and replayed by appnp_plan_launch on any
 * stream with a single graph launch.  For small, launch-bound graphs and serving loops that
 * refill H in place.  Creating a plan captures on an internal stream (no kernels run).
 */
typedef struct appnp_plan appnp_plan;
int appnp_plan_create(const appnp_graph* g, const void* H, int64_t ld_h, void* Z, int64_t ld_z,
                      int64_t f, int dtype, int K, float alpha, float p_drop, uint64_t seed,
                      void* ws, size_t ws_bytes, appnp_plan** out);
int appnp_plan_launch(const appnp_plan* p, void* stream);
void appnp_plan_destroy(appnp_plan* p);

/*
 * Row-partitioned multi-GPU propagation: SURVEY.md 8(b)'s appnp_dist_create, the loop of
 * ppnp_amd/dist.py PartitionedAPPNP.run for a pure row layout, and the replacement of the
 * reference's single-device product model.py:63 for graphs that outgrow one GPU.
 *
 * Rank r of P holds rows [r S, min(n, (r+1) S)) of A_hat, S = ceil(n / P).  After every
 * iteration but the last, the ranks exchange their new row shards through a caller-supplied
 * all-gather, so the library owns no communicator.  With overlap, each iteration first
 * applies the local-column part of the rows on `stream`, while the previous exchange still
 * runs on an internal stream, then waits for it and finishes with the remote columns.
 */
typedef struct appnp_dist appnp_dist;

/*
 * In-place all-gather of equal row shards.  `buf` is a device buffer of nranks * shard_bytes;
 * this rank's shard sits at rank * shard_bytes and is complete in stream order on `stream`.
 * The function must leave every rank's shard in place in stream order on `stream`. It can
 * enqueue the exchange there, as ncclAllGather(buf + rank * shard_bytes, buf, shard_bytes,
 * ncclChar, comm, stream) does (appnp_allgather_rccl). Or it can synchronise `stream`, exchange
 * and return.  It returns 0 or a negative code, which appnp_dist_propagate passes on.
 */
typedef int (*appnp_allgather_fn)(void* buf, size_t shard_bytes, int rank, int nranks,
                                  void* stream, void* ctx);

/* indptr/indices/vals/n/nnz/mode: the WHOLE graph's A on this device, as appnp_graph_create.
 * `mode` may carry APPNP_GRAPH_SOURCE_BLOCKS / _SB_W8 / _SB_W16: then fp32 propagations whose
 * F splits (appnp_split_layout) with 16-B aligned H / Z run on the split layout (main part
 * gathers whole lines, remainder pass; appnp_step_split).  Every rank must take that path or
 * none: the rule is the same on every rank (its gather-locality measure is taken over the whole
 * A), and since the copy is best-effort, the first fp32 propagation with K >= 2 agrees through
 * one small exchange in the workspace that every rank built it (that call synchronises the
 * stream once).  A rank whose agreement fails after that exchange keeps failing (the handle is
 * poisoned: every later call returns the stored error without exchanging); a failure before it
 * (the flag's memset, or the callback itself) leaves the peers waiting in that exchange, as
 * any collective does when one rank drops out, so the caller must then end its communicator.
 * The decision does not depend on H or Z: a rank whose H or Z is not 16-B aligned (base pointer
 * or leading dimension) stages it through the workspace, so every rank exchanges the same
 * parts.
 * overlap != 0 keeps the held rows as local- and remote-column CSRs (fp32 propagation only).
 * allgather/ctx: the exchange, called by every rank once per exchanged iterate (twice on the
 * split layout: its main part, then its remainder part). */
int appnp_dist_create(const int32_t* indptr, const int32_t* indices, const float* vals,
                      int64_t n, int64_t nnz, int mode, int rank, int nranks, int overlap,
                      appnp_allgather_fn allgather, void* ctx, void* stream, appnp_dist** out);

/* The held rows [row_lo, row_hi), the shard height S, and the graph of those rows. */
int appnp_dist_rows(const appnp_dist* d, int64_t* row_lo, int64_t* row_hi, int64_t* shard);
const appnp_graph* appnp_dist_graph(const appnp_dist* d);

/* Workspace of appnp_dist_propagate: two full-height iterates (P S rows, line-aligned, or the
 * two parts of the split layout) and, with overlap, the fp32 local-column partial of the held
 * rows; the larger of the two layouts when F splits, the split one with room to stage a
 * misaligned H and Z ([S, F rounded up to 4] fp32 each). */
size_t appnp_dist_workspace_bytes(const appnp_dist* d, int64_t f, int dtype);

/*
 * Z = the held rows of APPNP_K(H), given the held rows of H (row_hi - row_lo rows each;
 * leading dimensions ld_h, ld_z; same semantics, dropout hash and results as appnp_propagate
 * on the whole graph).  Collective: every rank calls it with the same f, dtype, K, alpha,
 * p_drop and seed.  Stream-ordered on `stream`; no allocation; the exchange callback runs on
 * the calling thread.
 */
int appnp_dist_propagate(appnp_dist* d, const void* H, int64_t ld_h, void* Z, int64_t ld_z,
                         int64_t f, int dtype, int K, float alpha, float p_drop, uint64_t seed,
                         void* ws, size_t ws_bytes, void* stream);
void appnp_dist_destroy(appnp_dist* d);

/*
 * The pipelined exchange of the row loop.  With overlap and
 * P >= 3 ranks, a broadcast callback makes appnp_dist_propagate send every iterate as P in-place
 * broadcasts, one row shard each (roots 0 .. P-1 in turn, on the engine's exchange stream, each
 * followed by an event), and run the product as appnp_step(_split)_shards launches: FIRST on the
 * rank's own shard, then ACC per group of arrived remote shards (sized 1, 2, 4, ... from the last
 * to arrive, appnp_dist_pipeline_groups), LAST on the last group -- so after the exchange only
 * one shard's share of the product is left instead of every remote shard's.  The split layout's
 * remainder part keeps the all-gather (it is exchanged first).  Collective: every rank sets it.
 * appnp_bcast_fn: in-place broadcast of `bytes` at `buf` from rank `root` to every rank, in stream
 * order on `stream` (ncclBroadcast(buf, buf, bytes, ncclChar, root, comm, stream) for RCCL:
 * appnp_bcast_rccl), or synchronous; returns 0 or a negative code.
 * appnp_dist_set_broadcast builds the held rows' shard offsets (allocates, synchronises `stream`);
 * APPNP_ENOTSUP without overlap or with P < 3 (one remote shard: nothing to pipeline).
 */
typedef int (*appnp_bcast_fn)(void* buf, size_t bytes, int root, int nranks, void* stream,
                              void* ctx);
int appnp_dist_set_broadcast(appnp_dist* d, appnp_bcast_fn fn, void* ctx, void* stream);
/* The groups [lo[i], hi[i]) of remote shards, *n_out of them (0: not pipelined). */
int appnp_dist_pipeline_groups(const appnp_dist* d, int* lo, int* hi, int max, int* n_out);
int appnp_bcast_rccl(void* buf, size_t bytes, int root, int nranks, void* stream, void* ctx);

/* appnp_allgather_fn over RCCL; ctx is the ncclComm_t of the P ranks, rank order = row order.
 * RCCL is resolved at first use (the librccl.so.1 already loaded in the process, e.g.
 * PyTorch's, else the system one; APPNP_RCCL_LIB overrides), so the library does not link it.
 * APPNP_ENOTSUP if it cannot be loaded, APPNP_EDEVICE if the call fails. */
int appnp_allgather_rccl(void* buf, size_t shard_bytes, int rank, int nranks, void* stream,
                         void* ctx);

/*
 * Measurement aid (no counterpart in the reference): gathers `lines` random 128-B lines of the
 * device buffer `table` (table_bytes, 128-B aligned; read only) on `stream`, 8 lanes per line
 * and 64 lines in flight per wave, line indices hashed from `seed`.  The caller times it with
 * events; lines / time is the box's random-line rate, the quantity that bounds the SpMM on a
 * uniform random graph.  bench.py runs it before its timed region
 * (roofline.box_line_rate).  `sink`: one device float, written only if the gathered sum hits a
 * sentinel value.
 */
int appnp_line_rate_probe(const void* table, int64_t table_bytes, int64_t lines, uint64_t seed,
                          float* sink, void* stream);

/*
 * Measurement aid (no counterpart in the reference): the device time of every launch of the
 * calls made between appnp_kernel_timer_begin and appnp_kernel_timer_end on the calling thread.
 * While the timer is on, appnp_propagate, appnp_propagate_bwd, appnp_step, appnp_step_split
 * and appnp_split_copy (and so appnp_dist_propagate) bracket each launch by two timing events on
 * its stream, one right before and one right after it, tagged with its kind; appnp_dist_propagate
 * brackets each exchange call the same way (APPNP_KT_XCHG, on the stream it is enqueued on).  So
 * an interval covers its launch only: a wait for another stream, or host time, before a launch is
 * never counted in it (`stream` of begin is unused).  The events sit between launches that are
 * stream-ordered anyway, so the launches run as they would without them, but a call timed this
 * way is not graph-capturable, and a replayed plan (appnp_plan_launch) records nothing.  end
 * waits for the events and writes, for the first min(n, max) launches, kinds[i] (APPNP_KT_*) and
 * ms[i], NaN if the pair cannot be timed.  *n_out = launches recorded; APPNP_ERANGE if more than
 * max_launches were enqueued (the rest were not timed).  bench.py prints the split of one
 * propagation as roofline.kernel_ms.
 */
enum appnp_kernel_kind {
  APPNP_KT_COPY = 1,   /* H (or dZ) into the split layout, or a plain copy / scale of rows  */
  APPNP_KT_STEP = 2,   /* the fused SpMM + AXPBY kernel (whole rows or the main columns)   */
  APPNP_KT_REM = 3,    /* the persistent L2-blocked remainder pass                          */
  APPNP_KT_LOCAL = 4,  /* appnp_step(_split) PART_LOCAL: the local-column product           */
  APPNP_KT_REMOTE = 5, /* appnp_step(_split) PART_REMOTE: the remote columns + epilogue     */
  APPNP_KT_XCHG = 6    /* appnp_dist_propagate: one call of the exchange (all-gather)       */
};
int appnp_kernel_timer_begin(int max_launches, void* stream);
int appnp_kernel_timer_end(float* ms, int* kinds, int max, int* n_out);

/*
 * Tuning overrides.  A few environment variables (appnp_tuning_names: ';'-separated) reshape
 * kernels for the measurement sweeps of tools/ -- vector width, entries in flight, the split
 * rule, the remainder pass's block size and barriers.  The library reads them only when
 * APPNP_TUNING=1 is set too; otherwise they are ignored and the measured defaults run.
 * appnp_tuning_overrides returns the ones in effect in this process ("NAME=value;..."), "" when
 * none; bench.py prints it as build.overrides.
 */
const char* appnp_tuning_overrides(void);
const char* appnp_tuning_names(void);

#ifdef __cplusplus
}
#endif

#endif /* PPNP_AMD_H */
