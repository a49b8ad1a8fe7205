// appnp_internal.h -- host-side internals shared by the translation units of libppnp_amd.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "appnp_device.h"
#include "../../include/ppnp_amd.h"

struct appnp_graph {
  int64_t n = 0;         // global node count
  int64_t row_lo = 0;    // held rows [row_lo, row_hi)
  int64_t row_hi = 0;
  int64_t nnz_hat = 0;   // nnz of the held A_hat rows
  int64_t nnz_local = 0, nnz_remote = 0;
  int mode = 0;          // APPNP_NORM_SYM / APPNP_NORM_RW
  int symmetric = 0;     // A's pattern and weights are symmetric
  int unit = 0;          // every entry of A+I is 1 (unweighted A, no self loops): A_hat is
                         // dl_i * dr_j with per-row scales (sym: dinv, dinv; rw: dinv, 1)
  int split = 0;         // local/remote CSRs present
  int device = 0;
  int32_t* row_ptr = nullptr;   // [rows+1]
  int32_t* col = nullptr;       // [nnz_hat]
  float* val = nullptr;         // [nnz_hat]
  int32_t* lrow_ptr = nullptr;  // local-column CSR (split only)
  int32_t* lcol = nullptr;
  float* lval = nullptr;
  int32_t* rrow_ptr = nullptr;  // remote-column CSR (split only)
  int32_t* rcol = nullptr;
  float* rval = nullptr;
  double* dinv = nullptr;       // [n] 1/sqrt(D) (sym) or 1/D (rw), fp64
  int32_t* heavy = nullptr;     // rows with > kHeavyRow entries (ascending)
  int64_t n_heavy = 0;
  int32_t* t_heavy = nullptr;   // the same for A_hat^T
  int64_t t_n_heavy = 0;
  int32_t* hub = nullptr;       // rows with > kHubRow entries: dispatched first (wide kernels)
  int64_t n_hub = 0;
  int32_t* t_hub = nullptr;
  int64_t t_n_hub = 0;
  int32_t* t_row_ptr = nullptr; // A_hat^T (APPNP_GRAPH_TRANSPOSE, when A_hat is not symmetric)
  int32_t* t_col = nullptr;
  float* t_val = nullptr;
  // A_hat regrouped for the persistent remainder pass (APPNP_GRAPH_SOURCE_BLOCKS,
  // appnp_blocks.hip): segment (group, source block) holds the entries of one wave's group of
  // rows whose column lies in that block, sorted by (row, column), padded to 64 entries
  int32_t* rb_off = nullptr;    // [rb_passes * rb_slots * rb_nb + 1] segment starts
  uint32_t* rb_ent = nullptr;   // [rb_total] (row in group << kRemColBits) | column in block
  float* rb_val = nullptr;      // [rb_total]; null for a unit graph (values from rb_dl/rb_dr)
  float* rb_dl = nullptr;       // unit graph: [n] fp32 dinv, the row scale of A_hat
  float* rb_dr = nullptr;       // unit graph, sym: [n] fp32 dinv, the column scale (rw: null)
  int32_t* rb_cblk = nullptr;   // [rb_total / 64] source block of each chunk of 64 entries
  int64_t rb_total = 0;         // entries including the padding
  int32_t rb_nb = 0;            // source blocks of 2^rb_br_log2 rows
  int32_t rb_br_log2 = 0;
  int32_t rb_grid = 0;          // workgroups of the pass (one per CU)
  int32_t rb_slots = 0;         // groups per pass = rb_grid * kRemWaves
  int32_t rb_rg = 0;            // rows per group
  int32_t rb_passes = 0;
  int32_t rb_lpe = 0;           // lanes per entry of the pass: remainder rows of 4 rb_lpe columns
  // shard offsets of the held rows (appnp_graph_shard_offsets): entries of held row i with a
  // column in shard s ([s sh_rows, (s+1) sh_rows)) are sh_off[s rows + i] .. sh_off[(s+1) rows + i]
  int32_t* sh_off = nullptr;    // [(sh_n + 1) * rows]
  int32_t sh_n = 0;
  int64_t sh_rows = 0;
  double near_frac = 0.0;       // off-diagonal entries within kNearRows of their row / nnz
  // remainder-pass launches enqueued on this graph (appnp_graph_source_block_layout): the path
  // witness the tests read
  mutable std::atomic<int64_t> rem_launches{0};
};

struct appnp_csr;

namespace appnp {

// appnp_graph.hip
int graph_build(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t n,
                int64_t nnz, int mode, int64_t row_lo, int64_t row_hi, int split,
                hipStream_t s, appnp_graph* g);
void graph_free(appnp_graph* g);
int graph_build_shard_offsets(appnp_graph* g, int nshards, int64_t shard_rows, hipStream_t s);
int graph_build_transpose(appnp_graph* g, hipStream_t s);
int build_heavy(const int32_t* rp, int64_t rows, int32_t thr, hipStream_t s, int32_t** out,
                int64_t* n_out);
int64_t scan_partials(int64_t rows);

// appnp_ingest.hip
int csr_transpose(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t rows,
                  int64_t cols, int64_t nnz, hipStream_t s, appnp_csr* out);
void csr_free(appnp_csr* c);
hipError_t exclusive_scan(const int32_t* cnt, int64_t rows, int32_t* out, int64_t* d_bsum,
                          int64_t* d_total, hipStream_t s);

// appnp_blocks.hip
// lpe: lanes per entry of the remainder pass (1, 2, 4: remainder rows of 4, 8, 16 columns)
// a_indptr / a_indices / a_nnz: the whole graph's A (the row partition's gather-locality
// measure is taken over all of it, so every rank decides the same split)
int graph_build_source_blocks(appnp_graph* g, int lpe, const int32_t* a_indptr,
                              const int32_t* a_indices, int64_t a_nnz, hipStream_t s);
// to_rem: out is the next remainder buffer (a unit graph stores dr o y there), not Z / dH
hipError_t launch_remainder(const appnp_graph* g, const StepArgs& a, int epi,
                            const float* z_rem, const float* h_rem, int64_t ld_h, float* out,
                            int64_t ld_out, int nv, bool to_rem, hipStream_t s);
// rem_scale (nullable): per-row factor of the remainder part (remainder_scale(g))
// rw: floats per remainder row (4 rb_lpe)
hipError_t launch_split_copy(const float* h, int64_t ld_h, int64_t n, int64_t f, int64_t fs,
                             int64_t rw, float* main, float* rem, const float* rem_scale,
                             hipStream_t s);
// the factor the remainder buffers carry: dr for a value-free (unit) layout, else none
inline const float* remainder_scale(const appnp_graph* g) {
  return g->rb_val ? nullptr : g->rb_dr;
}

// appnp_spmm.hip
int pick_vec(int dtype, int64_t f, const int64_t* lds, int n_ld, const void* const* ptrs,
             int n_ptr);
hipError_t launch_step(int dtype, int epi, int V, const StepArgs& a, hipStream_t s);
hipError_t launch_scale_rows(int dtype, const void* src, int64_t ld_src, void* dst,
                             int64_t ld_dst, int64_t n, int64_t f, float alpha, hipStream_t s);

// appnp_capi.hip: a tuning override (measurement only, tools/): `name` is read from the
// environment when APPNP_TUNING=1, else dflt.  Each is read once, at its first use; every name
// must be listed in kTuningNames (appnp_capi.hip), which appnp_tuning_overrides reports.
int tuning_env(const char* name, int dflt);

// appnp_capi.hip: the per-launch timer of appnp_kernel_timer_begin / _end.  While it is on
// (on this thread), every launch (or exchange) of the propagation entry points is bracketed by
// two timing events on its stream: ktimer_begin right before it, ktimer_mark right after it,
// tagged with its kind (APPNP_KT_*).  So an interval covers that launch only, never a wait that
// precedes it on the stream.  Off: one thread-local load each.
void ktimer_begin(hipStream_t s);
void ktimer_mark(hipStream_t s, int kind);

// Leading dimension of the internal ping-pong buffers.  A random row gather costs 128-B line
// requests, not bytes, so rows are padded to start on a line
// (next power of two up to one line, then whole lines) -- but only when that lowers the
// average number of lines a row spans; otherwise (e.g. 400-B fp32 rows: 4 lines either way)
// packed rows avoid a partially written line per row.
inline double avg_lines(int64_t row_bytes, int64_t stride) {
  // rows start at offsets (i * stride) mod 128, periodic
  int64_t g = stride % 128 == 0 ? 128 : stride;
  int64_t a = 128, b = g;
  while (b) { const int64_t t = a % b; a = b; b = t; }
  const int64_t period = 128 / a;
  double sum = 0.0;
  for (int64_t i = 0; i < period; ++i) {
    const int64_t o = (i * stride) % 128;
    sum += (double)((o + row_bytes - 1) / 128 + 1);
  }
  return sum / (double)period;
}

inline int64_t line_ld(int64_t f, int dtype) {
  const int64_t es = dtype == APPNP_F32 ? 4 : 2;
  const int64_t line = 128 / es;
  if (f <= 0) return 1;
  int64_t padded;
  if (f <= line) {
    padded = 1;
    while (padded < f) padded <<= 1;
  } else {
    padded = (f + line - 1) / line * line;
  }
  const int64_t v = es == 4 ? 4 : 8;  // keep 16-B vectors possible for the packed layout
  const int64_t packed = (f + v - 1) / v * v;
  return avg_lines(f * es, padded * es) < avg_lines(f * es, packed * es) ? padded : packed;
}

}  // namespace appnp
