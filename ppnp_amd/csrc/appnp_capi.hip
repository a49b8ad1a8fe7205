// appnp_capi.hip -- the extern "C" boundary declared in include/ppnp_amd.h.
//
// Argument validation, workspace ping-pong and the K-iteration launch sequence.  No host
// synchronisation or allocation happens in appnp_propagate / appnp_propagate_bwd /
// appnp_step, so a caller may capture them in a hipGraph.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <new>
#include <string>
#include <vector>

#include "../../include/ppnp_amd.h"
#include "appnp_internal.h"

using appnp::StepArgs;

namespace appnp {
namespace {

// appnp_kernel_timer_*: two timing events per launch, recorded on the launch's stream right
// before and right after it
struct KTimer {
  bool on = false;
  int dropped = 0;              // launches past the capacity (not timed)
  std::vector<hipEvent_t> ev;   // ev[2 i]: before launch i; ev[2 i + 1]: after it
  std::vector<int> kind;
  int n = 0;                    // launches recorded
  bool open = false;            // ev[2 n] recorded, its launch's end not yet
  bool over = false;            // the launch begun now is past the capacity
  hipStream_t open_s = nullptr;

  void release() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    ev.clear();
    kind.clear();
    n = dropped = 0;
    on = open = over = false;
    open_s = nullptr;
  }
};
thread_local KTimer g_ktimer;

}  // namespace

void ktimer_begin(hipStream_t s) {
  KTimer& t = g_ktimer;
  if (!t.on) return;
  t.open = false;
  t.over = 2 * t.n + 1 >= (int)t.ev.size();
  if (!t.over && hipEventRecord(t.ev[2 * t.n], s) == hipSuccess) {
    t.open = true;
    t.open_s = s;
  }
}

void ktimer_mark(hipStream_t s, int kind) {
  KTimer& t = g_ktimer;
  if (!t.on) return;
  if (t.over) {
    ++t.dropped;
    t.over = false;
    return;
  }
  if (!t.open || t.open_s != s) return;  // no begin on this stream: not a timed launch
  t.open = false;
  if (hipEventRecord(t.ev[2 * t.n + 1], s) != hipSuccess) {
    ++t.dropped;
    return;
  }
  t.kind[t.n] = kind;
  ++t.n;
}

// Every tuning override the library reads (tuning_env).  They change which kernel variant runs
// or how it is shaped, never results beyond fp32 summation order, and exist for the sweeps of
// tools/; a product run leaves APPNP_TUNING unset and gets the measured defaults.
const char* const kTuningNames[] = {
    "APPNP_SPLIT",       "APPNP_VEC",         "APPNP_WIDE",         "APPNP_UW",
    "APPNP_UN",          "APPNP_NT",          "APPNP_MAX_BLOCKS",   "APPNP_REM_SYNC_W4",
    "APPNP_REM_SYNC_W8", "APPNP_REM_SYNC_W16", "APPNP_SB_ROWS",     "APPNP_REM_VF"};

bool tuning_on() {
  static const bool on = [] {
    const char* v = getenv("APPNP_TUNING");
    return v && v[0] == '1' && v[1] == '\0';
  }();
  return on;
}

int tuning_env(const char* name, int dflt) {
  if (!tuning_on()) return dflt;
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

}  // namespace appnp

namespace {

using appnp::ktimer_begin;
using appnp::ktimer_mark;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int dev_err(hipError_t e) {
  if (e == hipSuccess) return APPNP_OK;
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return APPNP_ENOMEM;
  if (e == hipErrorInvalidValue) return APPNP_EINVAL;
  return APPNP_EDEVICE;
}

inline int64_t elem_size(int dtype) { return dtype == APPNP_F32 ? 4 : 2; }

inline bool valid_dtype(int dtype) { return dtype == APPNP_F32 || dtype == APPNP_BF16; }

using appnp::line_ld;  // appnp_internal.h

// Per-iteration dropout parameters (identical to oracle/ppnp_oracle.py edge_keep_mask).
void set_drop(StepArgs& a, float p_drop, uint64_t seed, int k) {
  if (p_drop > 0.0f) {
    a.mkey = appnp::splitmix64(seed + (uint64_t)(k + 1) * 0x9E3779B97F4A7C15ull);
    double thr = (double)p_drop * (double)(1u << 24);
    a.drop_thr = (uint32_t)thr;
    a.drop_on = 1;  // even when the 24-bit threshold rounds to 0, kept edges are rescaled
    a.drop_scale = 1.0f / (1.0f - p_drop);
  } else {
    a.mkey = 0;
    a.drop_thr = 0u;
    a.drop_on = 0;
    a.drop_scale = 1.0f;
  }
}

int check_common(const appnp_graph* g, int64_t f, int dtype, int K, float alpha, float p_drop) {
  if (!g) return APPNP_EINVAL;
  if (f < 0 || f > INT32_MAX || K < 0 || !valid_dtype(dtype)) return APPNP_EINVAL;
  if (!(alpha >= 0.0f && alpha <= 1.0f)) return APPNP_EINVAL;
  if (!(p_drop >= 0.0f && p_drop < 1.0f)) return APPNP_EINVAL;
  return APPNP_OK;
}

StepArgs base_args(const appnp_graph* g, int64_t f, float alpha) {
  StepArgs a{};
  a.row_ptr = g->row_ptr;
  a.col = g->col;
  a.val = g->val;
  a.n_rows = g->row_hi - g->row_lo;
  a.nnz = g->nnz_hat;
  a.nnz_rows = g->nnz_hat;  // a step over part of the rows' entries overrides nnz only
  a.zin_rows = g->n;
  a.row_lo = g->row_lo;
  a.f = (int32_t)f;
  a.scale = 1.0f - alpha;
  a.alpha = alpha;
  a.drop_scale = 1.0f;
  a.heavy = g->heavy;
  a.n_heavy = g->n_heavy;
  a.heavy_thr = appnp::kHeavyRow;
  a.hub = g->hub;
  a.n_hub = g->n_hub;
  return a;
}

constexpr double kSplitMaxNear = 0.5;

// the timer kind of an appnp_step / appnp_step_split launch on `part`
inline int part_kind(int part) {
  return part == APPNP_PART_LOCAL ? APPNP_KT_LOCAL
                                  : part == APPNP_PART_REMOTE ? APPNP_KT_REMOTE : APPNP_KT_STEP;
}  // split rows only below this gather locality

// Whether every operand allows 16-B vectors: leading dimensions multiples of 4 floats and
// 16-B aligned base pointers (null pointers ignored).  The split path reads and writes H / Z
// (dZ / dH) in 16-B pieces: the split copy, the main kernel at V = 4 and the remainder epilogue.
bool vec16(const int64_t* lds, int n_ld, const void* const* ptrs, int n_ptr) {
  for (int i = 0; i < n_ld; ++i)
    if (lds[i] % 4) return false;
  for (int i = 0; i < n_ptr; ++i)
    if (ptrs[i] && (reinterpret_cast<uintptr_t>(ptrs[i]) % 16)) return false;
  return true;
}

// Split rows (appnp_blocks.hip): the remainder columns r of fp32 rows of F = 32q + r features run
// as a separate chain of persistent L2-resident passes over the source-blocked A_hat, and the
// main part f - r (a multiple of 32, possibly 0) gathers whole lines from the split layout
// [n, 32q].  1-4 columns on a graph built with APPNP_GRAPH_SOURCE_BLOCKS, up to 8 with
// APPNP_GRAPH_SB_W8; narrow rows (f <= 4 rb_lpe: 4 / 8 / 16 with _W16) run wholly in the pass.
// Returns 0 (rows gathered whole) when the path does not apply: no blocked copy, bf16,
// latency-regime graph, F outside [1, 256], operands that do not allow 16-B vectors
// (``aligned``), or a graph with gather locality.  APPNP_SPLIT=0 disables it (measurement).
int64_t remainder_cols(const appnp_graph* g, int64_t f, int dtype, bool aligned) {
  static const int enabled = appnp::tuning_env("APPNP_SPLIT", 1);
  if (!enabled || !g->rb_off || dtype != APPNP_F32 || !aligned) return 0;
  if (g->n <= (1 << 16) || f < 1 || f > 256) return 0;
  // graphs with gather locality keep whole rows: their last line is mostly an L2 hit, cheaper
  // than the remainder pass (products-local, ~90 % near entries: 4.0 ms whole rows, 3.7 ms for
  // the 3-line main part alone, 8.5 ms split).  Uniform products-synth: 1.3 % near.
  if (g->near_frac > kSplitMaxNear && enabled != 2) return 0;  // APPNP_SPLIT=2: regardless
  const int64_t w = 4 * (int64_t)g->rb_lpe;
  const int64_t r = f > 32 ? f % 32 : f;
  if (f <= 32 && f > w) return 0;  // one line per row already, or too wide for the pass
  // beside a main part, a remainder of 9-16 columns costs as much as its extra line
  // (products-synth F = 47: 4.53 ms split against 4.41 ms whole rows; F = 40 = 32 + 8: 3.68
  // against 4.44 ms; profiles/r2_wide_remainder.txt)
  if (f > 32 && r > 8) return 0;
  // and beside a main part, the 4-lane pass of a W16 copy (4 row passes) costs more than the
  // extra line even for r <= 4 (products-synth F = 100: 9.44 ms split on W16 against 9.20 whole
  // rows and 7.77 on W4; F = 36: 4.50 against 4.42; profiles/r3_wide_copy_f100.txt).
  // A W8 copy still wins there (F = 100: 8.21 ms), so only W16 keeps whole rows
  if (f > 32 && g->rb_lpe == 4) return 0;
  return (r >= 1 && r <= w) ? r : 0;
}

// the main part of the split (columns [0, fs)), 0 when there is no split or no main part
int64_t split_point(const appnp_graph* g, int64_t f, int dtype, bool aligned) {
  const int64_t r = remainder_cols(g, f, dtype, aligned);
  return r ? f - r : 0;
}

// Bytes of the two split buffers ([n, fs] + [n, 4 rb_lpe] fp32 each, 256-B aligned)
inline void split_sizes(const appnp_graph* g, int64_t n, int64_t fs, int64_t* main_b,
                        int64_t* buf_b) {
  *main_b = (n * fs * 4 + 255) / 256 * 256;
  *buf_b = (*main_b + n * 16 * g->rb_lpe + 255) / 256 * 256;
}

// The forward loop in the split layout (appnp_blocks.hip).  Propagation is column-separable,
// so the main columns [0, fs) and the remainder columns [fs, f) are two independent K-step
// chains that meet only in Z:
//   * H is copied once into split buffer 0 (main part [n, fs], remainder part [n, 4]);
//   * main chain: K launches of the SpMM kernel on fs columns, gathering whole lines of the
//     main parts (ping-pong between the two buffers, the last into Z[:, :fs]);
//   * remainder chain: K persistent L2-resident passes over the remainder parts (the last
//     into Z[:, fs:f]).
// The chains touch disjoint parts of the buffers and disjoint columns of Z.  Both run on the
// caller's stream: on a side stream they overlapped in time but shared the memory system, and
// the total measured within 1 % of running them one after the other.
int propagate_split(const appnp_graph* g, const StepArgs& a0, const void* H, int64_t ld_h,
                    void* Z, int64_t ld_z, int64_t fs, int K, float p_drop, uint64_t seed,
                    char* ws, int64_t main_b, int64_t buf_b, hipStream_t s) {
  const int64_t n = a0.n_rows, f = a0.f;
  const int lpe = g->rb_lpe, rw = 4 * lpe;  // floats per remainder row
  char* bufs[2] = {ws, ws + buf_b};
  auto main_of = [&](int i) { return reinterpret_cast<float*>(bufs[i]); };
  auto rem_of = [&](int i) { return reinterpret_cast<float*>(bufs[i] + main_b); };
  const float* h = static_cast<const float*>(H);
  float* z = static_cast<float*>(Z);
  ktimer_begin(s);
  int rc = dev_err(appnp::launch_split_copy(h, ld_h, n, f, fs, rw, main_of(0), rem_of(0),
                                            appnp::remainder_scale(g), s));
  ktimer_mark(s, APPNP_KT_COPY);
  g->rem_launches.fetch_add(K, std::memory_order_relaxed);
  StepArgs am = a0, ar = a0;  // main / remainder chain
  am.f = (int32_t)fs;
  am.h = H;
  am.ld_h = ld_h;
  am.ld_in = fs;
  int cur = 0;
  for (int k = 0; k < K && !rc; ++k) {
    const int dst = cur ^ 1;
    const bool last = k == K - 1;
    set_drop(am, p_drop, seed, k);
    am.zin = main_of(cur);
    am.out = last ? Z : main_of(dst);
    am.ld_out = last ? ld_z : fs;
    if (fs > 0) {
      ktimer_begin(s);
      rc = dev_err(appnp::launch_step(APPNP_F32, appnp::EPI_FWD, 4, am, s));
      ktimer_mark(s, APPNP_KT_STEP);
    }
    if (rc) break;
    set_drop(ar, p_drop, seed, k);
    // LPE = 1: nv = 4 into the next remainder buffer (the shipped form); LPE > 1: nv is always
    // the valid remainder columns, to_rem says where the row goes
    const int nv = (lpe == 1 && !last) ? 4 : (int)(f - fs);
    ktimer_begin(s);
    rc = dev_err(appnp::launch_remainder(g, ar, appnp::EPI_FWD, rem_of(cur), h + fs, ld_h,
                                         last ? z + fs : rem_of(dst), last ? ld_z : rw, nv,
                                         !last, s));
    ktimer_mark(s, APPNP_KT_REM);
    cur = dst;
  }
  return rc;
}

// The adjoint loop in the split layout: the same two independent chains as propagate_split,
// run backwards (G_K = dZ, G_k = (1-alpha) M_k^T G_{k+1}, dH += alpha' G_k), for a
// self-adjoint A_hat.  dH = alpha dZ is set by the caller.
int propagate_bwd_split(const appnp_graph* g, const StepArgs& a0, const void* dZ, int64_t ld_dz,
                        void* dH, int64_t ld_dh, int64_t fs, int K, float alpha, float p_drop,
                        uint64_t seed, char* ws, int64_t main_b, int64_t buf_b,
                        hipStream_t s) {
  const int64_t n = a0.n_rows, f = a0.f;
  const int lpe = g->rb_lpe, rw = 4 * lpe;
  char* bufs[2] = {ws, ws + buf_b};
  auto main_of = [&](int i) { return reinterpret_cast<float*>(bufs[i]); };
  auto rem_of = [&](int i) { return reinterpret_cast<float*>(bufs[i] + main_b); };
  ktimer_begin(s);
  int rc = dev_err(appnp::launch_split_copy(static_cast<const float*>(dZ), ld_dz, n, f, fs, rw,
                                            main_of(0), rem_of(0), appnp::remainder_scale(g),
                                            s));
  ktimer_mark(s, APPNP_KT_COPY);
  g->rem_launches.fetch_add(K, std::memory_order_relaxed);
  StepArgs am = a0, ar = a0;  // main / remainder chain
  am.f = (int32_t)fs;
  am.aux = dH;
  am.ld_aux = ld_dh;
  am.ld_in = fs;
  am.ld_out = fs;
  float* dh_rem = static_cast<float*>(dH) + fs;
  int cur = 0;
  for (int k = K - 1; k >= 0 && !rc; --k) {
    const int dst = cur ^ 1;
    const float a_k = k >= 1 ? alpha : 1.0f;
    set_drop(am, p_drop, seed, k);
    am.alpha = a_k;
    am.zin = main_of(cur);
    am.out = k == 0 ? nullptr : main_of(dst);
    if (fs > 0) {
      ktimer_begin(s);
      rc = dev_err(appnp::launch_step(APPNP_F32, appnp::EPI_BWD, 4, am, s));
      ktimer_mark(s, APPNP_KT_STEP);
    }
    if (rc) break;
    set_drop(ar, p_drop, seed, k);
    ar.alpha = a_k;
    ktimer_begin(s);
    rc = dev_err(appnp::launch_remainder(g, ar, appnp::EPI_BWD, rem_of(cur), dh_rem, ld_dh,
                                         k == 0 ? nullptr : rem_of(dst), rw, (int)(f - fs),
                                         true, s));
    ktimer_mark(s, APPNP_KT_REM);
    cur = dst;
  }
  return rc;
}

}  // namespace

extern "C" {

int appnp_abi_version(void) { return PPNP_AMD_ABI_VERSION; }

#ifndef APPNP_SRC_DIGEST
#define APPNP_SRC_DIGEST "unknown"
#endif
#define APPNP_STR2(x) #x
#define APPNP_STR(x) APPNP_STR2(x)

#ifndef APPNP_ARCH
#define APPNP_ARCH "unknown"
#endif

const char* appnp_build_info(void) {
  return "src=" APPNP_SRC_DIGEST ";abi=" APPNP_STR(PPNP_AMD_ABI_VERSION) ";arch=" APPNP_ARCH
#ifdef APPNP_TESTING
      ";testing=1"
#endif
      ";compiler=" __VERSION__ ";built=" __DATE__ " " __TIME__;
}

const char* appnp_strerror(int code) {
  switch (code) {
    case APPNP_OK: return "ok";
    case APPNP_EDEVICE: return "HIP device error";
    case APPNP_ENOMEM: return "out of device memory";
    case APPNP_EINVAL: return "invalid argument";
    case APPNP_ERANGE: return "size exceeds int32 CSR index range";
    case APPNP_ENOTSUP: return "not supported";
    default: return "unknown error";
  }
}

int appnp_graph_create_rows(const int32_t* indptr, const int32_t* indices, const float* vals,
                            int64_t n, int64_t nnz, int mode, int64_t row_lo, int64_t row_hi,
                            int split_local, void* stream, appnp_graph** out) {
  if (!out) return APPNP_EINVAL;
  *out = nullptr;
  if (n < 0 || nnz < 0 || n > INT32_MAX || nnz > INT32_MAX) return n > INT32_MAX || nnz > INT32_MAX ? APPNP_ERANGE : APPNP_EINVAL;
  const bool want_t = (mode & APPNP_GRAPH_TRANSPOSE) != 0;
  // remainder width of the source-blocked copy: 4 columns, or 8 / 16 (APPNP_GRAPH_SB_W8 / _W16)
  const int sb_lpe = (mode & APPNP_GRAPH_SB_W16) ? 4 : (mode & APPNP_GRAPH_SB_W8) ? 2 : 1;
  const bool want_sb = (mode & (APPNP_GRAPH_SOURCE_BLOCKS | APPNP_GRAPH_SB_W8 |
                                APPNP_GRAPH_SB_W16)) != 0;
  mode &= ~(APPNP_GRAPH_TRANSPOSE | APPNP_GRAPH_SOURCE_BLOCKS | APPNP_GRAPH_SB_W8 |
            APPNP_GRAPH_SB_W16);
  if (mode != APPNP_NORM_SYM && mode != APPNP_NORM_RW) return APPNP_EINVAL;
  if (row_lo < 0 || row_hi < row_lo || row_hi > n) return APPNP_EINVAL;
  if (want_t && (row_lo != 0 || row_hi != n)) return APPNP_EINVAL;
  if (n > 0 && !indptr) return APPNP_EINVAL;
  if (nnz > 0 && !indices) return APPNP_EINVAL;
  appnp_graph* g = new (std::nothrow) appnp_graph();
  if (!g) return APPNP_ENOMEM;
  int rc = appnp::graph_build(indptr, indices, vals, n, nnz, mode, row_lo, row_hi,
                              split_local, as_stream(stream), g);
  // A_hat^T for the adjoint, unless A_hat is symmetric already ('sym' on undirected A)
  if (rc == APPNP_OK && want_t && !(g->mode == APPNP_NORM_SYM && g->symmetric))
    rc = appnp::graph_build_transpose(g, as_stream(stream));
  // source-blocked copy for the remainder pass (appnp_propagate on a full graph,
  // appnp_step_split on the held rows of a row-partitioned one).  Best-effort: a graph too
  // large for the copy (block or segment count, device memory) keeps whole-row gathers --
  // appnp_graph_source_blocks reports whether it was built.
  if (rc == APPNP_OK && want_sb) {
    const int sb =
        appnp::graph_build_source_blocks(g, sb_lpe, indptr, indices, nnz, as_stream(stream));
    if (sb != APPNP_OK && sb != APPNP_ENOTSUP && sb != APPNP_ERANGE && sb != APPNP_ENOMEM)
      rc = sb;
  }
  if (rc != APPNP_OK) {
    appnp::graph_free(g);
    delete g;
    return rc;
  }
  *out = g;
  return APPNP_OK;
}

int appnp_graph_create(const int32_t* indptr, const int32_t* indices, const float* vals,
                       int64_t n, int64_t nnz, int mode, void* stream, appnp_graph** out) {
  return appnp_graph_create_rows(indptr, indices, vals, n, nnz, mode, 0, n, 0, stream, out);
}

void appnp_graph_destroy(appnp_graph* g) {
  if (!g) return;
  appnp::graph_free(g);
  delete g;
}

int appnp_graph_info(const appnp_graph* g, int64_t* n, int64_t* row_lo, int64_t* row_hi,
                     int64_t* nnz_hat, int* mode, int* symmetric) {
  if (!g) return APPNP_EINVAL;
  if (n) *n = g->n;
  if (row_lo) *row_lo = g->row_lo;
  if (row_hi) *row_hi = g->row_hi;
  if (nnz_hat) *nnz_hat = g->nnz_hat;
  if (mode) *mode = g->mode;
  if (symmetric) *symmetric = g->symmetric;
  return APPNP_OK;
}

int appnp_graph_csr(const appnp_graph* g, const int32_t** row_ptr, const int32_t** col,
                    const float** val) {
  if (!g) return APPNP_EINVAL;
  if (row_ptr) *row_ptr = g->row_ptr;
  if (col) *col = g->col;
  if (val) *val = g->val;
  return APPNP_OK;
}

int appnp_graph_copy_csr(const appnp_graph* g, int32_t* row_ptr, int32_t* col, float* val,
                         double* dinv, void* stream) {
  if (!g) return APPNP_EINVAL;
  const hipStream_t s = as_stream(stream);
  const int64_t rows = g->row_hi - g->row_lo;
  hipError_t e = hipSuccess;
  if (row_ptr && e == hipSuccess)
    e = hipMemcpyAsync(row_ptr, g->row_ptr, (rows + 1) * sizeof(int32_t), hipMemcpyDeviceToDevice, s);
  if (col && g->nnz_hat && e == hipSuccess)
    e = hipMemcpyAsync(col, g->col, g->nnz_hat * sizeof(int32_t), hipMemcpyDeviceToDevice, s);
  if (val && g->nnz_hat && e == hipSuccess)
    e = hipMemcpyAsync(val, g->val, g->nnz_hat * sizeof(float), hipMemcpyDeviceToDevice, s);
  if (dinv && g->n && e == hipSuccess)
    e = hipMemcpyAsync(dinv, g->dinv, g->n * sizeof(double), hipMemcpyDeviceToDevice, s);
  return dev_err(e);
}

int appnp_graph_dinv(const appnp_graph* g, const double** dinv) {
  if (!g || !dinv) return APPNP_EINVAL;
  *dinv = g->dinv;
  return APPNP_OK;
}

size_t appnp_workspace_bytes(const appnp_graph* g, int64_t f, int64_t ld, int dtype) {
  if (!g || f < 0 || !valid_dtype(dtype)) return 0;
  (void)ld;  // the workspace uses its own line-aligned leading dimension
  const int64_t rows = g->row_hi - g->row_lo;
  // two ping-pong buffers (the forward needs one, the adjoint two), 256-B aligned each
  int64_t need = 2 * rows * line_ld(f, dtype) * elem_size(dtype) + 2048;
  // the split layout: two buffers [n, fs] + [n, 4 rb_lpe] (a W8 / W16 remainder row is wider
  // than the packed row's tail), plus the alignment of the base
  const int64_t r = (g->row_lo == 0 && g->row_hi == g->n) ? remainder_cols(g, f, dtype, true) : 0;
  if (r > 0) {
    int64_t main_b = 0, buf_b = 0;
    split_sizes(g, rows, f - r, &main_b, &buf_b);
    need = std::max<int64_t>(need, 2 * buf_b + 256);
  }
  return (size_t)need;
}

int appnp_graph_source_blocks(const appnp_graph* g, int64_t* bytes) {
  if (!g || !bytes) return APPNP_EINVAL;
  *bytes = 0;
  if (g->rb_off)
    *bytes = g->rb_total * (g->rb_val ? 8 : 4) + g->rb_total / 16 * g->rb_lpe +
             ((int64_t)g->rb_passes * g->rb_nb * g->rb_slots + 1) * (int64_t)sizeof(int32_t) +
             (g->rb_dl ? g->n * 4 : 0) + (g->rb_dr ? g->n * 4 : 0);
  return APPNP_OK;
}

int appnp_graph_source_block_layout(const appnp_graph* g, int* width, int64_t* entries,
                                    int* value_free, int* row_passes, int64_t* launches) {
  if (!g) return APPNP_EINVAL;
  const bool built = g->rb_off != nullptr;
  if (width) *width = built ? 4 * g->rb_lpe : 0;
  if (entries) *entries = built ? g->rb_total : 0;
  if (value_free) *value_free = built && g->rb_val == nullptr ? 1 : 0;
  if (row_passes) *row_passes = built ? g->rb_passes : 0;
  if (launches) *launches = g->rem_launches.load(std::memory_order_relaxed);
  return APPNP_OK;
}

int appnp_propagate_split_point(const appnp_graph* g, int64_t f, int dtype, int64_t* fs) {
  if (!g || !fs || f < 0 || !valid_dtype(dtype)) return APPNP_EINVAL;
  *fs = split_point(g, f, dtype, true);
  return APPNP_OK;
}

int appnp_propagate_remainder_cols(const appnp_graph* g, int64_t f, int dtype, int64_t* r) {
  if (!g || !r || f < 0 || !valid_dtype(dtype)) return APPNP_EINVAL;
  *r = remainder_cols(g, f, dtype, true);
  return APPNP_OK;
}

int appnp_propagate(const appnp_graph* g, const void* H, int64_t ld_h, void* Z, int64_t ld_z,
                    int64_t f, int dtype, int K, float alpha, float p_drop, uint64_t seed,
                    void* ws, size_t ws_bytes, void* stream) {
  int rc = check_common(g, f, dtype, K, alpha, p_drop);
  if (rc) return rc;
  if (g->row_lo != 0 || g->row_hi != g->n) return APPNP_EINVAL;  // needs the whole graph
  const int64_t n = g->n;
  if (n == 0 || f == 0) return APPNP_OK;
  if (!H || !Z || ld_h < f || ld_z < f || H == Z) return APPNP_EINVAL;
  const hipStream_t s = as_stream(stream);
  const int64_t es = elem_size(dtype);
  if (K == 0) {
    ktimer_begin(s);
    rc = dev_err(hipMemcpy2DAsync(Z, ld_z * es, H, ld_h * es, f * es, n,
                                  hipMemcpyDeviceToDevice, s));
    ktimer_mark(s, APPNP_KT_COPY);
    return rc;
  }
  const int64_t ld_w = line_ld(f, dtype);
  void* const ws_orig = ws;
  if (K >= 2) {
    if (!ws) return APPNP_EINVAL;
    const uintptr_t base = reinterpret_cast<uintptr_t>(ws);
    const uintptr_t aligned = (base + 255) & ~uintptr_t(255);
    if (ws_bytes < (size_t)(n * ld_w * es) + (aligned - base)) return APPNP_EINVAL;
    ws = reinterpret_cast<void*>(aligned);
  }
  const int64_t lds[3] = {ld_h, ld_z, ld_w};
  const void* ptrs[3] = {H, Z, K >= 2 ? ws : nullptr};
  const int V = appnp::pick_vec(dtype, f, lds, 3, ptrs, 3);

  StepArgs a = base_args(g, f, alpha);
  a.h = H;
  a.ld_h = ld_h;
  const int64_t hz_lds[2] = {ld_h, ld_z};
  const void* hz[2] = {H, Z};
  const int64_t r = K >= 2 ? remainder_cols(g, f, dtype, vec16(hz_lds, 2, hz, 2)) : 0;
  if (r > 0) {
    // two split buffers [n, fs] + [n, 4 rb_lpe] fp32 in the workspace, each 256-B aligned
    // (fs = 0: narrow rows, all in the remainder pass)
    const int64_t fs = f - r;
    int64_t main_b = 0, buf_b = 0;
    split_sizes(g, n, fs, &main_b, &buf_b);
    const size_t used = (size_t)(reinterpret_cast<uintptr_t>(ws) -
                                 reinterpret_cast<uintptr_t>(ws_orig));
    if (ws_bytes >= used + 2 * (size_t)buf_b)
      return propagate_split(g, a, H, ld_h, Z, ld_z, fs, K, p_drop, seed,
                             static_cast<char*>(ws), main_b, buf_b, s);
  }
  const void* src = H;
  int64_t ld_src = ld_h;
  for (int k = 0; k < K; ++k) {
    // the last iteration must land in Z: alternate backwards from it
    const bool to_z = ((K - 1 - k) % 2) == 0;
    void* dst = to_z ? Z : ws;
    const int64_t ld_dst = to_z ? ld_z : ld_w;
    a.zin = src;
    a.ld_in = ld_src;
    a.out = dst;
    a.ld_out = ld_dst;
    set_drop(a, p_drop, seed, k);
    ktimer_begin(s);
    rc = dev_err(appnp::launch_step(dtype, appnp::EPI_FWD, V, a, s));
    ktimer_mark(s, APPNP_KT_STEP);
    if (rc) return rc;
    src = dst;
    ld_src = ld_dst;
  }
  return APPNP_OK;
}

int appnp_propagate_bwd(const appnp_graph* g, const void* dZ, int64_t ld_dz, void* dH,
                        int64_t ld_dh, int64_t f, int dtype, int K, float alpha, float p_drop,
                        uint64_t seed, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_common(g, f, dtype, K, alpha, p_drop);
  if (rc) return rc;
  if (g->row_lo != 0 || g->row_hi != g->n) return APPNP_EINVAL;
  // A_hat^T: A_hat itself for 'sym' on an undirected graph, else the transposed CSR built at
  // creation (APPNP_GRAPH_TRANSPOSE)
  const bool self_adjoint = g->mode == APPNP_NORM_SYM && g->symmetric;
  if (!self_adjoint && !g->t_row_ptr) return APPNP_ENOTSUP;
  const int64_t n = g->n;
  if (n == 0 || f == 0) return APPNP_OK;
  if (!dZ || !dH || ld_dz < f || ld_dh < f || dZ == dH) return APPNP_EINVAL;
  const hipStream_t s = as_stream(stream);
  const int64_t es = elem_size(dtype);
  if (K == 0) {
    ktimer_begin(s);
    rc = dev_err(hipMemcpy2DAsync(dH, ld_dh * es, dZ, ld_dz * es, f * es, n,
                                  hipMemcpyDeviceToDevice, s));
    ktimer_mark(s, APPNP_KT_COPY);
    return rc;
  }
  const int64_t ld_w = line_ld(f, dtype);
  const int64_t buf = n * ld_w * es;
  const int nbuf = K >= 3 ? 2 : (K == 2 ? 1 : 0);
  void* const ws_orig = ws;
  if (nbuf > 0) {
    if (!ws) return APPNP_EINVAL;
    const uintptr_t base = reinterpret_cast<uintptr_t>(ws);
    const uintptr_t aligned = (base + 255) & ~uintptr_t(255);
    if (ws_bytes < (size_t)(nbuf * buf) + (aligned - base)) return APPNP_EINVAL;
    ws = reinterpret_cast<void*>(aligned);
  }
  void* w0 = ws;
  void* w1 = nbuf == 2 ? static_cast<char*>(ws) + buf : nullptr;
  const int64_t lds[3] = {ld_dz, ld_dh, ld_w};
  const void* ptrs[4] = {dZ, dH, w0, w1};
  const int V = appnp::pick_vec(dtype, f, lds, 3, ptrs, 4);

  // dH = alpha * dZ  (the k = K term), then G_k = (1-alpha) M_k^T G_{k+1},
  // dH += alpha G_k (k >= 1) / dH += G_0.
  ktimer_begin(s);
  rc = dev_err(appnp::launch_scale_rows(dtype, dZ, ld_dz, dH, ld_dh, n, f, alpha, s));
  ktimer_mark(s, APPNP_KT_COPY);
  if (rc) return rc;
  // split rows (self-adjoint A_hat: the source-blocked copy of A_hat is that of A_hat^T)
  const int64_t dd_lds[2] = {ld_dz, ld_dh};
  const void* dd[2] = {dZ, dH};
  const int64_t r =
      (self_adjoint && K >= 2) ? remainder_cols(g, f, dtype, vec16(dd_lds, 2, dd, 2)) : 0;
  const int64_t fs = f - r;
  int64_t main_b = 0, buf_b = 0;
  bool split = r > 0;
  if (split) {
    split_sizes(g, n, fs, &main_b, &buf_b);
    const size_t used = (size_t)(reinterpret_cast<uintptr_t>(ws) -
                                 reinterpret_cast<uintptr_t>(ws_orig));
    if (ws_bytes < used + 2 * (size_t)buf_b) split = false;  // too small: whole rows
  }
  StepArgs a = base_args(g, f, alpha);
  if (!self_adjoint) {
    a.row_ptr = g->t_row_ptr;
    a.col = g->t_col;
    a.val = g->t_val;
    a.heavy = g->t_heavy;
    a.n_heavy = g->t_n_heavy;
    a.hub = g->t_hub;
    a.n_hub = g->t_n_hub;
  }
  a.tkey = 1;  // entry (j, i) of A_hat^T carries the mask of forward edge (i, j)
  if (split)
    return propagate_bwd_split(g, a, dZ, ld_dz, dH, ld_dh, fs, K, alpha, p_drop, seed,
                               static_cast<char*>(ws), main_b, buf_b, s);
  a.aux = dH;
  a.ld_aux = ld_dh;
  const void* src = dZ;
  int64_t ld_src = ld_dz;
  int flip = 0;
  for (int k = K - 1; k >= 0; --k) {
    void* dst = k == 0 ? nullptr : (flip ? w1 : w0);
    a.zin = src;
    a.ld_in = ld_src;
    a.out = dst;
    a.ld_out = ld_w;
    a.alpha = k >= 1 ? alpha : 1.0f;
    set_drop(a, p_drop, seed, k);
    ktimer_begin(s);
    rc = dev_err(appnp::launch_step(dtype, appnp::EPI_BWD, V, a, s));
    ktimer_mark(s, APPNP_KT_STEP);
    if (rc) return rc;
    src = dst;
    ld_src = ld_w;
    flip ^= 1;
  }
  return APPNP_OK;
}

int appnp_spmm(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t rows,
               int64_t cols, const float* B, int64_t ld_b, float* Cm, int64_t ld_c, int64_t f,
               float p_drop, uint64_t seed, int transposed_key, void* stream) {
  if (rows < 0 || cols < 0 || f < 0 || f > INT32_MAX) return APPNP_EINVAL;
  if (!(p_drop >= 0.0f && p_drop < 1.0f)) return APPNP_EINVAL;
  if (rows == 0 || f == 0) return APPNP_OK;
  if (!indptr || !Cm || ld_c < f || (cols > 0 && (!B || ld_b < f))) return APPNP_EINVAL;
  StepArgs a{};
  a.row_ptr = indptr;
  a.col = indices;
  a.val = vals;
  a.zin = B;
  a.ld_in = ld_b;
  a.out = Cm;
  a.ld_out = ld_c;
  a.n_rows = rows;
  a.nnz = -1;  // not known on the host without a device read
  a.zin_rows = cols;
  a.row_lo = 0;
  a.f = (int32_t)f;
  a.scale = 1.0f;
  a.alpha = 0.0f;
  a.tkey = transposed_key ? 1 : 0;
  set_drop(a, p_drop, seed, 0);
  const int64_t lds[2] = {ld_b, ld_c};
  const void* ptrs[2] = {B, Cm};
  const int V = appnp::pick_vec(APPNP_F32, f, lds, 2, ptrs, 2);
  return dev_err(appnp::launch_step(APPNP_F32, appnp::EPI_PARTIAL, V, a, as_stream(stream)));
}

int appnp_step(const appnp_graph* g, int part, const void* Zin, int64_t ld_in, const void* H,
               int64_t ld_h, void* Zout, int64_t ld_out, const float* partial,
               int64_t ld_partial, int64_t f, int dtype, int k, float alpha, float p_drop,
               uint64_t seed, void* stream) {
  int rc = check_common(g, f, dtype, 0, alpha, p_drop);
  if (rc) return rc;
  if (k < 0) return APPNP_EINVAL;
  const int64_t rows = g->row_hi - g->row_lo;
  if (rows == 0 || f == 0) return APPNP_OK;
  if (!Zin || !Zout || ld_in < f || ld_out < f) return APPNP_EINVAL;
  StepArgs a = base_args(g, f, alpha);
  a.zin = Zin;
  a.ld_in = ld_in;
  a.out = Zout;
  a.ld_out = ld_out;
  set_drop(a, p_drop, seed, k);
  int epi = appnp::EPI_FWD;
  int64_t lds[4] = {ld_in, ld_out, ld_h, ld_partial};
  const void* ptrs[4] = {Zin, Zout, H, partial};
  int n_ld = 2;
  if (part == APPNP_PART_ALL) {
    if (!H || ld_h < f) return APPNP_EINVAL;
    a.h = H;
    a.ld_h = ld_h;
    n_ld = 3;
  } else {
    if (!g->split) return APPNP_EINVAL;
    if (dtype != APPNP_F32) return APPNP_ENOTSUP;
    a.heavy = nullptr;  // the heavy/hub lists describe the full rows, not their halves
    a.n_heavy = 0;
    a.hub = nullptr;
    a.n_hub = 0;
    if (part == APPNP_PART_LOCAL) {
      epi = appnp::EPI_PARTIAL;
      a.nnz = g->nnz_local;
      a.row_ptr = g->lrow_ptr;
      a.col = g->lcol;
      a.val = g->lval;
    } else if (part == APPNP_PART_REMOTE) {
      if (!H || ld_h < f || !partial || ld_partial < f) return APPNP_EINVAL;
      epi = appnp::EPI_FINISH;
      a.nnz = g->nnz_remote;
      a.row_ptr = g->rrow_ptr;
      a.col = g->rcol;
      a.val = g->rval;
      a.h = H;
      a.ld_h = ld_h;
      a.aux = const_cast<float*>(partial);
      a.ld_aux = ld_partial;
      n_ld = 4;
    } else {
      return APPNP_EINVAL;
    }
  }
  const int V = appnp::pick_vec(dtype, f, lds, n_ld, ptrs, 4);
  ktimer_begin(as_stream(stream));
  rc = dev_err(appnp::launch_step(dtype, epi, V, a, as_stream(stream)));
  ktimer_mark(as_stream(stream), part_kind(part));
  return rc;
}

// ---- the split layout on the held rows of a row-partitioned graph -------------------------

namespace {

// remainder columns of a held-rows split step (appnp_step_split / appnp_split_copy); 0: none
int64_t rows_split(const appnp_graph* g, int64_t f) {
  return g ? remainder_cols(g, f, APPNP_F32, true) : 0;
}

}  // namespace

int appnp_split_layout(const appnp_graph* g, int64_t f, int64_t* fs, int64_t* rem_width) {
  if (!g || f < 0) return APPNP_EINVAL;
  const int64_t r = rows_split(g, f);
  if (fs) *fs = r ? f - r : 0;
  if (rem_width) *rem_width = r ? 4 * (int64_t)g->rb_lpe : 0;
  return r ? APPNP_OK : APPNP_ENOTSUP;
}

int appnp_split_copy(const appnp_graph* g, const float* H, int64_t ld_h, int64_t f, float* main,
                     float* rem, void* stream) {
  if (!g || f <= 0) return APPNP_EINVAL;
  const int64_t r = rows_split(g, f);
  if (!r) return APPNP_ENOTSUP;
  const int64_t rows = g->row_hi - g->row_lo, fs = f - r, rw = 4 * (int64_t)g->rb_lpe;
  if (rows == 0) return APPNP_OK;
  const int64_t lds[1] = {ld_h};
  const void* ptrs[3] = {H, main, rem};
  if (!H || !rem || (fs > 0 && !main) || ld_h < f || !vec16(lds, 1, ptrs, 3)) return APPNP_EINVAL;
  const float* sc = appnp::remainder_scale(g);
  ktimer_begin(as_stream(stream));
  const int rc = dev_err(appnp::launch_split_copy(H, ld_h, rows, f, fs, rw,
                                                  main ? main + g->row_lo * fs : nullptr,
                                                  rem + g->row_lo * rw,
                                                  sc ? sc + g->row_lo : nullptr,
                                                  as_stream(stream)));
  ktimer_mark(as_stream(stream), APPNP_KT_COPY);
  return rc;
}

int appnp_step_split(const appnp_graph* g, int part, const float* zin_main, const float* zin_rem,
                     const float* H, int64_t ld_h, float* zout_main, float* zout_rem, float* Z,
                     int64_t ld_z, float* partial, int64_t ld_partial, int64_t f, int k,
                     float alpha, float p_drop, uint64_t seed, void* stream) {
  int rc = check_common(g, f, APPNP_F32, 0, alpha, p_drop);
  if (rc) return rc;
  if (k < 0 || part < APPNP_PART_ALL || part > APPNP_PART_REMOTE) return APPNP_EINVAL;
  const int64_t r = rows_split(g, f);
  if (!r) return APPNP_ENOTSUP;
  const int64_t rows = g->row_hi - g->row_lo, fs = f - r, rw = 4 * (int64_t)g->rb_lpe;
  if (rows == 0 || f == 0) return APPNP_OK;
  if (part != APPNP_PART_ALL && (!g->split || fs == 0)) return APPNP_EINVAL;
  const bool to_z = Z != nullptr;
  // inputs: every row of both parts (the remainder only where the pass runs)
  if (fs > 0 && !zin_main) return APPNP_EINVAL;
  if (part != APPNP_PART_LOCAL && !zin_rem) return APPNP_EINVAL;
  if (part != APPNP_PART_LOCAL && (!H || ld_h < f)) return APPNP_EINVAL;
  if (part != APPNP_PART_LOCAL && !to_z && (!zout_rem || (fs > 0 && !zout_main)))
    return APPNP_EINVAL;
  if (to_z && ld_z < f) return APPNP_EINVAL;
  if (part != APPNP_PART_ALL && (!partial || ld_partial < fs)) return APPNP_EINVAL;
  const int64_t lds[3] = {part != APPNP_PART_LOCAL ? ld_h : 4, to_z ? ld_z : 4,
                          part != APPNP_PART_ALL ? ld_partial : 4};
  const void* ptrs[8] = {zin_main, zin_rem, H, zout_main, zout_rem, Z, partial, nullptr};
  if (!vec16(lds, 3, ptrs, 7)) return APPNP_EINVAL;
  const hipStream_t s = as_stream(stream);
  StepArgs a = base_args(g, f, alpha);
  set_drop(a, p_drop, seed, k);
  if (fs > 0) {
    StepArgs am = a;
    am.f = (int32_t)fs;
    am.zin = zin_main;
    am.ld_in = fs;
    am.out = to_z ? static_cast<void*>(Z) : static_cast<void*>(zout_main + g->row_lo * fs);
    am.ld_out = to_z ? ld_z : fs;
    int epi = appnp::EPI_FWD;
    if (part == APPNP_PART_ALL) {
      am.h = H;
      am.ld_h = ld_h;
    } else {
      am.heavy = nullptr;  // the heavy / hub lists describe the full rows, not their halves
      am.n_heavy = 0;
      am.hub = nullptr;
      am.n_hub = 0;
      if (part == APPNP_PART_LOCAL) {
        epi = appnp::EPI_PARTIAL;
        am.nnz = g->nnz_local;
        am.row_ptr = g->lrow_ptr;
        am.col = g->lcol;
        am.val = g->lval;
        am.out = partial;
        am.ld_out = ld_partial;
      } else {
        epi = appnp::EPI_FINISH;
        am.nnz = g->nnz_remote;
        am.row_ptr = g->rrow_ptr;
        am.col = g->rcol;
        am.val = g->rval;
        am.h = H;
        am.ld_h = ld_h;
        am.aux = partial;
        am.ld_aux = ld_partial;
      }
    }
    ktimer_begin(s);
    rc = dev_err(appnp::launch_step(APPNP_F32, epi, 4, am, s));
    ktimer_mark(s, part_kind(part));
    if (rc) return rc;
  }
  if (part == APPNP_PART_LOCAL) return APPNP_OK;  // the pass needs every row of zin_rem
  // the remainder pass over every source block: into the next remainder buffer at the held
  // rows (a unit graph stores dr o y there), or into Z's last r columns
  const int nv = (g->rb_lpe == 1 && !to_z) ? 4 : (int)r;
  g->rem_launches.fetch_add(1, std::memory_order_relaxed);
  ktimer_begin(s);
  rc = dev_err(appnp::launch_remainder(g, a, appnp::EPI_FWD, zin_rem, H + fs, ld_h,
                                       to_z ? Z + fs : zout_rem + g->row_lo * rw,
                                       to_z ? ld_z : rw, nv, !to_z, s));
  ktimer_mark(s, APPNP_KT_REM);
  return rc;
}

// ---- pipelined row steps: the held rows' entries of a range of source shards -------------

int appnp_graph_shard_offsets(appnp_graph* g, int nshards, int64_t shard_rows, void* stream) {
  if (!g) return APPNP_EINVAL;
  return appnp::graph_build_shard_offsets(g, nshards, shard_rows, as_stream(stream));
}

namespace {

// The step's CSR restricted to the held rows' entries with a column in shards [s_lo, s_hi), and
// the epilogue of `mode` (appnp_shard_mode): FIRST partial = y, ACC partial += y, LAST out = y +
// partial + alpha H, ONLY out = y + alpha H.  Returns APPNP_OK or a code.
int shard_step_args(const appnp_graph* g, int s_lo, int s_hi, int mode, StepArgs& a, int* epi) {
  if (!g->sh_off) return APPNP_EINVAL;  // appnp_graph_shard_offsets first
  if (s_lo < 0 || s_hi > g->sh_n || s_lo >= s_hi) return APPNP_EINVAL;
  const int64_t rows = g->row_hi - g->row_lo;
  a.row_ptr = g->sh_off + (int64_t)s_lo * rows;
  a.row_end = g->sh_off + (int64_t)s_hi * rows;
  // the kernel shape follows the average row length: the range's share of the entries
  a.nnz = g->nnz_hat * (int64_t)(s_hi - s_lo) / g->sh_n;
  a.heavy = nullptr;  // the heavy / hub lists describe whole rows, not their shard ranges
  a.n_heavy = 0;
  a.hub = nullptr;
  a.n_hub = 0;
  switch (mode) {
    case APPNP_SHARDS_FIRST: *epi = appnp::EPI_PARTIAL; return APPNP_OK;
    case APPNP_SHARDS_ACC: *epi = appnp::EPI_ACCUM; return APPNP_OK;
    case APPNP_SHARDS_LAST: *epi = appnp::EPI_FINISH; return APPNP_OK;
    case APPNP_SHARDS_ONLY: *epi = appnp::EPI_FWD; return APPNP_OK;
    default: return APPNP_EINVAL;
  }
}

inline int shard_kind(int mode) {
  return mode == APPNP_SHARDS_FIRST ? APPNP_KT_LOCAL : APPNP_KT_REMOTE;
}

}  // namespace

int appnp_step_shards(const appnp_graph* g, int s_lo, int s_hi, int mode, const float* Zin,
                      int64_t ld_in, const float* H, int64_t ld_h, float* Zout, int64_t ld_out,
                      float* partial, int64_t ld_partial, int64_t f, int k, float alpha,
                      float p_drop, uint64_t seed, void* stream) {
  int rc = check_common(g, f, APPNP_F32, 0, alpha, p_drop);
  if (rc) return rc;
  if (k < 0) return APPNP_EINVAL;
  const int64_t rows = g->row_hi - g->row_lo;
  StepArgs a = base_args(g, f, alpha);
  int epi = appnp::EPI_FWD;
  rc = shard_step_args(g, s_lo, s_hi, mode, a, &epi);
  if (rc) return rc;
  if (rows == 0 || f == 0) return APPNP_OK;
  const bool to_partial = mode == APPNP_SHARDS_FIRST || mode == APPNP_SHARDS_ACC;
  const bool reads_partial = mode == APPNP_SHARDS_ACC || mode == APPNP_SHARDS_LAST;
  const bool reads_h = mode == APPNP_SHARDS_LAST || mode == APPNP_SHARDS_ONLY;
  if (!Zin || ld_in < f) return APPNP_EINVAL;
  if ((to_partial || reads_partial) && (!partial || ld_partial < f)) return APPNP_EINVAL;
  if (!to_partial && (!Zout || ld_out < f)) return APPNP_EINVAL;
  if (reads_h && (!H || ld_h < f)) return APPNP_EINVAL;
  a.zin = Zin;
  a.ld_in = ld_in;
  a.out = to_partial ? static_cast<void*>(partial) : static_cast<void*>(Zout);
  a.ld_out = to_partial ? ld_partial : ld_out;
  if (reads_h) {
    a.h = H;
    a.ld_h = ld_h;
  }
  if (mode == APPNP_SHARDS_LAST) {
    a.aux = partial;
    a.ld_aux = ld_partial;
  }
  set_drop(a, p_drop, seed, k);
  const int64_t lds[4] = {ld_in, a.ld_out, reads_h ? ld_h : ld_in,
                          reads_partial ? ld_partial : ld_in};
  const void* ptrs[4] = {Zin, a.out, reads_h ? H : nullptr, reads_partial ? partial : nullptr};
  const int V = appnp::pick_vec(APPNP_F32, f, lds, 4, ptrs, 4);
  const hipStream_t s = as_stream(stream);
  ktimer_begin(s);
  rc = dev_err(appnp::launch_step(APPNP_F32, epi, V, a, s));
  ktimer_mark(s, shard_kind(mode));
  return rc;
}

int appnp_step_split_shards(const appnp_graph* g, int s_lo, int s_hi, int mode,
                            const float* zin_main, const float* zin_rem, const float* H,
                            int64_t ld_h, float* zout_main, float* zout_rem, float* Z,
                            int64_t ld_z, float* partial, int64_t ld_partial, int64_t f, int k,
                            float alpha, float p_drop, uint64_t seed, void* stream) {
  int rc = check_common(g, f, APPNP_F32, 0, alpha, p_drop);
  if (rc) return rc;
  if (k < 0) return APPNP_EINVAL;
  const int64_t r = rows_split(g, f);
  if (!r) return APPNP_ENOTSUP;
  const int64_t rows = g->row_hi - g->row_lo, fs = f - r, rw = 4 * (int64_t)g->rb_lpe;
  StepArgs a = base_args(g, f, alpha);
  StepArgs am = a;
  int epi = appnp::EPI_FWD;
  rc = shard_step_args(g, s_lo, s_hi, mode, am, &epi);
  if (rc) return rc;
  if (rows == 0 || f == 0) return APPNP_OK;
  const bool to_partial = mode == APPNP_SHARDS_FIRST || mode == APPNP_SHARDS_ACC;
  const bool reads_partial = mode == APPNP_SHARDS_ACC || mode == APPNP_SHARDS_LAST;
  const bool finishes = !to_partial;  // LAST / ONLY: the row's output, then the remainder pass
  const bool to_z = Z != nullptr;
  if (fs == 0 && mode != APPNP_SHARDS_ONLY) return APPNP_EINVAL;  // nothing to pipeline
  if (fs > 0 && !zin_main) return APPNP_EINVAL;
  if (finishes && (!zin_rem || !H || ld_h < f)) return APPNP_EINVAL;
  if (finishes && !to_z && (!zout_rem || (fs > 0 && !zout_main))) return APPNP_EINVAL;
  if (to_z && ld_z < f) return APPNP_EINVAL;
  if ((to_partial || reads_partial) && (!partial || ld_partial < fs)) return APPNP_EINVAL;
  const int64_t lds[3] = {finishes ? ld_h : 4, to_z ? ld_z : 4,
                          (to_partial || reads_partial) ? ld_partial : 4};
  const void* ptrs[8] = {zin_main, zin_rem, H, zout_main, zout_rem, Z, partial, nullptr};
  if (!vec16(lds, 3, ptrs, 7)) return APPNP_EINVAL;
  const hipStream_t s = as_stream(stream);
  set_drop(a, p_drop, seed, k);
  set_drop(am, p_drop, seed, k);
  if (fs > 0) {
    am.f = (int32_t)fs;
    am.zin = zin_main;
    am.ld_in = fs;
    if (to_partial) {
      am.out = partial;
      am.ld_out = ld_partial;
    } else {
      am.out = to_z ? static_cast<void*>(Z) : static_cast<void*>(zout_main + g->row_lo * fs);
      am.ld_out = to_z ? ld_z : fs;
      am.h = H;
      am.ld_h = ld_h;
      if (reads_partial) {
        am.aux = partial;
        am.ld_aux = ld_partial;
      }
    }
    ktimer_begin(s);
    rc = dev_err(appnp::launch_step(APPNP_F32, epi, 4, am, s));
    ktimer_mark(s, shard_kind(mode));
    if (rc) return rc;
  }
  if (!finishes) return APPNP_OK;  // the pass needs every row of zin_rem
  const int nv = (g->rb_lpe == 1 && !to_z) ? 4 : (int)r;
  g->rem_launches.fetch_add(1, std::memory_order_relaxed);
  ktimer_begin(s);
  rc = dev_err(appnp::launch_remainder(g, a, appnp::EPI_FWD, zin_rem, H + fs, ld_h,
                                       to_z ? Z + fs : zout_rem + g->row_lo * rw,
                                       to_z ? ld_z : rw, nv, !to_z, s));
  ktimer_mark(s, APPNP_KT_REM);
  return rc;
}

// ---- the per-launch timer (measurement aid; include/ppnp_amd.h) ----------------------------

int appnp_kernel_timer_begin(int max_launches, void* stream) {
  appnp::KTimer& t = appnp::g_ktimer;
  if (max_launches < 1 || max_launches > (1 << 20)) return APPNP_EINVAL;
  t.release();
  t.ev.assign(2 * (size_t)max_launches, nullptr);
  t.kind.assign((size_t)max_launches, 0);
  for (hipEvent_t& e : t.ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      e = nullptr;
      t.release();
      return APPNP_EDEVICE;
    }
  }
  t.on = true;
  (void)stream;  // every launch is bracketed by events on its own stream (ktimer_begin / _mark)
  return APPNP_OK;
}

int appnp_kernel_timer_end(float* ms, int* kinds, int max, int* n_out) {
  appnp::KTimer& t = appnp::g_ktimer;
  if (!t.on) return APPNP_EINVAL;
  t.on = false;
  int rc = APPNP_OK;
  for (int i = 0; i < 2 * t.n && rc == APPNP_OK; ++i)
    rc = dev_err(hipEventSynchronize(t.ev[i]));
  for (int i = 0; i < t.n && i < max && rc == APPNP_OK; ++i) {
    float e = NAN;
    if (hipEventElapsedTime(&e, t.ev[2 * i], t.ev[2 * i + 1]) != hipSuccess) e = NAN;
    if (ms) ms[i] = e;
    if (kinds) kinds[i] = t.kind[i];
  }
  if (n_out) *n_out = t.n;
  if (rc == APPNP_OK && t.dropped) rc = APPNP_ERANGE;
  t.release();
  return rc;
}

// ---- tuning overrides (include/ppnp_amd.h) ------------------------------------------------

const char* appnp_tuning_overrides(void) {
  static const std::string s = [] {
    std::string out;
    if (!appnp::tuning_on()) return out;
    for (const char* name : appnp::kTuningNames) {
      const char* v = getenv(name);
      if (!v || !*v) continue;
      if (!out.empty()) out += ';';
      out += name;
      out += '=';
      out += v;
    }
    return out;
  }();
  return s.c_str();
}

const char* appnp_tuning_names(void) {
  static const std::string s = [] {
    std::string out;
    for (const char* name : appnp::kTuningNames) {
      if (!out.empty()) out += ';';
      out += name;
    }
    return out;
  }();
  return s.c_str();
}

// ---- captured plans: the K launches of appnp_propagate replayed as one hipGraph -----------

struct appnp_plan {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};

int appnp_plan_create(const appnp_graph* g, const void* H, int64_t ld_h, void* Z, int64_t ld_z,
                      int64_t f, int dtype, int K, float alpha, float p_drop, uint64_t seed,
                      void* ws, size_t ws_bytes, appnp_plan** out) {
  if (!out) return APPNP_EINVAL;
  *out = nullptr;
  hipStream_t cs = nullptr;
  if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return APPNP_EDEVICE;
  appnp_plan* p = new (std::nothrow) appnp_plan();
  if (!p) {
    (void)hipStreamDestroy(cs);
    return APPNP_ENOMEM;
  }
  int rc = dev_err(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  if (rc == APPNP_OK) {
    rc = appnp_propagate(g, H, ld_h, Z, ld_z, f, dtype, K, alpha, p_drop, seed, ws, ws_bytes, cs);
    const hipError_t e = hipStreamEndCapture(cs, &p->graph);  // always end the capture
    if (rc == APPNP_OK) rc = dev_err(e);
  }
  if (rc == APPNP_OK) rc = dev_err(hipGraphInstantiate(&p->exec, p->graph, nullptr, nullptr, 0));
  (void)hipStreamDestroy(cs);
  if (rc != APPNP_OK) {
    appnp_plan_destroy(p);
    return rc;
  }
  *out = p;
  return APPNP_OK;
}

int appnp_plan_launch(const appnp_plan* p, void* stream) {
  if (!p || !p->exec) return APPNP_EINVAL;
  return dev_err(hipGraphLaunch(p->exec, as_stream(stream)));
}

void appnp_plan_destroy(appnp_plan* p) {
  if (!p) return;
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  delete p;
}

}  // extern "C"
