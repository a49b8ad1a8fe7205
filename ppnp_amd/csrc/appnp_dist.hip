// appnp_dist.hip -- row-partitioned multi-GPU propagation behind the C ABI
// (include/ppnp_amd.h appnp_dist_*; SURVEY.md 8(b) "appnp_dist_create").
//
// Host orchestration only: every iteration is one or two appnp_step launches on the held rows
// (appnp_capi.hip), and the row shards travel through the caller's all-gather callback.  The
// schedule is ppnp_amd/dist.py PartitionedAPPNP.run for a pure row layout:
//
//   Z_0: H's held rows -> buffer 0 at [lo, hi), all-gather (every rank needs all of Z_0)
//   k = 0 .. K-1:  src = buffer k&1 (all P S rows), dst = buffer (k+1)&1 at [lo, hi)
//                  -- or Z itself on the last iteration (no exchange follows it)
//     overlap:     LOCAL  (columns in [lo, hi): own shard, complete)  -> fp32 partial
//                  wait for the exchange of src (internal stream)
//                  REMOTE (the other columns) + partial + alpha H      -> dst
//     otherwise:   ALL                                                -> dst
//     k < K-1:     exchange dst (overlap: on the internal stream, behind an event on `stream`;
//                  waited for inside the next iteration)
//
// The two buffers alternate, and each exchange is waited for before its buffer is written
// again.  So the only concurrent accesses are the exchange of src, which writes the other
// ranks' shards, and the local-column step, which reads this rank's shard.
//
// Split rows (fp32 F = 32q + r, a graph built with a source-blocked copy of the held rows,
// appnp_step_split): each iterate is kept as two full-height parts, main [P S, 32q] (whole
// cache lines per gathered row) and remainder [P S, width of the copy]; both are exchanged
// (two all-gather calls per exchange), the main part runs the SpMM kernel (local / remote with
// overlap) and the remainder part the persistent L2-blocked pass once the exchange has landed.
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <new>
#include <vector>

#include "../../include/ppnp_amd.h"
#include "appnp_internal.h"

struct appnp_dist {
  appnp_graph* g = nullptr;
  int64_t n = 0, lo = 0, hi = 0, shard = 0;
  int rank = 0, nranks = 1, overlap = 0;
  appnp_allgather_fn allgather = nullptr;
  void* ctx = nullptr;
  int sb_requested = 0;                // `mode` asked for the source-blocked copy (all ranks)
  int split_agreed = 0;                // the ranks have agreed on split_ok (first propagation)
  int split_ok = 0;                    // every rank holds its rows' source-blocked copy
  int poisoned = APPNP_OK;             // the split agreement failed on this rank: every later
                                       // call returns this code (the ranks may disagree now)
  hipStream_t xs = nullptr;            // exchange stream (overlap)
  hipEvent_t produced = nullptr;       // dst rows written on the caller's stream
  hipEvent_t exchanged = nullptr;      // exchange finished on xs
  // pipelined exchange (appnp_dist_set_broadcast): one broadcast per row shard on xs, each
  // followed by its event, and the groups of remote shards the product waits for in turn
  appnp_bcast_fn bcast = nullptr;
  void* bctx = nullptr;
  std::vector<hipEvent_t> arrived;     // [nranks]: shard r has landed (on xs)
  std::vector<std::pair<int, int>> groups;
};

namespace {

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int dev_err(hipError_t e) {
  if (e == hipSuccess) return APPNP_OK;
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return APPNP_ENOMEM;
  if (e == hipErrorInvalidValue) return APPNP_EINVAL;
  return APPNP_EDEVICE;
}

constexpr size_t kAlign = 256;

inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct WsLayout {
  int64_t ld = 0;          // elements per row of the iterate buffers
  size_t buf_bytes = 0;    // one full-height iterate
  size_t partial_off = 0;  // fp32 partial (overlap)
  size_t total = 0;
  // split rows: main [P S, fs] and remainder [P S, rw] parts of each iterate
  int64_t fs = 0, rw = 0;
  size_t main_bytes = 0, part_bytes = 0;  // one main part; one iterate (main + remainder)
  // staging of a held-rows H or Z whose base or leading dimension does not allow 16-B vectors:
  // [S, f4] fp32 each (f4 = f rounded up to 4), after the iterates and the partial
  int64_t f4 = 0;
  size_t stage_off = 0, stage_bytes = 0;
  size_t split_total = 0;
};

WsLayout ws_layout(const appnp_dist* d, int64_t f, int dtype) {
  WsLayout w;
  const int64_t es = dtype == APPNP_F32 ? 4 : 2;
  const size_t rows_pad = (size_t)(d->shard * d->nranks);
  w.ld = appnp::line_ld(f, dtype);
  w.buf_bytes = align_up(rows_pad * (size_t)(w.ld * es));
  w.partial_off = 2 * w.buf_bytes;
  const size_t partial = d->overlap ? align_up((size_t)d->shard * (size_t)w.ld * 4) : 0;
  w.total = w.partial_off + partial;
  if (dtype == APPNP_F32 && appnp_split_layout(d->g, f, &w.fs, &w.rw) == APPNP_OK) {
    w.main_bytes = align_up(rows_pad * (size_t)w.fs * 4);
    w.part_bytes = w.main_bytes + align_up(rows_pad * (size_t)w.rw * 4);
    w.f4 = (f + 3) / 4 * 4;
    w.stage_off = 2 * w.part_bytes + (d->overlap ? align_up((size_t)d->shard * w.fs * 4) : 0);
    w.stage_bytes = align_up((size_t)d->shard * (size_t)w.f4 * 4);
    w.split_total = w.stage_off + 2 * w.stage_bytes;
  }
  return w;
}

// The split layout exchanges two parts per iterate, so every rank must take it or none.  The
// rule is the same on every rank (its locality measure is the whole graph's), but the
// regrouped copy is best-effort: at the first fp32 propagation with K >= 2 of an engine whose
// `mode` asked for the copy, the ranks agree through the exchange itself -- each sets one byte
// of its slot of a small in-place all-gather in the workspace, and the copy is used only if
// every rank built it.  Synchronises the stream once.  If the agreement itself fails on this
// rank (exchange or copy error), its peers may have completed it and decided differently, so
// the handle is poisoned: this and every later call returns the error instead of running a
// loop that exchanges a different number of parts than the peers' (ADVICE r3).
int agree_split(appnp_dist* d, void* ws, hipStream_t s) {
  constexpr size_t kSlot = 256;
  d->split_ok = d->g->rb_off != nullptr;
  if (d->nranks <= 1) {
    d->split_agreed = 1;
    return APPNP_OK;
  }
  char* flags = static_cast<char*>(ws);
  std::vector<unsigned char> host((size_t)d->nranks, 0);
  int rc = dev_err(hipMemsetAsync(flags, 0, kSlot * d->nranks, s));
  if (rc == APPNP_OK && d->split_ok)
    rc = dev_err(hipMemsetAsync(flags + kSlot * d->rank, 1, 1, s));
  if (rc == APPNP_OK) rc = d->allgather(flags, kSlot, d->rank, d->nranks, s, d->ctx);
#ifdef APPNP_TESTING
  // APPNP_DIST_TEST_AGREE_FAIL (test library): a failure on this rank after the exchange, so
  // the poisoned handle can be observed
  const char* inj = std::getenv("APPNP_DIST_TEST_AGREE_FAIL");
  if (rc == APPNP_OK && inj && *inj && std::atoi(inj)) rc = APPNP_EDEVICE;
#endif
  for (int p = 0; p < d->nranks && rc == APPNP_OK; ++p)
    rc = dev_err(hipMemcpyAsync(&host[p], flags + kSlot * p, 1, hipMemcpyDeviceToHost, s));
  if (rc == APPNP_OK) rc = dev_err(hipStreamSynchronize(s));
  for (int p = 0; p < d->nranks; ++p)
    if (rc != APPNP_OK || host[p] != 1) d->split_ok = 0;
  if (rc != APPNP_OK) d->poisoned = rc;
  d->split_agreed = 1;
  return rc;
}

// One exchange through the caller's all-gather on stream s, bracketed for the per-launch timer
// (APPNP_KT_XCHG), so the time it takes is never counted in the launch that waits for it
int exchange_on(appnp_dist* d, void* buf, size_t shard_bytes, hipStream_t s) {
  appnp::ktimer_begin(s);
  const int rc = d->allgather(buf, shard_bytes, d->rank, d->nranks, s, d->ctx);
  appnp::ktimer_mark(s, APPNP_KT_XCHG);
  return rc;
}

// The pipelined exchange of one iterate: xs waits for the producer, then broadcasts row shard r
// from rank r, r = 0 .. P-1 in turn (the same order on every rank), each bracketed for the timer
// and followed by its arrival event.
int exchange_shards(appnp_dist* d, char* full, size_t shard_bytes, hipStream_t s) {
  int rc = dev_err(hipEventRecord(d->produced, s));
  if (rc == APPNP_OK) rc = dev_err(hipStreamWaitEvent(d->xs, d->produced, 0));
  for (int r = 0; r < d->nranks && rc == APPNP_OK; ++r) {
    appnp::ktimer_begin(d->xs);
    rc = d->bcast(full + (size_t)r * shard_bytes, shard_bytes, r, d->nranks, d->xs, d->bctx);
    appnp::ktimer_mark(d->xs, APPNP_KT_XCHG);
    if (rc == APPNP_OK) rc = dev_err(hipEventRecord(d->arrived[r], d->xs));
  }
  return rc;
}

// Groups of remote shards in arrival order (ppnp_amd/dist.py shard_groups): sized 1, 2, 4, ...
// from the last to arrive backwards, cut where a group would span the own shard, then adjacent
// groups merged, front first, down to ceil(log2 R) groups.
std::vector<std::pair<int, int>> shard_groups(int R, int ri) {
  std::vector<int> arrival;
  for (int s = 0; s < R; ++s)
    if (s != ri) arrival.push_back(s);
  std::vector<int> sizes;
  for (int left = (int)arrival.size(), sz = 1; left > 0; sz *= 2) {
    const int take = std::min(sz, left);
    sizes.push_back(take);
    left -= take;
  }
  std::vector<std::pair<int, int>> groups;
  size_t pos = 0;
  for (auto it = sizes.rbegin(); it != sizes.rend(); ++it) {
    int start = arrival[pos];
    for (int j = 0; j < *it; ++j) {
      const int a = arrival[pos + j];
      const bool end = j + 1 == *it || arrival[pos + j + 1] != a + 1;
      if (end) {
        groups.emplace_back(start, a + 1);
        if (j + 1 < *it) start = arrival[pos + j + 1];
      }
    }
    pos += *it;
  }
  int cap = 1;
  while ((1 << cap) < R) ++cap;  // ceil(log2 R)
  for (size_t i = 0; groups.size() > (size_t)cap && i + 2 < groups.size();) {  // not the last
    if (groups[i].second == groups[i + 1].first) {
      groups[i].second = groups[i + 1].second;
      groups.erase(groups.begin() + (long)i + 1);
    } else {
      ++i;
    }
  }
  return groups;
}

bool aligned16(const void* p, int64_t ld) {
  return ld % 4 == 0 && (reinterpret_cast<uintptr_t>(p) % 16) == 0;
}

// The loop of appnp_dist_propagate on the split layout (see the file comment).
int propagate_split_rows(appnp_dist* d, const WsLayout& w, const float* H, int64_t ld_h, float* Z,
                         int64_t ld_z, int64_t f, int K, float alpha, float p_drop,
                         uint64_t seed, char* base, hipStream_t s) {
  float* mainb[2] = {reinterpret_cast<float*>(base),
                     reinterpret_cast<float*>(base + w.part_bytes)};
  float* remb[2] = {reinterpret_cast<float*>(base + w.main_bytes),
                    reinterpret_cast<float*>(base + w.part_bytes + w.main_bytes)};
  float* partial = d->overlap ? reinterpret_cast<float*>(base + 2 * w.part_bytes) : nullptr;
  const size_t main_shard = (size_t)d->shard * (size_t)w.fs * 4;
  const size_t rem_shard = (size_t)d->shard * (size_t)w.rw * 4;
  auto exchange = [&](int b, hipStream_t xs) {
    int rc = APPNP_OK;
    if (w.fs > 0) rc = exchange_on(d, mainb[b], main_shard, xs);
    if (rc == APPNP_OK) rc = exchange_on(d, remb[b], rem_shard, xs);
    return rc;
  };
  int rc = appnp_split_copy(d->g, H, ld_h, f, w.fs ? mainb[0] : nullptr, remb[0], s);
  if (rc == APPNP_OK && d->nranks > 1) rc = exchange(0, s);
  bool pending = false;
  for (int k = 0; k < K && rc == APPNP_OK; ++k) {
    const bool last = k == K - 1;
    const int cur = k & 1, nxt = cur ^ 1;
    float* zm_out = last ? nullptr : mainb[nxt];
    float* zr_out = last ? nullptr : remb[nxt];
    float* zout = last ? Z : nullptr;
    if (d->overlap && w.fs > 0) {
      rc = appnp_step_split(d->g, APPNP_PART_LOCAL, mainb[cur], remb[cur], H, ld_h, zm_out, zr_out,
                            zout, ld_z, partial, w.fs, f, k, alpha, p_drop, seed, s);
      if (rc == APPNP_OK && pending) {
        rc = dev_err(hipStreamWaitEvent(s, d->exchanged, 0));
        pending = false;
      }
      if (rc == APPNP_OK)
        rc = appnp_step_split(d->g, APPNP_PART_REMOTE, mainb[cur], remb[cur], H, ld_h, zm_out,
                              zr_out, zout, ld_z, partial, w.fs, f, k, alpha, p_drop, seed, s);
    } else {
      if (pending) {
        rc = dev_err(hipStreamWaitEvent(s, d->exchanged, 0));
        pending = false;
      }
      if (rc == APPNP_OK)
        rc = appnp_step_split(d->g, APPNP_PART_ALL, mainb[cur], remb[cur], H, ld_h, zm_out,
                              zr_out, zout, ld_z, nullptr, 0, f, k, alpha, p_drop, seed, s);
    }
    if (rc != APPNP_OK || last || d->nranks == 1) continue;
    if (d->overlap) {
      rc = dev_err(hipEventRecord(d->produced, s));
      if (rc == APPNP_OK) rc = dev_err(hipStreamWaitEvent(d->xs, d->produced, 0));
      if (rc == APPNP_OK) rc = exchange(nxt, d->xs);
      if (rc == APPNP_OK) rc = dev_err(hipEventRecord(d->exchanged, d->xs));
      pending = rc == APPNP_OK;
    } else {
      rc = exchange(nxt, s);
    }
  }
  if (pending) (void)hipStreamWaitEvent(s, d->exchanged, 0);
  return rc;
}

hipError_t copy_rows(void* dst, int64_t ld_dst, const void* src, int64_t ld_src, int64_t rows,
                     int64_t f, int64_t es, hipStream_t s);

// appnp_dist_propagate on the split layout with the pipelined exchange: the remainder part is
// all-gathered first on xs, the main part by one broadcast per shard; the main product runs FIRST
// on the own shard, ACC per group of arrived shards, LAST on the last group (then the remainder
// pass, after the remainder part's exchange).
int propagate_split_rows_pipelined(appnp_dist* d, const WsLayout& w, const float* H, int64_t ld_h,
                                   float* Z, int64_t ld_z, int64_t f, int K, float alpha,
                                   float p_drop, uint64_t seed, char* base, hipStream_t s) {
  float* mainb[2] = {reinterpret_cast<float*>(base),
                     reinterpret_cast<float*>(base + w.part_bytes)};
  float* remb[2] = {reinterpret_cast<float*>(base + w.main_bytes),
                    reinterpret_cast<float*>(base + w.part_bytes + w.main_bytes)};
  float* partial = reinterpret_cast<float*>(base + 2 * w.part_bytes);
  const size_t main_shard = (size_t)d->shard * (size_t)w.fs * 4;
  const size_t rem_shard = (size_t)d->shard * (size_t)w.rw * 4;
  auto exchange = [&](int b) {
    // the remainder part first (small: it lands before the main shards), then the main part
    int rc = dev_err(hipEventRecord(d->produced, s));
    if (rc == APPNP_OK) rc = dev_err(hipStreamWaitEvent(d->xs, d->produced, 0));
    if (rc == APPNP_OK) rc = exchange_on(d, remb[b], rem_shard, d->xs);
    if (rc == APPNP_OK) rc = dev_err(hipEventRecord(d->exchanged, d->xs));
    if (rc == APPNP_OK) rc = exchange_shards(d, reinterpret_cast<char*>(mainb[b]), main_shard, s);
    return rc;
  };
  const int ri = d->rank;
  int rc = appnp_split_copy(d->g, H, ld_h, f, mainb[0], remb[0], s);
  if (rc == APPNP_OK) rc = exchange(0);
  for (int k = 0; k < K && rc == APPNP_OK; ++k) {
    const bool last = k == K - 1;
    const int cur = k & 1, nxt = cur ^ 1;
    rc = appnp_step_split_shards(d->g, ri, ri + 1, APPNP_SHARDS_FIRST, mainb[cur], nullptr,
                                 nullptr, 0, nullptr, nullptr, nullptr, 0, partial, w.fs, f, k,
                                 alpha, p_drop, seed, s);
    for (size_t i = 0; i < d->groups.size() && rc == APPNP_OK; ++i) {
      const int a = d->groups[i].first, b = d->groups[i].second;
      rc = dev_err(hipStreamWaitEvent(s, d->arrived[b - 1], 0));
      if (rc != APPNP_OK) break;
      if (i + 1 < d->groups.size()) {
        rc = appnp_step_split_shards(d->g, a, b, APPNP_SHARDS_ACC, mainb[cur], nullptr, nullptr,
                                     0, nullptr, nullptr, nullptr, 0, partial, w.fs, f, k, alpha,
                                     p_drop, seed, s);
        continue;
      }
      rc = dev_err(hipStreamWaitEvent(s, d->exchanged, 0));  // the remainder part
      if (rc == APPNP_OK)
        rc = appnp_step_split_shards(d->g, a, b, APPNP_SHARDS_LAST, mainb[cur], remb[cur], H,
                                     ld_h, last ? nullptr : mainb[nxt], last ? nullptr : remb[nxt],
                                     last ? Z : nullptr, ld_z, partial, w.fs, f, k, alpha, p_drop,
                                     seed, s);
    }
    // the own shard's send: the last thing on xs of this exchange (s waits for it before the
    // next exchange reuses the buffer, at no cost: it precedes that exchange on xs anyway)
    if (rc == APPNP_OK) rc = dev_err(hipStreamWaitEvent(s, d->arrived[d->nranks - 1], 0));
    if (rc == APPNP_OK && !last) rc = exchange(nxt);
  }
  return rc;
}

// The same for whole rows (appnp_step_shards), the iterate in [P S, ld] buffers.
int propagate_rows_pipelined(appnp_dist* d, const WsLayout& w, const void* H, int64_t ld_h,
                             void* Z, int64_t ld_z, int64_t f, int K, float alpha, float p_drop,
                             uint64_t seed, char* base, hipStream_t s) {
  char* buf[2] = {base, base + w.buf_bytes};
  float* partial = reinterpret_cast<float*>(base + w.partial_off);
  const size_t row_bytes = (size_t)(w.ld * 4);
  const size_t shard_bytes = (size_t)d->shard * row_bytes;
  const int64_t rows = d->hi - d->lo;
  auto own = [&](char* b) { return b + (size_t)d->lo * row_bytes; };
  const int ri = d->rank;
  int rc = dev_err(copy_rows(own(buf[0]), w.ld, H, ld_h, rows, f, 4, s));
  if (rc == APPNP_OK) rc = exchange_shards(d, buf[0], shard_bytes, s);
  for (int k = 0; k < K && rc == APPNP_OK; ++k) {
    const bool last = k == K - 1;
    const float* src = reinterpret_cast<const float*>(buf[k & 1]);
    float* dst = last ? static_cast<float*>(Z) : reinterpret_cast<float*>(own(buf[(k + 1) & 1]));
    const int64_t ld_dst = last ? ld_z : w.ld;
    rc = appnp_step_shards(d->g, ri, ri + 1, APPNP_SHARDS_FIRST, src, w.ld, nullptr, 0, nullptr,
                           0, partial, w.ld, f, k, alpha, p_drop, seed, s);
    for (size_t i = 0; i < d->groups.size() && rc == APPNP_OK; ++i) {
      const int a = d->groups[i].first, b = d->groups[i].second;
      rc = dev_err(hipStreamWaitEvent(s, d->arrived[b - 1], 0));
      const int mode = i + 1 < d->groups.size() ? APPNP_SHARDS_ACC : APPNP_SHARDS_LAST;
      if (rc == APPNP_OK)
        rc = appnp_step_shards(d->g, a, b, mode, src, w.ld, static_cast<const float*>(H), ld_h,
                               dst, ld_dst, partial, w.ld, f, k, alpha, p_drop, seed, s);
    }
    if (rc == APPNP_OK) rc = dev_err(hipStreamWaitEvent(s, d->arrived[d->nranks - 1], 0));
    if (rc == APPNP_OK && !last) rc = exchange_shards(d, buf[(k + 1) & 1], shard_bytes, s);
  }
  return rc;
}

// rows x (f elements) between two row-major matrices with leading dimensions in elements
hipError_t copy_rows(void* dst, int64_t ld_dst, const void* src, int64_t ld_src, int64_t rows,
                     int64_t f, int64_t es, hipStream_t s) {
  if (rows <= 0 || f <= 0) return hipSuccess;
  return hipMemcpy2DAsync(dst, (size_t)(ld_dst * es), src, (size_t)(ld_src * es),
                          (size_t)(f * es), (size_t)rows, hipMemcpyDeviceToDevice, s);
}

// RCCL, resolved at first use (appnp_allgather_rccl, appnp_bcast_rccl)
typedef int (*nccl_allgather_t)(const void*, void*, size_t, int, void*, hipStream_t);
typedef int (*nccl_bcast_t)(const void*, void*, size_t, int, int, void*, hipStream_t);

void* rccl_handle() {
  static void* h = [] {
    const char* env = std::getenv("APPNP_RCCL_LIB");
    void* x = nullptr;
    if (env && *env) {
      x = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    } else {
      // the copy already in the process (PyTorch's), so its communicators are valid here
      x = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
      if (!x) x = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    }
    return x;
  }();
  return h;
}

nccl_allgather_t rccl_allgather() {
  static nccl_allgather_t fn = rccl_handle() ? reinterpret_cast<nccl_allgather_t>(
                                                   dlsym(rccl_handle(), "ncclAllGather"))
                                             : nullptr;
  return fn;
}

nccl_bcast_t rccl_bcast() {
  static nccl_bcast_t fn =
      rccl_handle() ? reinterpret_cast<nccl_bcast_t>(dlsym(rccl_handle(), "ncclBroadcast"))
                    : nullptr;
  return fn;
}

}  // namespace

extern "C" {

int appnp_dist_create(const int32_t* indptr, const int32_t* indices, const float* vals,
                      int64_t n, int64_t nnz, int mode, int rank, int nranks, int overlap,
                      appnp_allgather_fn allgather, void* ctx, void* stream, appnp_dist** out) {
  if (!out) return APPNP_EINVAL;
  *out = nullptr;
  if (n <= 0 || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !allgather))
    return APPNP_EINVAL;
  appnp_dist* d = new (std::nothrow) appnp_dist();
  if (!d) return APPNP_ENOMEM;
  d->n = n;
  d->rank = rank;
  d->nranks = nranks;
  d->overlap = (overlap && nranks > 1) ? 1 : 0;
  d->allgather = allgather;
  d->ctx = ctx;
  d->shard = (n + nranks - 1) / nranks;
  d->lo = std::min<int64_t>(n, (int64_t)rank * d->shard);
  d->hi = std::min<int64_t>(n, d->lo + d->shard);
  int rc = appnp_graph_create_rows(indptr, indices, vals, n, nnz, mode, d->lo, d->hi,
                                   d->overlap, stream, &d->g);
  d->sb_requested = (mode & (APPNP_GRAPH_SOURCE_BLOCKS | APPNP_GRAPH_SB_W8 |
                             APPNP_GRAPH_SB_W16)) != 0;
  if (rc == APPNP_OK && d->overlap) {
    rc = dev_err(hipStreamCreateWithFlags(&d->xs, hipStreamNonBlocking));
    if (rc == APPNP_OK) rc = dev_err(hipEventCreateWithFlags(&d->produced, hipEventDisableTiming));
    if (rc == APPNP_OK)
      rc = dev_err(hipEventCreateWithFlags(&d->exchanged, hipEventDisableTiming));
  }
  if (rc != APPNP_OK) {
    appnp_dist_destroy(d);
    return rc;
  }
  *out = d;
  return APPNP_OK;
}

int appnp_dist_rows(const appnp_dist* d, int64_t* row_lo, int64_t* row_hi, int64_t* shard) {
  if (!d) return APPNP_EINVAL;
  if (row_lo) *row_lo = d->lo;
  if (row_hi) *row_hi = d->hi;
  if (shard) *shard = d->shard;
  return APPNP_OK;
}

const appnp_graph* appnp_dist_graph(const appnp_dist* d) { return d ? d->g : nullptr; }

size_t appnp_dist_workspace_bytes(const appnp_dist* d, int64_t f, int dtype) {
  if (!d || f <= 0 || (dtype != APPNP_F32 && dtype != APPNP_BF16)) return 0;
  const WsLayout w = ws_layout(d, f, dtype);
  return std::max(w.total, w.split_total);
}

int appnp_dist_propagate(appnp_dist* d, const void* H, int64_t ld_h, void* Z, int64_t ld_z,
                         int64_t f, int dtype, int K, float alpha, float p_drop, uint64_t seed,
                         void* ws, size_t ws_bytes, void* stream) {
  if (!d || f < 0 || K < 0 || (dtype != APPNP_F32 && dtype != APPNP_BF16)) return APPNP_EINVAL;
  if (d->overlap && dtype != APPNP_F32) return APPNP_ENOTSUP;
  if (!(alpha >= 0.0f && alpha <= 1.0f) || !(p_drop >= 0.0f && p_drop < 1.0f))
    return APPNP_EINVAL;
  if (d->poisoned != APPNP_OK) return d->poisoned;
  const int64_t rows = d->hi - d->lo;
  if (f == 0) return APPNP_OK;
  if (rows > 0 && (!H || !Z || ld_h < f || ld_z < f)) return APPNP_EINVAL;
  const int64_t es = dtype == APPNP_F32 ? 4 : 2;
  hipStream_t s = as_stream(stream);
  if (K == 0) return dev_err(copy_rows(Z, ld_z, H, ld_h, rows, f, es, s));
  const WsLayout w = ws_layout(d, f, dtype);
  if (d->sb_requested && !d->split_agreed && dtype == APPNP_F32 && K >= 2) {
    if (!ws || ws_bytes < w.total || ws_bytes < 256 * (size_t)d->nranks) return APPNP_EINVAL;
    const int arc = agree_split(d, ws, s);
    if (arc != APPNP_OK) return arc;
  }
  // split rows whenever every rank's copy allows it (K >= 2: one iteration gains nothing from
  // the split layout).  The decision depends only on what the ranks agreed on, so every rank
  // exchanges the same parts: an H or Z whose base pointer or leading dimension does not allow
  // 16-B vectors is this rank's alone, and it is staged through the workspace ([S, f4] fp32,
  // copied in before the loop and out after it) rather than changing this rank's path (ADVICE
  // r4: round 4 returned APPNP_EINVAL there while the peers waited in the split loop's exchange)
  if (d->split_ok && w.split_total && K >= 2) {
    if (!ws || ws_bytes < w.split_total) return APPNP_EINVAL;
    char* base = static_cast<char*>(ws);
    const float* h = static_cast<const float*>(H);
    float* z = static_cast<float*>(Z);
    int64_t lh = ld_h, lz = ld_z;
    const bool stage_h = rows > 0 && !aligned16(H, ld_h);
    const bool stage_z = rows > 0 && !aligned16(Z, ld_z);
    float* hs = reinterpret_cast<float*>(base + w.stage_off);
    float* zs = reinterpret_cast<float*>(base + w.stage_off + w.stage_bytes);
    int rc = APPNP_OK;
    if (stage_h) {
      rc = dev_err(copy_rows(hs, w.f4, H, ld_h, rows, f, 4, s));
      h = hs;
      lh = w.f4;
    }
    if (stage_z) {
      z = zs;
      lz = w.f4;
    }
    if (rc == APPNP_OK)
      rc = (d->bcast && w.fs > 0)
               ? propagate_split_rows_pipelined(d, w, h, lh, z, lz, f, K, alpha, p_drop, seed,
                                                base, s)
               : propagate_split_rows(d, w, h, lh, z, lz, f, K, alpha, p_drop, seed, base, s);
    if (rc == APPNP_OK && stage_z) rc = dev_err(copy_rows(Z, ld_z, zs, w.f4, rows, f, 4, s));
    return rc;
  }
  if (!ws || ws_bytes < w.total) return APPNP_EINVAL;
  char* base = static_cast<char*>(ws);
  if (d->bcast && dtype == APPNP_F32)
    return propagate_rows_pipelined(d, w, H, ld_h, Z, ld_z, f, K, alpha, p_drop, seed, base, s);
  char* buf[2] = {base, base + w.buf_bytes};
  float* partial = d->overlap ? reinterpret_cast<float*>(base + w.partial_off) : nullptr;
  const size_t row_bytes = (size_t)(w.ld * es);
  const size_t shard_bytes = (size_t)d->shard * row_bytes;
  auto own = [&](char* b) { return b + (size_t)d->lo * row_bytes; };

  // Z_0: the held rows of H, then the whole of it by exchange (synchronous in stream order)
  int rc = dev_err(copy_rows(own(buf[0]), w.ld, H, ld_h, rows, f, es, s));
  if (rc == APPNP_OK && d->nranks > 1)
    rc = exchange_on(d, buf[0], shard_bytes, s);
  bool pending = false;  // an exchange on xs not yet waited for by `s`
  for (int k = 0; k < K && rc == APPNP_OK; ++k) {
    const bool last = k == K - 1;
    char* src = buf[k & 1];
    void* dst = last ? Z : static_cast<void*>(own(buf[(k + 1) & 1]));
    const int64_t ld_dst = last ? ld_z : w.ld;
    if (d->overlap) {
      rc = appnp_step(d->g, APPNP_PART_LOCAL, src, w.ld, nullptr, 0, partial, w.ld, nullptr, 0,
                      f, dtype, k, alpha, p_drop, seed, s);
      if (rc == APPNP_OK && pending) {
        rc = dev_err(hipStreamWaitEvent(s, d->exchanged, 0));
        pending = false;
      }
      if (rc == APPNP_OK)
        rc = appnp_step(d->g, APPNP_PART_REMOTE, src, w.ld, H, ld_h, dst, ld_dst, partial, w.ld,
                        f, dtype, k, alpha, p_drop, seed, s);
    } else {
      rc = appnp_step(d->g, APPNP_PART_ALL, src, w.ld, H, ld_h, dst, ld_dst, nullptr, 0, f,
                      dtype, k, alpha, p_drop, seed, s);
    }
    if (rc != APPNP_OK || last || d->nranks == 1) continue;
    char* next = buf[(k + 1) & 1];
    if (d->overlap) {
      rc = dev_err(hipEventRecord(d->produced, s));
      if (rc == APPNP_OK) rc = dev_err(hipStreamWaitEvent(d->xs, d->produced, 0));
      if (rc == APPNP_OK) rc = exchange_on(d, next, shard_bytes, d->xs);
      if (rc == APPNP_OK) rc = dev_err(hipEventRecord(d->exchanged, d->xs));
      pending = rc == APPNP_OK;
    } else {
      rc = exchange_on(d, next, shard_bytes, s);
    }
  }
  if (pending) (void)hipStreamWaitEvent(s, d->exchanged, 0);  // never leave xs running ahead
  return rc;
}

int appnp_dist_set_broadcast(appnp_dist* d, appnp_bcast_fn fn, void* ctx, void* stream) {
  if (!d || !fn) return APPNP_EINVAL;
  if (!d->overlap || d->nranks < 3) return APPNP_ENOTSUP;  // nothing to pipeline
  if (d->poisoned != APPNP_OK) return d->poisoned;
  int rc = appnp_graph_shard_offsets(d->g, d->nranks, d->shard, stream);
  std::vector<hipEvent_t> ev((size_t)d->nranks, nullptr);
  for (size_t r = 0; r < ev.size() && rc == APPNP_OK; ++r)
    rc = dev_err(hipEventCreateWithFlags(&ev[r], hipEventDisableTiming));
  if (rc != APPNP_OK) {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    return rc;
  }
  for (hipEvent_t e : d->arrived) (void)hipEventDestroy(e);
  d->arrived = ev;
  d->groups = shard_groups(d->nranks, d->rank);
  d->bcast = fn;
  d->bctx = ctx;
  return APPNP_OK;
}

int appnp_dist_pipeline_groups(const appnp_dist* d, int* lo, int* hi, int max, int* n_out) {
  if (!d || !n_out) return APPNP_EINVAL;
  *n_out = d->bcast ? (int)d->groups.size() : 0;
  for (int i = 0; i < *n_out && i < max; ++i) {
    if (lo) lo[i] = d->groups[i].first;
    if (hi) hi[i] = d->groups[i].second;
  }
  return APPNP_OK;
}

void appnp_dist_destroy(appnp_dist* d) {
  if (!d) return;
  if (d->xs) (void)hipStreamSynchronize(d->xs);
  for (hipEvent_t e : d->arrived) (void)hipEventDestroy(e);
  if (d->produced) (void)hipEventDestroy(d->produced);
  if (d->exchanged) (void)hipEventDestroy(d->exchanged);
  if (d->xs) (void)hipStreamDestroy(d->xs);
  appnp_graph_destroy(d->g);
  delete d;
}

int appnp_bcast_rccl(void* buf, size_t bytes, int root, int nranks, void* stream, void* ctx) {
  if (!buf || !ctx || root < 0 || root >= nranks) return APPNP_EINVAL;
  const nccl_bcast_t fn = rccl_bcast();
  if (!fn) return APPNP_ENOTSUP;
  // ncclChar = 0; in place (sendbuff == recvbuff); ncclSuccess = 0
  return fn(buf, buf, bytes, 0, root, ctx, as_stream(stream)) == 0 ? APPNP_OK : APPNP_EDEVICE;
}

int appnp_allgather_rccl(void* buf, size_t shard_bytes, int rank, int nranks, void* stream,
                         void* ctx) {
  if (!buf || !ctx || rank < 0 || rank >= nranks) return APPNP_EINVAL;
  const nccl_allgather_t fn = rccl_allgather();
  if (!fn) return APPNP_ENOTSUP;
  char* b = static_cast<char*>(buf);
  // ncclChar = 0; ncclSuccess = 0
  return fn(b + (size_t)rank * shard_bytes, b, shard_bytes, 0, ctx, as_stream(stream)) == 0
             ? APPNP_OK
             : APPNP_EDEVICE;
}

}  // extern "C"
