// appnp_ingest.hip -- device-side SparseGraph.standardize (ppnp/data/sparsegraph.py:191-222).
//
// The reference standardizes the adjacency on the host with scipy, in this order:
//   to_unweighted   (sparsegraph.py:135-138)  every stored edge gets weight 1
//   to_undirected   (sparsegraph.py:112-128)  pattern of A + A^T (weights stay 1)
//   remove_self_loops (sparsegraph.py:380-395)
//   largest_connected_components (sparsegraph.py:355-377 -> create_subgraph 300-352): keep
//     the nodes of the largest weakly connected component, relabelled in increasing order.
// Here the same result is produced on the GPU:
//   1. emit (i,j) and (j,i) as 64-bit keys for every stored off-diagonal entry (explicit zero
//      weights count as absent), radix-sort and de-duplicate them (rocPRIM) -> sorted CSR;
//   2. connected components by min-label hooking with pointer jumping (parents only ever
//      decrease, so the forest stays acyclic; iterate until no hook happens);
//   3. the largest component wins; ties go to the component with the largest smallest node
//      index, which is what the reference's np.argsort(sizes)[::-1][:1] picks for a stable
//      sort of scipy's labels (labels are assigned in order of the smallest node);
//   4. kept nodes are renumbered by an exclusive scan (monotone, so rows stay sorted).
#include <algorithm>
#include <new>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>

#include "../../include/ppnp_amd.h"
#include "appnp_internal.h"

struct appnp_csr {
  int64_t n = 0;        // nodes kept
  int64_t nnz = 0;      // stored entries (symmetric, unweighted, no diagonal)
  int64_t n_in = 0;     // nodes of the input graph
  int32_t* indptr = nullptr;
  int32_t* indices = nullptr;
  int64_t* node_map = nullptr;  // [n] input node id of each kept node (ascending)
  float* data = nullptr;        // values (transpose of a weighted CSR only)
};

namespace appnp {
namespace {

constexpr uint64_t kNoKey = ~0ull;

__global__ __launch_bounds__(kBlock) void k_emit_keys(const int32_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ indices,
                                                      const float* __restrict__ vals, int64_t n,
                                                      uint64_t* __restrict__ keys,
                                                      unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int32_t b = indptr[i], e = indptr[i + 1];
  for (int32_t p = b; p < e; ++p) {
    const int64_t j = indices[p];
    uint64_t k0 = kNoKey, k1 = kNoKey;
    if (j < 0 || j >= n) {
      atomicOr(err, 2u);
    } else if (j != i && (!vals || vals[p] != 0.0f)) {
      k0 = ((uint64_t)i << 32) | (uint64_t)j;
      k1 = ((uint64_t)j << 32) | (uint64_t)i;
    }
    keys[2 * (int64_t)p] = k0;
    keys[2 * (int64_t)p + 1] = k1;
  }
}

// rp[r] = first position of row r in the sorted key array (binary search; no atomics)
__global__ __launch_bounds__(kBlock) void k_row_ptr(const uint64_t* __restrict__ keys, int64_t m,
                                                    int64_t n, int32_t* __restrict__ rp) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r > n) return;
  const uint64_t target = (uint64_t)r << 32;
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < target) lo = mid + 1; else hi = mid;
  }
  rp[r] = (int32_t)lo;
}

__global__ __launch_bounds__(kBlock) void k_init_parent(int32_t* __restrict__ parent, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) parent[i] = (int32_t)i;
}

__device__ __forceinline__ int32_t find_root(int32_t* parent, int32_t x) {
  int32_t p = __hip_atomic_load(&parent[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (p != x) {
    const int32_t gp = __hip_atomic_load(&parent[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (gp != p) atomicMin(&parent[x], gp);  // path halving; parents only decrease
    x = p;
    p = gp;
  }
  return x;
}

// One hooking sweep over the edges i<j: the larger root is hooked under the smaller.
__global__ __launch_bounds__(kBlock) void k_hook(const uint64_t* __restrict__ keys, int64_t m,
                                                 int32_t* parent, unsigned* changed) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= m) return;
  const uint64_t k = keys[e];
  const int32_t u = (int32_t)(k >> 32), v = (int32_t)(k & 0xffffffffu);
  if (u >= v) return;  // each undirected edge once
  const int32_t ru = find_root(parent, u), rv = find_root(parent, v);
  if (ru == rv) return;
  const int32_t hi = max(ru, rv), lo = min(ru, rv);
  atomicMin(&parent[hi], lo);
  *changed = 1u;
}

__global__ __launch_bounds__(kBlock) void k_compress_count(int32_t* parent, int64_t n,
                                                           int32_t* __restrict__ size) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int32_t r = find_root(parent, (int32_t)i);
  parent[i] = r;
  atomicAdd(&size[r], 1);
}

// best = max over roots of (size << 32 | root): largest component, ties -> largest root
__global__ __launch_bounds__(kBlock) void k_best(const int32_t* __restrict__ parent,
                                                 const int32_t* __restrict__ size, int64_t n,
                                                 unsigned long long* best) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || parent[i] != (int32_t)i) return;
  atomicMax(best, ((unsigned long long)(uint32_t)size[i] << 32) | (unsigned long long)i);
}

__global__ __launch_bounds__(kBlock) void k_keep(const int32_t* __restrict__ parent, int64_t n,
                                                 const unsigned long long* best, int select,
                                                 int32_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  keep[i] = (!select || parent[i] == (int32_t)(*best & 0xffffffffull)) ? 1 : 0;
}

// kept rows: out row new_id[i] gets the row's columns, renumbered
__global__ __launch_bounds__(kBlock) void k_row_len_kept(const int32_t* __restrict__ rp,
                                                         const int32_t* __restrict__ keep,
                                                         const int32_t* __restrict__ new_id,
                                                         int64_t n, int32_t* __restrict__ len,
                                                         int64_t* __restrict__ node_map) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || !keep[i]) return;
  len[new_id[i]] = rp[i + 1] - rp[i];
  node_map[new_id[i]] = i;
}

__global__ __launch_bounds__(kBlock) void k_fill_kept(const uint64_t* __restrict__ keys,
                                                      const int32_t* __restrict__ rp,
                                                      const int32_t* __restrict__ keep,
                                                      const int32_t* __restrict__ new_id,
                                                      const int32_t* __restrict__ out_ptr,
                                                      int64_t n, int32_t* __restrict__ out_idx) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || !keep[i]) return;
  int32_t o = out_ptr[new_id[i]];
  for (int32_t p = rp[i]; p < rp[i + 1]; ++p)
    out_idx[o++] = new_id[(int32_t)(keys[p] & 0xffffffffu)];
}

struct Buffers {
  uint64_t* keys = nullptr;
  uint64_t* keys_sorted = nullptr;
  void* tmp = nullptr;
  unsigned* flags = nullptr;  // [0] err, [1] changed
  unsigned int* uniq = nullptr;
  int32_t *cnt = nullptr, *rp = nullptr, *parent = nullptr, *size = nullptr;
  int32_t *keep = nullptr, *new_id = nullptr, *len = nullptr;
  int64_t *bsum = nullptr, *tot = nullptr;
  unsigned long long* best = nullptr;
  ~Buffers() {
    void* ps[] = {keys, keys_sorted, tmp, flags, uniq, cnt, rp, parent, size,
                  keep, new_id, len, bsum, tot, best};
    for (void* p : ps)
      if (p) (void)hipFree(p);
  }
};

template <typename T>
hipError_t alloc(T** p, int64_t count) {
  if (count <= 0) count = 1;
  return hipMalloc(reinterpret_cast<void**>(p), (size_t)count * sizeof(T));
}

inline unsigned grid_of(int64_t n) {
  return (unsigned)std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
}

}  // namespace

int standardize(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t n,
                int64_t nnz, int select_lcc, hipStream_t s, appnp_csr* out) {
#define TRY(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      return (e_ == hipErrorOutOfMemory || e_ == hipErrorMemoryAllocation) ? APPNP_ENOMEM   \
                                                                           : APPNP_EDEVICE; \
  } while (0)
  Buffers b;
  const int64_t m = 2 * nnz;
  unsigned h_flags[2] = {0, 0};
  unsigned int h_uniq = 0;
  int64_t h_tot[2] = {0, 0};
  unsigned long long h_best = 0;
  out->n_in = n;
  TRY(alloc(&b.flags, 2));
  TRY(hipMemsetAsync(b.flags, 0, 2 * sizeof(unsigned), s));
  TRY(alloc(&b.keys, m));
  TRY(alloc(&b.keys_sorted, m));
  TRY(alloc(&b.uniq, 1));
  if (n > 0) {
    hipLaunchKernelGGL(k_emit_keys, dim3(grid_of(n)), dim3(kBlock), 0, s, indptr, indices, vals,
                       n, b.keys, b.flags);
    TRY(hipGetLastError());
  }
  // sort + unique (sentinel keys sort last and collapse to one)
  unsigned end_bit = 64;
  {
    size_t tmp_sort = 0, tmp_uniq = 0;
    TRY(rocprim::radix_sort_keys(nullptr, tmp_sort, b.keys, b.keys_sorted, (size_t)m, 0u,
                                 end_bit, s));
    TRY(rocprim::unique(nullptr, tmp_uniq, b.keys_sorted, b.keys, b.uniq, (size_t)m,
                        rocprim::equal_to<uint64_t>(), s));
    TRY(alloc(reinterpret_cast<char**>(&b.tmp), (int64_t)std::max(tmp_sort, tmp_uniq)));
    if (m > 0) {
      size_t t1 = tmp_sort, t2 = tmp_uniq;
      TRY(rocprim::radix_sort_keys(b.tmp, t1, b.keys, b.keys_sorted, (size_t)m, 0u, end_bit, s));
      TRY(rocprim::unique(b.tmp, t2, b.keys_sorted, b.keys, b.uniq, (size_t)m,
                          rocprim::equal_to<uint64_t>(), s));
    } else {
      TRY(hipMemsetAsync(b.uniq, 0, sizeof(unsigned int), s));
    }
  }
  TRY(hipMemcpyAsync(&h_uniq, b.uniq, sizeof(h_uniq), hipMemcpyDeviceToHost, s));
  TRY(hipMemcpyAsync(h_flags, b.flags, sizeof(h_flags), hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  if (h_flags[0]) return APPNP_EINVAL;
  int64_t me = h_uniq;  // unique keys incl. at most one sentinel (sorted last)
  if (me > 0) {
    uint64_t last = 0;
    TRY(hipMemcpy(&last, b.keys + (me - 1), sizeof(last), hipMemcpyDeviceToHost));
    if (last == kNoKey) --me;
  }
  // symmetric CSR of the whole graph
  TRY(alloc(&b.rp, n + 1));
  TRY(alloc(&b.bsum, scan_partials(n)));
  TRY(alloc(&b.tot, 2));
  hipLaunchKernelGGL(k_row_ptr, dim3(grid_of(n + 1)), dim3(kBlock), 0, s, b.keys, me, n, b.rp);
  TRY(hipGetLastError());
  // components
  TRY(alloc(&b.parent, n));
  TRY(alloc(&b.size, n));
  TRY(alloc(&b.best, 1));
  TRY(hipMemsetAsync(b.size, 0, std::max<int64_t>(1, n) * sizeof(int32_t), s));
  TRY(hipMemsetAsync(b.best, 0, sizeof(unsigned long long), s));
  if (n > 0) {
    hipLaunchKernelGGL(k_init_parent, dim3(grid_of(n)), dim3(kBlock), 0, s, b.parent, n);
    TRY(hipGetLastError());
  }
  if (select_lcc && me > 0) {
    for (int it = 0; it < 4096; ++it) {  // a few sweeps in practice; bounded regardless
      unsigned changed = 0;
      TRY(hipMemsetAsync(b.flags + 1, 0, sizeof(unsigned), s));
      hipLaunchKernelGGL(k_hook, dim3(grid_of(me)), dim3(kBlock), 0, s, b.keys, me, b.parent,
                         b.flags + 1);
      TRY(hipGetLastError());
      TRY(hipMemcpyAsync(&changed, b.flags + 1, sizeof(unsigned), hipMemcpyDeviceToHost, s));
      TRY(hipStreamSynchronize(s));
      if (!changed) break;
      if (it == 4095) return APPNP_EDEVICE;  // every sweep hooks >= 1 root: unreachable
    }
  }
  if (n > 0) {
    hipLaunchKernelGGL(k_compress_count, dim3(grid_of(n)), dim3(kBlock), 0, s, b.parent, n,
                       b.size);
    hipLaunchKernelGGL(k_best, dim3(grid_of(n)), dim3(kBlock), 0, s, b.parent, b.size, n, b.best);
    TRY(hipGetLastError());
  }
  // keep + renumber
  TRY(alloc(&b.keep, n));
  TRY(alloc(&b.new_id, n + 1));
  if (n > 0) {
    hipLaunchKernelGGL(k_keep, dim3(grid_of(n)), dim3(kBlock), 0, s, b.parent, n, b.best,
                       select_lcc ? 1 : 0, b.keep);
    TRY(hipGetLastError());
  }
  TRY(exclusive_scan(b.keep, n, b.new_id, b.bsum, b.tot + 1, s));
  TRY(hipMemcpyAsync(&h_tot[1], b.tot + 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TRY(hipMemcpyAsync(&h_best, b.best, sizeof(h_best), hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  const int64_t n_out = h_tot[1];
  out->n = n_out;
  TRY(alloc(&out->node_map, n_out));
  TRY(alloc(&b.len, n_out));
  TRY(alloc(&out->indptr, n_out + 1));
  if (n > 0) {
    hipLaunchKernelGGL(k_row_len_kept, dim3(grid_of(n)), dim3(kBlock), 0, s, b.rp, b.keep,
                       b.new_id, n, b.len, out->node_map);
    TRY(hipGetLastError());
  }
  TRY(exclusive_scan(b.len, n_out, out->indptr, b.bsum, b.tot, s));
  TRY(hipMemcpyAsync(&h_tot[0], b.tot, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  out->nnz = h_tot[0];
  TRY(alloc(&out->indices, out->nnz));
  if (n > 0) {
    hipLaunchKernelGGL(k_fill_kept, dim3(grid_of(n)), dim3(kBlock), 0, s, b.keys, b.rp, b.keep,
                       b.new_id, out->indptr, n, out->indices);
    TRY(hipGetLastError());
  }
  TRY(hipStreamSynchronize(s));
  return APPNP_OK;
#undef TRY
}

namespace {

__global__ __launch_bounds__(kBlock) void k_emit_t(const int32_t* __restrict__ indptr,
                                                   const int32_t* __restrict__ indices,
                                                   int64_t rows, int64_t cols,
                                                   uint64_t* __restrict__ keys, unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= rows) return;
  for (int32_t p = indptr[i]; p < indptr[i + 1]; ++p) {
    const int64_t j = indices[p];
    if (j < 0 || j >= cols) atomicOr(err, 2u);
    keys[p] = ((uint64_t)(uint32_t)j << 32) | (uint64_t)i;
  }
}

__global__ __launch_bounds__(kBlock) void k_low_word(const uint64_t* __restrict__ keys, int64_t m,
                                                     int32_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e < m) out[e] = (int32_t)(keys[e] & 0xffffffffu);
}

}  // namespace

// Stable transpose: sort (col, row) keys, carrying the values; rows of the transpose list the
// input rows in increasing order, so the result is canonical CSR.
int csr_transpose(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t rows,
                  int64_t cols, int64_t nnz, hipStream_t s, appnp_csr* out) {
#define TRY(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      return (e_ == hipErrorOutOfMemory || e_ == hipErrorMemoryAllocation) ? APPNP_ENOMEM   \
                                                                           : APPNP_EDEVICE; \
  } while (0)
  Buffers b;
  unsigned h_err = 0;
  out->n = cols;
  out->n_in = rows;
  out->nnz = nnz;
  TRY(alloc(&b.flags, 2));
  TRY(hipMemsetAsync(b.flags, 0, 2 * sizeof(unsigned), s));
  TRY(alloc(&b.keys, nnz));
  TRY(alloc(&b.keys_sorted, nnz));
  if (rows > 0) {
    hipLaunchKernelGGL(k_emit_t, dim3(grid_of(rows)), dim3(kBlock), 0, s, indptr, indices, rows,
                       cols, b.keys, b.flags);
    TRY(hipGetLastError());
  }
  TRY(alloc(&out->indptr, cols + 1));
  TRY(alloc(&out->indices, nnz));
  if (vals) TRY(alloc(&out->data, nnz));
  if (nnz > 0) {
    size_t tmp = 0;
    if (vals) {
      TRY(rocprim::radix_sort_pairs(nullptr, tmp, b.keys, b.keys_sorted, vals, out->data,
                                    (size_t)nnz, 0u, 64u, s));
    } else {
      TRY(rocprim::radix_sort_keys(nullptr, tmp, b.keys, b.keys_sorted, (size_t)nnz, 0u, 64u, s));
    }
    TRY(alloc(reinterpret_cast<char**>(&b.tmp), (int64_t)tmp));
    if (vals) {
      TRY(rocprim::radix_sort_pairs(b.tmp, tmp, b.keys, b.keys_sorted, vals, out->data,
                                    (size_t)nnz, 0u, 64u, s));
    } else {
      TRY(rocprim::radix_sort_keys(b.tmp, tmp, b.keys, b.keys_sorted, (size_t)nnz, 0u, 64u, s));
    }
    hipLaunchKernelGGL(k_low_word, dim3(grid_of(nnz)), dim3(kBlock), 0, s, b.keys_sorted, nnz,
                       out->indices);
    TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_row_ptr, dim3(grid_of(cols + 1)), dim3(kBlock), 0, s, b.keys_sorted, nnz,
                     cols, out->indptr);
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(&h_err, b.flags, sizeof(h_err), hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  return h_err ? APPNP_EINVAL : APPNP_OK;
#undef TRY
}

// A_hat^T of a built graph, moved into the graph's t_* arrays.
int graph_build_transpose(appnp_graph* g, hipStream_t s) {
  appnp_csr t;
  const int rc = csr_transpose(g->row_ptr, g->col, g->val, g->n, g->n, g->nnz_hat, s, &t);
  if (rc != APPNP_OK) {
    csr_free(&t);
    return rc;
  }
  g->t_row_ptr = t.indptr;
  g->t_col = t.indices;
  g->t_val = t.data;
  if (t.node_map) (void)hipFree(t.node_map);
  int rc2 = build_heavy(g->t_row_ptr, g->n, kHeavyRow, s, &g->t_heavy, &g->t_n_heavy);
  if (rc2 == APPNP_OK) rc2 = build_heavy(g->t_row_ptr, g->n, kHubRow, s, &g->t_hub, &g->t_n_hub);
  return rc2;
}

void csr_free(appnp_csr* c) {
  if (!c) return;
  if (c->indptr) (void)hipFree(c->indptr);
  if (c->indices) (void)hipFree(c->indices);
  if (c->node_map) (void)hipFree(c->node_map);
  if (c->data) (void)hipFree(c->data);
  c->indptr = c->indices = nullptr;
  c->node_map = nullptr;
  c->data = nullptr;
}

}  // namespace appnp

extern "C" {

int appnp_standardize(const int32_t* indptr, const int32_t* indices, const float* vals,
                      int64_t n, int64_t nnz, int select_lcc, void* stream, appnp_csr** out) {
  if (!out) return APPNP_EINVAL;
  *out = nullptr;
  if (n < 0 || nnz < 0) return APPNP_EINVAL;
  if (n > INT32_MAX || 2 * nnz > UINT32_MAX) return APPNP_ERANGE;
  if ((n > 0 && !indptr) || (nnz > 0 && !indices)) return APPNP_EINVAL;
  appnp_csr* c = new (std::nothrow) appnp_csr();
  if (!c) return APPNP_ENOMEM;
  const int rc = appnp::standardize(indptr, indices, vals, n, nnz, select_lcc,
                                    reinterpret_cast<hipStream_t>(stream), c);
  if (rc != APPNP_OK) {
    appnp::csr_free(c);
    delete c;
    return rc;
  }
  *out = c;
  return APPNP_OK;
}

int appnp_csr_info(const appnp_csr* c, int64_t* n, int64_t* nnz, int64_t* n_in) {
  if (!c) return APPNP_EINVAL;
  if (n) *n = c->n;
  if (nnz) *nnz = c->nnz;
  if (n_in) *n_in = c->n_in;
  return APPNP_OK;
}

int appnp_csr_copy(const appnp_csr* c, int32_t* indptr, int32_t* indices, int64_t* node_map,
                   void* stream) {
  if (!c) return APPNP_EINVAL;
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = hipSuccess;
  if (indptr) e = hipMemcpyAsync(indptr, c->indptr, (c->n + 1) * sizeof(int32_t),
                                 hipMemcpyDeviceToDevice, s);
  if (e == hipSuccess && indices && c->nnz)
    e = hipMemcpyAsync(indices, c->indices, c->nnz * sizeof(int32_t), hipMemcpyDeviceToDevice, s);
  if (e == hipSuccess && node_map && c->n)
    e = hipMemcpyAsync(node_map, c->node_map, c->n * sizeof(int64_t), hipMemcpyDeviceToDevice, s);
  return e == hipSuccess ? APPNP_OK : APPNP_EDEVICE;
}

int appnp_csr_transpose(const int32_t* indptr, const int32_t* indices, const float* vals,
                        int64_t rows, int64_t cols, int64_t nnz, void* stream, appnp_csr** out) {
  if (!out) return APPNP_EINVAL;
  *out = nullptr;
  if (rows < 0 || cols < 0 || nnz < 0) return APPNP_EINVAL;
  if (rows > INT32_MAX || cols > INT32_MAX || nnz > INT32_MAX) return APPNP_ERANGE;
  if ((rows > 0 && !indptr) || (nnz > 0 && !indices)) return APPNP_EINVAL;
  appnp_csr* c = new (std::nothrow) appnp_csr();
  if (!c) return APPNP_ENOMEM;
  const int rc = appnp::csr_transpose(indptr, indices, vals, rows, cols, nnz,
                                      reinterpret_cast<hipStream_t>(stream), c);
  if (rc != APPNP_OK) {
    appnp::csr_free(c);
    delete c;
    return rc;
  }
  *out = c;
  return APPNP_OK;
}

int appnp_csr_values(const appnp_csr* c, float* data, void* stream) {
  if (!c || !data) return APPNP_EINVAL;
  if (!c->data || c->nnz == 0) return c->data ? APPNP_OK : APPNP_EINVAL;
  return hipMemcpyAsync(data, c->data, c->nnz * sizeof(float), hipMemcpyDeviceToDevice,
                        reinterpret_cast<hipStream_t>(stream)) == hipSuccess ? APPNP_OK
                                                                             : APPNP_EDEVICE;
}

void appnp_csr_destroy(appnp_csr* c) {
  if (!c) return;
  appnp::csr_free(c);
  delete c;
}

}  // extern "C"
