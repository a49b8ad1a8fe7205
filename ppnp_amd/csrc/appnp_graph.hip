// appnp_graph.hip -- device-side construction of A_hat (restates helpers.py:58-66 calc_A_hat).
//
//   A' = A + I           diagonal merged in column order (a_ii + 1), zero results dropped,
//                        exactly scipy's `adj + sp.eye(n)` (helpers.py:59)
//   D_i = sum_j A'_ij    fp64, sequential in column order (helpers.py:60, csr_matvec order)
//   sym: A_hat_ij = (dinv_i * A'_ij) * dinv_j,  dinv = 1/sqrt(D)   (helpers.py:61-63)
//   rw:  A_hat_ij = dinv_i * A'_ij,             dinv = 1/D         (helpers.py:64-66)
// Values are formed in fp64 (correctly rounded sqrt/div) and rounded once to fp32, so the
// device CSR equals float32(reference fp64 A_hat) bit for bit.
//
// Pipeline (all on the caller's stream): degree/count pass (thread per row) -> exclusive scan
// of the per-row counts (3 kernels) -> fill pass -> symmetry check.  Setup cost, O(nnz).
#include <algorithm>

#include "appnp_internal.h"
#include "../../include/ppnp_amd.h"

namespace appnp {
namespace {

enum : unsigned { ERR_UNSORTED = 1u, ERR_RANGE = 2u };

struct RowCounts {
  int32_t* all;  // [rows]
  int32_t* loc;  // [rows] (split only)
  int32_t* rem;  // [rows] (split only)
};

// Walk row i of A+I in column order, calling fn(col, merged value) for every nonzero.
template <typename Fn>
__device__ __forceinline__ void walk_merged_row(const int32_t* __restrict__ indptr,
                                                const int32_t* __restrict__ indices,
                                                const float* __restrict__ vals, int64_t i,
                                                int64_t n, unsigned* err, Fn&& fn) {
  const int32_t b = indptr[i], e = indptr[i + 1];
  bool diag_done = false;
  int64_t prev = -1;
  for (int32_t p = b; p < e; ++p) {
    const int64_t j = indices[p];
    if (j <= prev) atomicOr(err, ERR_UNSORTED);
    if (j < 0 || j >= n) {
      atomicOr(err, ERR_RANGE);
      prev = j;
      continue;
    }
    prev = j;
    double a = vals ? (double)vals[p] : 1.0;
    if (!diag_done && j > i) {
      fn((int32_t)i, 1.0);
      diag_done = true;
    }
    if (j == i) {
      a += 1.0;
      diag_done = true;
    }
    if (a != 0.0) fn((int32_t)j, a);
  }
  if (!diag_done) fn((int32_t)i, 1.0);
}

__global__ __launch_bounds__(kBlock) void k_degree(const int32_t* __restrict__ indptr,
                                                   const int32_t* __restrict__ indices,
                                                   const float* __restrict__ vals, int64_t n,
                                                   int mode, double* __restrict__ dinv,
                                                   int64_t row_lo, int64_t row_hi, RowCounts cnt,
                                                   unsigned* err) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  int32_t c_all = 0, c_loc = 0, c_rem = 0;
  bool unit = true;
  walk_merged_row(indptr, indices, vals, i, n, err, [&](int32_t j, double a) {
    s += a;
    unit = unit && a == 1.0;
    ++c_all;
    if (j >= row_lo && j < row_hi) ++c_loc; else ++c_rem;
  });
  dinv[i] = mode == APPNP_NORM_SYM ? 1.0 / sqrt(s) : 1.0 / s;
  if (!unit) atomicOr(err + 2, 1u);  // some entry of A+I is not 1 (flags[2])
  if (i >= row_lo && i < row_hi) {
    const int64_t r = i - row_lo;
    cnt.all[r] = c_all;
    if (cnt.loc) {
      cnt.loc[r] = c_loc;
      cnt.rem[r] = c_rem;
    }
  }
}

struct CsrOut {
  const int32_t* row_ptr;
  int32_t* col;
  float* val;
};

__global__ __launch_bounds__(kBlock) void k_fill(const int32_t* __restrict__ indptr,
                                                 const int32_t* __restrict__ indices,
                                                 const float* __restrict__ vals, int64_t n,
                                                 int mode, const double* __restrict__ dinv,
                                                 int64_t row_lo, int64_t row_hi, CsrOut all,
                                                 CsrOut loc, CsrOut rem, unsigned* err) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= row_hi - row_lo) return;
  const int64_t i = row_lo + r;
  const double di = dinv[i];
  int32_t pa = all.row_ptr[r];
  int32_t pl = loc.col ? loc.row_ptr[r] : 0;
  int32_t pr = rem.col ? rem.row_ptr[r] : 0;
  walk_merged_row(indptr, indices, vals, i, n, err, [&](int32_t j, double a) {
    const double v = mode == APPNP_NORM_SYM ? (di * a) * dinv[j] : di * a;
    const float vf = (float)v;
    all.col[pa] = j;
    all.val[pa] = vf;
    ++pa;
    if (loc.col) {
      if (j >= row_lo && j < row_hi) {
        loc.col[pl] = j;
        loc.val[pl] = vf;
        ++pl;
      } else {
        rem.col[pr] = j;
        rem.val[pr] = vf;
        ++pr;
      }
    }
  });
}

// err |= 4 if some off-diagonal A_ij has no equal A_ji (binary search in row j).
__global__ __launch_bounds__(kBlock) void k_symcheck(const int32_t* __restrict__ indptr,
                                                     const int32_t* __restrict__ indices,
                                                     const float* __restrict__ vals, int64_t n,
                                                     unsigned* asym) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int32_t b = indptr[i], e = indptr[i + 1];
  for (int32_t p = b; p < e; ++p) {
    const int32_t j = indices[p];
    if (j == i || j < 0 || j >= n) continue;
    int32_t lo = indptr[j], hi = indptr[j + 1];
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (indices[mid] < i) lo = mid + 1; else hi = mid;
    }
    const bool found = lo < indptr[j + 1] && indices[lo] == i;
    if (!found || (vals && vals[lo] != vals[p])) {
      atomicOr(asym, 1u);
      return;
    }
  }
}

// ---- exclusive scan of int32 counts into an int32 row_ptr[rows+1] (int64 total) ---------------

constexpr int kScanItems = 8;
constexpr int kScanTile = kBlock * kScanItems;  // 2048 rows per block

__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t* total) {
  __shared__ int64_t wsum[kWavesPerBlock];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int64_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) {
    if (w < wave) base += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const int32_t* __restrict__ cnt,
                                                        int64_t rows, int64_t* __restrict__ bsum) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < rows) s += cnt[base + k];
  int64_t tot;
  block_exclusive_scan(s, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_scan_spine(int64_t* __restrict__ bsum, int64_t nb,
                                                       int64_t* __restrict__ grand) {
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kBlock) {
    const int64_t b = b0 + threadIdx.x;
    const int64_t v = b < nb ? bsum[b] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan(v, &tot);
    if (b < nb) bsum[b] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(kBlock) void k_scan_apply(const int32_t* __restrict__ cnt, int64_t rows,
                                                       const int64_t* __restrict__ bsum,
                                                       const int64_t* __restrict__ grand,
                                                       int32_t* __restrict__ out) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int32_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = base + k < rows ? cnt[base + k] : 0;
    s += v[k];
  }
  int64_t tot;
  int64_t run = bsum[blockIdx.x] + block_exclusive_scan(s, &tot);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < rows) out[base + k] = (int32_t)run;  // range checked on the host
    run += v[k];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[rows] = (int32_t)*grand;
}

}  // namespace

// Scan cnt[rows] into out[rows+1]; the int64 total lands in *d_total (device).
// d_bsum needs scan_partials(rows) int64 entries.
int64_t scan_partials(int64_t rows) {
  return std::max<int64_t>(1, (rows + kScanTile - 1) / kScanTile);
}

hipError_t exclusive_scan(const int32_t* cnt, int64_t rows, int32_t* out, int64_t* d_bsum,
                          int64_t* d_total, hipStream_t s) {
  const int64_t nb = std::max<int64_t>(1, (rows + kScanTile - 1) / kScanTile);
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kBlock), 0, s, cnt, rows, d_bsum);
  hipLaunchKernelGGL(k_scan_spine, dim3(1), dim3(kBlock), 0, s, d_bsum, nb, d_total);
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(kBlock), 0, s, cnt, rows, d_bsum,
                     d_total, out);
  return hipGetLastError();
}

namespace {

template <typename T>
hipError_t dalloc(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) count = 1;
  return hipMalloc(reinterpret_cast<void**>(p), (size_t)count * sizeof(T));
}

}  // namespace

namespace {

__global__ __launch_bounds__(kBlock) void k_heavy_flags(const int32_t* __restrict__ rp, int64_t rows,
                                                        int32_t thr, int32_t* __restrict__ flag) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r < rows) flag[r] = (rp[r + 1] - rp[r]) > thr ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void k_heavy_scatter(const int32_t* __restrict__ flag,
                                                          const int32_t* __restrict__ pos,
                                                          int64_t rows, int32_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r < rows && flag[r]) out[pos[r]] = (int32_t)r;
}

}  // namespace

// Ascending list of the rows with more than `thr` entries (load balance on power-law graphs:
// kHeavyRow for the narrow kernels, kHubRow for hub-first dispatch).  Synchronises (setup).
int build_heavy(const int32_t* rp, int64_t rows, int32_t thr, hipStream_t s, int32_t** out,
                int64_t* n_out) {
  *out = nullptr;
  *n_out = 0;
  if (rows <= 0) return APPNP_OK;
  int32_t *flag = nullptr, *pos = nullptr;
  int64_t *bsum = nullptr, *tot = nullptr;
  int64_t h_tot = 0;
  int rc = APPNP_OK;
  const unsigned grid = (unsigned)((rows + kBlock - 1) / kBlock);
  if (hipMalloc(&flag, rows * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&pos, (rows + 1) * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&bsum, scan_partials(rows) * sizeof(int64_t)) != hipSuccess ||
      hipMalloc(&tot, sizeof(int64_t)) != hipSuccess) {
    rc = APPNP_ENOMEM;
  } else {
    hipLaunchKernelGGL(k_heavy_flags, dim3(grid), dim3(kBlock), 0, s, rp, rows, thr, flag);
    if (exclusive_scan(flag, rows, pos, bsum, tot, s) != hipSuccess ||
        hipMemcpyAsync(&h_tot, tot, sizeof(int64_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = APPNP_EDEVICE;
    } else if (h_tot > 0) {
      if (hipMalloc(out, h_tot * sizeof(int32_t)) != hipSuccess) {
        rc = APPNP_ENOMEM;
      } else {
        hipLaunchKernelGGL(k_heavy_scatter, dim3(grid), dim3(kBlock), 0, s, flag, pos, rows, *out);
        if (hipStreamSynchronize(s) != hipSuccess) rc = APPNP_EDEVICE;
        *n_out = h_tot;
      }
    }
  }
  if (flag) (void)hipFree(flag);
  if (pos) (void)hipFree(pos);
  if (bsum) (void)hipFree(bsum);
  if (tot) (void)hipFree(tot);
  return rc;
}

void graph_free(appnp_graph* g) {
  if (!g) return;
  void* ptrs[] = {g->row_ptr, g->col, g->val, g->lrow_ptr, g->lcol, g->lval,
                  g->rrow_ptr, g->rcol, g->rval, g->dinv, g->t_row_ptr, g->t_col, g->t_val,
                  g->heavy, g->t_heavy, g->hub, g->t_hub, g->rb_off, g->rb_ent, g->rb_val, g->rb_cblk,
                  g->rb_dl, g->rb_dr, g->sh_off};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  g->row_ptr = g->col = g->lrow_ptr = g->lcol = g->rrow_ptr = g->rcol = nullptr;
  g->val = g->lval = g->rval = nullptr;
  g->dinv = nullptr;
  g->t_row_ptr = g->t_col = nullptr;
  g->t_val = nullptr;
  g->heavy = g->t_heavy = g->hub = g->t_hub = nullptr;
  g->rb_off = nullptr;
  g->rb_ent = nullptr;
  g->rb_val = nullptr;
  g->rb_cblk = nullptr;
  g->rb_dl = g->rb_dr = nullptr;
  g->rb_nb = g->rb_passes = 0;
  g->rb_total = 0;
  g->sh_off = nullptr;
  g->sh_n = 0;
  g->sh_rows = 0;
}

// Shard offsets of the held rows (graph_build_shard_offsets): thread per row; its entries are
// sorted by column, so each shard boundary is found by a binary search of the row
__global__ __launch_bounds__(kBlock) void k_shard_offsets(const int32_t* __restrict__ rp,
                                                          const int32_t* __restrict__ col,
                                                          int64_t rows, int nshards,
                                                          int64_t shard_rows,
                                                          int32_t* __restrict__ off) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= rows) return;
  const int32_t beg = rp[i], end = rp[i + 1];
  off[i] = beg;
  off[(int64_t)nshards * rows + i] = end;
  for (int s = 1; s < nshards; ++s) {
    const int64_t bound = (int64_t)s * shard_rows;  // first column of shard s
    int32_t lo = beg, hi = end;                     // first entry with col >= bound
    while (lo < hi) {
      const int32_t mid = lo + (hi - lo) / 2;
      if ((int64_t)col[mid] < bound) lo = mid + 1; else hi = mid;
    }
    off[(int64_t)s * rows + i] = lo;
  }
}

int graph_build_shard_offsets(appnp_graph* g, int nshards, int64_t shard_rows, hipStream_t s) {
  if (!g || nshards < 1 || nshards > 1024 || shard_rows < 1 ||
      (int64_t)nshards * shard_rows < g->n)
    return APPNP_EINVAL;
  const int64_t rows = g->row_hi - g->row_lo;
  if (g->sh_off && g->sh_n == nshards && g->sh_rows == shard_rows) return APPNP_OK;
  int32_t* off = nullptr;
  hipError_t e = hipMalloc(&off, std::max<int64_t>(1, (nshards + 1) * rows) * sizeof(int32_t));
  if (e == hipSuccess && rows > 0) {
    hipLaunchKernelGGL(k_shard_offsets, dim3((unsigned)((rows + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, s, g->row_ptr, g->col, rows, nshards, shard_rows, off);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    if (off) (void)hipFree(off);
    (void)hipGetLastError();
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? APPNP_ENOMEM
                                                                       : APPNP_EDEVICE;
  }
  if (g->sh_off) (void)hipFree(g->sh_off);
  g->sh_off = off;
  g->sh_n = nshards;
  g->sh_rows = shard_rows;
  return APPNP_OK;
}

#define APPNP_TRY(expr)                                                         \
  do {                                                                          \
    hipError_t e_ = (expr);                                                     \
    if (e_ != hipSuccess) {                                                     \
      rc = (e_ == hipErrorOutOfMemory || e_ == hipErrorMemoryAllocation)        \
               ? APPNP_ENOMEM : APPNP_EDEVICE;                                  \
      goto done;                                                                \
    }                                                                           \
  } while (0)

int graph_build(const int32_t* indptr, const int32_t* indices, const float* vals, int64_t n,
                int64_t nnz, int mode, int64_t row_lo, int64_t row_hi, int split, hipStream_t s,
                appnp_graph* g) {
  int rc = APPNP_OK;
  const int64_t rows = row_hi - row_lo;
  int32_t *cnt = nullptr, *cnt_l = nullptr, *cnt_r = nullptr;
  int64_t* bsum = nullptr;
  int64_t* totals = nullptr;  // [3]
  unsigned* flags = nullptr;  // [3]: err, asym, non-unit weights
  int64_t h_tot[3] = {0, 0, 0};
  unsigned h_flags[3] = {0, 0, 0};
  const int64_t nb_scan = std::max<int64_t>(1, (rows + kScanTile - 1) / kScanTile);
  const unsigned blocks_n = (unsigned)std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
  const unsigned blocks_r = (unsigned)std::max<int64_t>(1, (rows + kBlock - 1) / kBlock);
  RowCounts rc_ptrs{};
  CsrOut o_all{}, o_loc{}, o_rem{};

  g->n = n;
  g->row_lo = row_lo;
  g->row_hi = row_hi;
  g->mode = mode;
  g->split = split ? 1 : 0;
  APPNP_TRY(hipGetDevice(&g->device));
  APPNP_TRY(dalloc(&g->dinv, n));
  APPNP_TRY(dalloc(&g->row_ptr, rows + 1));
  APPNP_TRY(dalloc(&cnt, rows));
  if (split) {
    APPNP_TRY(dalloc(&g->lrow_ptr, rows + 1));
    APPNP_TRY(dalloc(&g->rrow_ptr, rows + 1));
    APPNP_TRY(dalloc(&cnt_l, rows));
    APPNP_TRY(dalloc(&cnt_r, rows));
  }
  APPNP_TRY(dalloc(&bsum, nb_scan));
  APPNP_TRY(dalloc(&totals, 3));
  APPNP_TRY(dalloc(&flags, 3));
  APPNP_TRY(hipMemsetAsync(flags, 0, 3 * sizeof(unsigned), s));
  APPNP_TRY(hipMemsetAsync(totals, 0, 3 * sizeof(int64_t), s));

  rc_ptrs = RowCounts{cnt, cnt_l, cnt_r};
  if (n > 0) {
    hipLaunchKernelGGL(k_degree, dim3(blocks_n), dim3(kBlock), 0, s, indptr, indices, vals, n,
                       mode, g->dinv, row_lo, row_hi, rc_ptrs, flags);
    APPNP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_symcheck, dim3(blocks_n), dim3(kBlock), 0, s, indptr, indices, vals, n,
                       flags + 1);
    APPNP_TRY(hipGetLastError());
  }
  APPNP_TRY(exclusive_scan(cnt, rows, g->row_ptr, bsum, totals + 0, s));
  if (split) {
    APPNP_TRY(exclusive_scan(cnt_l, rows, g->lrow_ptr, bsum, totals + 1, s));
    APPNP_TRY(exclusive_scan(cnt_r, rows, g->rrow_ptr, bsum, totals + 2, s));
  }
  APPNP_TRY(hipMemcpyAsync(h_tot, totals, sizeof(h_tot), hipMemcpyDeviceToHost, s));
  APPNP_TRY(hipMemcpyAsync(h_flags, flags, sizeof(h_flags), hipMemcpyDeviceToHost, s));
  APPNP_TRY(hipStreamSynchronize(s));
  if (h_flags[0]) {
    rc = APPNP_EINVAL;  // unsorted / duplicate / out-of-range column indices
    goto done;
  }
  if (h_tot[0] > INT32_MAX) {
    rc = APPNP_ERANGE;
    goto done;
  }
  g->symmetric = h_flags[1] == 0 ? 1 : 0;
  g->unit = h_flags[2] == 0 ? 1 : 0;
  g->nnz_hat = h_tot[0];
  g->nnz_local = h_tot[1];
  g->nnz_remote = h_tot[2];
  APPNP_TRY(dalloc(&g->col, g->nnz_hat));
  APPNP_TRY(dalloc(&g->val, g->nnz_hat));
  if (split) {
    APPNP_TRY(dalloc(&g->lcol, g->nnz_local));
    APPNP_TRY(dalloc(&g->lval, g->nnz_local));
    APPNP_TRY(dalloc(&g->rcol, g->nnz_remote));
    APPNP_TRY(dalloc(&g->rval, g->nnz_remote));
  }
  o_all = CsrOut{g->row_ptr, g->col, g->val};
  if (split) {
    o_loc = CsrOut{g->lrow_ptr, g->lcol, g->lval};
    o_rem = CsrOut{g->rrow_ptr, g->rcol, g->rval};
  }
  if (rows > 0) {
    hipLaunchKernelGGL(k_fill, dim3(blocks_r), dim3(kBlock), 0, s, indptr, indices, vals, n, mode,
                       g->dinv, row_lo, row_hi, o_all, o_loc, o_rem, flags);
    APPNP_TRY(hipGetLastError());
  }
  APPNP_TRY(hipStreamSynchronize(s));
  (void)nnz;
  rc = build_heavy(g->row_ptr, rows, kHeavyRow, s, &g->heavy, &g->n_heavy);
  if (rc == APPNP_OK) rc = build_heavy(g->row_ptr, rows, kHubRow, s, &g->hub, &g->n_hub);

done:
  if (cnt) (void)hipFree(cnt);
  if (cnt_l) (void)hipFree(cnt_l);
  if (cnt_r) (void)hipFree(cnt_r);
  if (bsum) (void)hipFree(bsum);
  if (totals) (void)hipFree(totals);
  if (flags) (void)hipFree(flags);
  if (rc != APPNP_OK) graph_free(g);
  return rc;
}

}  // namespace appnp
