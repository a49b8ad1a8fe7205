// appnp_blocks.hip -- remainder columns of a row through an L2-resident pass (gfx950).
//
// Why.  The SpMM is bound by random 128-B line requests: every nonzero
// gathers one row of Z.  An fp32 row of F = 32q + r features (1 <= r <= 4: F = 100 is
// 96 + 4) spans q + 1 lines, and the last one carries only r * 4 <= 16 useful bytes -- a
// quarter of products-synth's line requests.  Those r columns are taken out of the gather:
//
//   * Z between iterations is kept "split": Z_main [n, 32q] (rows of whole lines, so a
//     gather is exactly q lines) and Z_rem [n, 4] (16 B per row).
//   * The remainder product  R = (M_k o A_hat) Z_rem  runs as a pass over A_hat blocked by
//     SOURCE rows: block b holds the entries whose column lies in [b*2^17, (b+1)*2^17), i.e.
//     2 MB of Z_rem, which stays resident in every XCD's 4 MB L2 while the block's launch
//     gathers from it.  One launch per block accumulates into R in block order (fixed order:
//     bitwise deterministic).
//   * The main kernel gathers the q lines of Z_main per nonzero and takes R as the
//     remainder lanes' pre-summed accumulator (appnp_spmm.hip wave_row, StepArgs::rem_in).
//
// The blocked copy of A_hat (APPNP_GRAPH_SOURCE_BLOCKS) is built at graph creation:
// sb_ptr[b * rows + i] is the first entry of row i in block b (block-major, row-minor, so the
// entries of one block are contiguous and one launch streams them once).
#include <algorithm>
#include <cstdlib>

#include "appnp_internal.h"
#include "../../include/ppnp_amd.h"

namespace appnp {
namespace {

// entries of each (block, row): the row's columns are sorted, so a block is a contiguous run.
// Also counts the off-diagonal entries within kNearRows of their row (*near: gather locality).
__global__ __launch_bounds__(kBlock) void k_sb_count(const int32_t* __restrict__ rp,
                                                     const int32_t* __restrict__ col, int64_t rows,
                                                     int64_t row_lo, int brows,
                                                     int32_t* __restrict__ cnt,
                                                     unsigned long long* __restrict__ near) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  unsigned long long nr = 0;
  if (i < rows) {
    int cur = -1, c = 0;
    for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
      const int32_t j = col[e];
      const int64_t d = (int64_t)j - (row_lo + i);
      nr += (d != 0 && d < kNearRows && d > -kNearRows) ? 1 : 0;  // the diagonal is no gather
      const int b = j / brows;
      if (b != cur) {
        if (cur >= 0) cnt[(int64_t)cur * rows + i] = c;
        cur = b;
        c = 0;
      }
      ++c;
    }
    if (cur >= 0) cnt[(int64_t)cur * rows + i] = c;
  }
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) nr += __shfl_xor(nr, off);
  if ((threadIdx.x & (kWave - 1)) == 0 && nr) atomicAdd(near, nr);
}

__global__ __launch_bounds__(kBlock) void k_sb_fill(const int32_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const float* __restrict__ val, int64_t rows,
                                                    int brows, const int32_t* __restrict__ ptr,
                                                    int32_t* __restrict__ bcol,
                                                    float* __restrict__ bval) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= rows) return;
  int cur = -1;
  int32_t pos = 0;
  for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
    const int32_t c = col[e];
    const int b = c / brows;
    if (b != cur) {
      cur = b;
      pos = ptr[(int64_t)b * rows + i];
    }
    bcol[pos] = c;
    bval[pos] = val[e];
    ++pos;
  }
}

// R[i] (+)= sum over the entries of row i in source block b of w_ij * Z_rem[j]; thread per
// row (a block holds ~nnz/(rows * n_sb) entries of a row: 2.7 on products-synth), U entries
// loaded and gathered at a time so that a wave's longest row takes few dependent rounds.
// One launch per block, so all resident waves gather from the same 2 MB of Z_rem; per row the
// sum runs over blocks in order and entries in column order (fixed: bitwise deterministic).
// a.zin = Z_rem (n x 4 fp32), a.aux = R (rows x 4 fp32 accumulator).  FIRST: R starts at 0.
// LAST: the iteration's epilogue, out[i, :nv] = (1-alpha) R[i] + alpha H_rem[i] (a.h = H_rem,
// a.out / a.ld_out, a.f = nv valid columns: 4 into the next Z_rem, 1-4 into Z's last columns).
// (A single launch keeping every row's sum in registers while all threads walk the blocks
// measured slower: threads drift apart and the blocks they gather from no longer fit L2.)
template <int EPI, bool FIRST, bool LAST>
__device__ __forceinline__ void rem_finish(const StepArgs& a, int64_t i, f32x4 acc) {
  if constexpr (!LAST) {
    static_cast<f32x4*>(a.aux)[i] = acc;
  } else if constexpr (EPI == EPI_BWD) {
    // adjoint: G_k = (1-alpha) R into the next remainder buffer (none at k = 0), and
    // dH[:, fs:f] += alpha' G_k (exactly nv columns)
    const float y[4] = {a.scale * acc.x, a.scale * acc.y, a.scale * acc.z, a.scale * acc.w};
    if (a.out)
      static_cast<f32x4*>(a.out)[i] = f32x4{y[0], y[1], y[2], y[3]};
    const int nv = a.f;
    float* d = a.rem_dh + i * a.ld_rem_dh;
    if (nv == 4) {
      f32x4 v = *reinterpret_cast<f32x4*>(d);
      v = f32x4{fmaf(a.alpha, y[0], v.x), fmaf(a.alpha, y[1], v.y), fmaf(a.alpha, y[2], v.z),
                fmaf(a.alpha, y[3], v.w)};
      *reinterpret_cast<f32x4*>(d) = v;
    } else {
      for (int v = 0; v < nv; ++v) d[v] = fmaf(a.alpha, y[v], d[v]);
    }
  } else {
    // H rows are 16-B aligned with ld_h >= roundup(f, 4): the 16 B at H_rem stay inside the
    // row's storage, except possibly on the buffer's last row (read exactly nv there)
    const int nv = a.f;
    const float* hp = static_cast<const float*>(a.h) + i * a.ld_h;
    f32x4 h = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (nv == 4 || i + 1 < a.n_rows) {
      h = *reinterpret_cast<const f32x4*>(hp);
    } else {
      h.x = hp[0];
      if (nv > 1) h.y = hp[1];
      if (nv > 2) h.z = hp[2];
    }
    const float y[4] = {fmaf(a.alpha, h.x, a.scale * acc.x),
                        fmaf(a.alpha, nv > 1 ? h.y : 0.0f, a.scale * acc.y),
                        fmaf(a.alpha, nv > 2 ? h.z : 0.0f, a.scale * acc.z),
                        fmaf(a.alpha, nv > 3 ? h.w : 0.0f, a.scale * acc.w)};
    float* o = static_cast<float*>(a.out) + i * a.ld_out;
    if (nv == 4) {
      *reinterpret_cast<f32x4*>(o) = f32x4{y[0], y[1], y[2], y[3]};
    } else {
      for (int v = 0; v < nv; ++v) o[v] = y[v];
    }
  }
}

// Blocks [0, light_blocks): thread per row.  Trailing blocks: hub rows (> kHubRow entries in
// all, listed in a.hub; the light threads skip them), a wavefront each -- its lanes stride
// over the row's entries of the block and a fixed butterfly adds them -- so a power-law hub
// does not serialise one thread while the launch waits.
template <int U, int EPI, bool FIRST, bool LAST>
__global__ __launch_bounds__(kBlock) void k_rem_block(StepArgs a, const int32_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ bcol,
                                                      const float* __restrict__ bval) {
  const f32x4* __restrict__ z = static_cast<const f32x4*>(a.zin);
  const f32x4* __restrict__ r = static_cast<const f32x4*>(a.aux);
  if ((int64_t)blockIdx.x >= a.light_blocks) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = ((int64_t)gridDim.x - a.light_blocks) * kWavesPerBlock;
    for (int64_t hw = ((int64_t)blockIdx.x - a.light_blocks) * kWavesPerBlock +
                      (threadIdx.x >> 6);
         hw < a.n_hub; hw += nw) {
      const int64_t i = a.hub[hw];
      f32x4 acc = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      const int32_t end = ptr[i + 1];
      for (int32_t e = ptr[i] + lane; e < end; e += kWave) {
        const int32_t c = ld_nt<int32_t>(bcol + e);
        const float w = edge_weight(ld_nt<float>(bval + e), a.row_lo + i, c, a);
        const f32x4 v = z[c];
        acc.x = fmaf(w, v.x, acc.x);
        acc.y = fmaf(w, v.y, acc.y);
        acc.z = fmaf(w, v.z, acc.z);
        acc.w = fmaf(w, v.w, acc.w);
      }
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        acc.x += __shfl_xor(acc.x, off);
        acc.y += __shfl_xor(acc.y, off);
        acc.z += __shfl_xor(acc.z, off);
        acc.w += __shfl_xor(acc.w, off);
      }
      if (lane == 0) {
        if constexpr (!FIRST) {
          const f32x4 p = r[i];
          acc = f32x4{p.x + acc.x, p.y + acc.y, p.z + acc.z, p.w + acc.w};
        }
        rem_finish<EPI, FIRST, LAST>(a, i, acc);
      }
    }
    return;
  }
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n_rows) return;
  if (a.n_hub && a.row_ptr[i + 1] - a.row_ptr[i] > kHubRow) return;  // hub: trailing blocks
  f32x4 acc = FIRST ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : r[i];
  const int32_t end = ptr[i + 1];
  for (int32_t e = ptr[i]; e < end; e += U) {
    int32_t c[U];
    float w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = 0;
      w[u] = 0.0f;
      if (e + u < end) {  // cached: neighbouring lanes' runs share lines (non-temporal: -1 %)
        c[u] = bcol[e + u];
        w[u] = bval[e + u];
      }
    }
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = e + u < end ? z[c[u]] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wu = e + u < end ? edge_weight(w[u], a.row_lo + i, c[u], a) : 0.0f;
      acc.x = fmaf(wu, v[u].x, acc.x);
      acc.y = fmaf(wu, v[u].y, acc.y);
      acc.z = fmaf(wu, v[u].z, acc.z);
      acc.w = fmaf(wu, v[u].w, acc.w);
    }
  }
  rem_finish<EPI, FIRST, LAST>(a, i, acc);
}

// H [n, ld_h] -> the split layout: main [n, fs] (whole lines per row) and rem [n, 4]
// (columns fs..f-1, zero padded).  Thread per 16-B piece of a row (fs / 4 + 1 pieces).
__global__ __launch_bounds__(kBlock) void k_split_copy(const float* __restrict__ h, int64_t ld_h,
                                                       int64_t n, int f, int fs,
                                                       float* __restrict__ main,
                                                       float* __restrict__ rem) {
  const int pieces = fs / 4 + 1;
  const int64_t total = n * pieces;
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kBlock) {
    const int64_t row = t / pieces;
    const int q = (int)(t - row * pieces);
    const float* p = h + row * ld_h + 4 * q;
    if (q < fs / 4) {
      *reinterpret_cast<f32x4*>(main + row * fs + 4 * q) = ld_nt<f32x4>(p);
    } else {
      // the remainder piece: a full 16-B read stays inside the row's storage except possibly
      // on the buffer's last row, which reads exactly its nv valid columns
      const int nv = f - fs;
      f32x4 v = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (nv == 4 || row + 1 < n) {
        v = ld_nt<f32x4>(p);
        if (nv < 4) v.w = 0.0f;
        if (nv < 3) v.z = 0.0f;
        if (nv < 2) v.y = 0.0f;
      } else {
        v.x = p[0];
        if (nv > 1) v.y = p[1];
        if (nv > 2) v.z = p[2];
      }
      *reinterpret_cast<f32x4*>(rem + row * 4) = v;
    }
  }
}

}  // namespace

int graph_build_source_blocks(appnp_graph* g, hipStream_t s) {
  const int64_t rows = g->row_hi - g->row_lo;
  static const int brows = [] {
    const char* v = getenv("APPNP_SB_ROWS");  // measurement override of kSourceBlockRows
    const int x = (v && *v) ? atoi(v) : kSourceBlockRows;
    return x >= 1024 ? x : kSourceBlockRows;
  }();
  const int64_t nb = std::max<int64_t>(1, (g->n + brows - 1) / brows);
  const int64_t cells = nb * rows;
  if (cells + 1 > INT32_MAX) return APPNP_ERANGE;
  int rc = APPNP_OK;
  int32_t* cnt = nullptr;
  int64_t *bsum = nullptr, *tot = nullptr;
  const unsigned grid = (unsigned)std::max<int64_t>(1, (rows + kBlock - 1) / kBlock);
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && rc == APPNP_OK)
      rc = (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? APPNP_ENOMEM
                                                                       : APPNP_EDEVICE;
    return rc == APPNP_OK;
  };
  if (ok(hipMalloc(&g->sb_ptr, (cells + 1) * sizeof(int32_t))) &&
      ok(hipMalloc(&g->sb_col, std::max<int64_t>(1, g->nnz_hat) * sizeof(int32_t))) &&
      ok(hipMalloc(&g->sb_val, std::max<int64_t>(1, g->nnz_hat) * sizeof(float))) &&
      ok(hipMalloc(&cnt, std::max<int64_t>(1, cells) * sizeof(int32_t))) &&
      ok(hipMalloc(&bsum, scan_partials(cells) * sizeof(int64_t))) &&
      ok(hipMalloc(&tot, 2 * sizeof(int64_t))) &&
      ok(hipMemsetAsync(tot, 0, 2 * sizeof(int64_t), s)) &&
      ok(hipMemsetAsync(cnt, 0, std::max<int64_t>(1, cells) * sizeof(int32_t), s))) {
    if (rows > 0) {
      hipLaunchKernelGGL(k_sb_count, dim3(grid), dim3(kBlock), 0, s, g->row_ptr, g->col, rows,
                         g->row_lo, brows, cnt, reinterpret_cast<unsigned long long*>(tot + 1));
      ok(hipGetLastError());
    }
    if (rc == APPNP_OK && ok(exclusive_scan(cnt, cells, g->sb_ptr, bsum, tot, s)) && rows > 0) {
      hipLaunchKernelGGL(k_sb_fill, dim3(grid), dim3(kBlock), 0, s, g->row_ptr, g->col, g->val,
                         rows, brows, g->sb_ptr, g->sb_col, g->sb_val);
      ok(hipGetLastError());
    }
    int64_t near = 0;
    if (rc == APPNP_OK)
      ok(hipMemcpyAsync(&near, tot + 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    if (rc == APPNP_OK && ok(hipStreamSynchronize(s)))
      g->near_frac = g->nnz_hat > 0 ? (double)near / (double)g->nnz_hat : 0.0;
  }
  if (cnt) (void)hipFree(cnt);
  if (bsum) (void)hipFree(bsum);
  if (tot) (void)hipFree(tot);
  if (rc != APPNP_OK) {
    if (g->sb_ptr) (void)hipFree(g->sb_ptr);
    if (g->sb_col) (void)hipFree(g->sb_col);
    if (g->sb_val) (void)hipFree(g->sb_val);
    g->sb_ptr = g->sb_col = nullptr;
    g->sb_val = nullptr;
    return rc;
  }
  g->n_sb = (int32_t)nb;
  return APPNP_OK;
}

// One iteration of the remainder columns: R = (M_k o A_hat) Z_rem over all source blocks, one
// launch per block in block order, the last one applying the epilogue (k_rem_block).
// a: the iteration's StepArgs (dropout key, row_lo, n_rows, scale, alpha); z_rem [n, 4];
// acc [rows, 4] scratch (may be `out` itself when out is a Z_rem buffer); h_rem = H + fs;
// out / ld_out / nv: where the nv valid columns of Z_{k+1} go.  epi = EPI_BWD (adjoint): h_rem
// / ld_h are dH's remainder columns, accumulated into; out (G_k's remainder) may be null.
// Entries in flight per thread: 16 (products-synth per iteration: 1 -> 1.6 ms, 8 -> 1.4 ms,
// 16 0.05 ms less; tools/sweep_split.sh).  Blocks of 2^17 source rows measured best
// (2^16, 96k, 160k, 192k and 2^18 rows: +0.01-0.3 ms).
hipError_t launch_remainder(const appnp_graph* g, const StepArgs& a_in, int epi,
                            const float* z_rem, float* acc, const float* h_rem, int64_t ld_h,
                            float* out, int64_t ld_out, int nv, hipStream_t s) {
  StepArgs a = a_in;
  a.zin = z_rem;
  a.aux = acc;
  if (epi == EPI_BWD) {  // h_rem / ld_h: dH's remainder columns, accumulated into
    a.h = nullptr;
    a.rem_dh = const_cast<float*>(h_rem);
    a.ld_rem_dh = ld_h;
  } else {
    a.h = h_rem;
    a.ld_h = ld_h;
  }
  a.out = out;
  a.ld_out = ld_out;
  a.f = nv;
  const int64_t rows = a.n_rows;
  if (rows <= 0) return hipSuccess;
  a.row_ptr = g->row_ptr;  // whole-row lengths: hub rows are left to the trailing blocks
  a.hub = g->hub;
  a.n_hub = g->hub ? g->n_hub : 0;
  a.light_blocks = (rows + kBlock - 1) / kBlock;
  const int64_t heavy = std::min<int64_t>((a.n_hub + kWavesPerBlock - 1) / kWavesPerBlock, 4096);
  const dim3 grid((unsigned)(a.light_blocks + heavy)), block(kBlock);
  const int nb = g->n_sb;
  for (int32_t b = 0; b < nb; ++b) {
    const int32_t* p = g->sb_ptr + (int64_t)b * rows;
    const bool first = b == 0, last = b == nb - 1;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, block, 0, s, a, p, g->sb_col, g->sb_val);
    };
    if (epi == EPI_BWD) {
      if (first && last) go(k_rem_block<16, EPI_BWD, true, true>);
      else if (first) go(k_rem_block<16, EPI_BWD, true, false>);
      else if (last) go(k_rem_block<16, EPI_BWD, false, true>);
      else go(k_rem_block<16, EPI_BWD, false, false>);
    } else {
      if (first && last) go(k_rem_block<16, EPI_FWD, true, true>);
      else if (first) go(k_rem_block<16, EPI_FWD, true, false>);
      else if (last) go(k_rem_block<16, EPI_FWD, false, true>);
      else go(k_rem_block<16, EPI_FWD, false, false>);
    }
  }
  return hipGetLastError();
}

hipError_t launch_split_copy(const float* h, int64_t ld_h, int64_t n, int64_t f, int64_t fs,
                             float* main, float* rem, hipStream_t s) {
  const int64_t total = n * (fs / 4 + 1);
  if (total <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((total + kBlock - 1) / kBlock, 1 << 20);
  hipLaunchKernelGGL(k_split_copy, dim3((unsigned)blocks), dim3(kBlock), 0, s, h, ld_h, n,
                     (int)f, (int)fs, main, rem);
  return hipGetLastError();
}

}  // namespace appnp
