// appnp_spmm.hip -- one fused APPNP iteration as a CSR x dense SpMM + AXPBY kernel (gfx950).
//
//   Zout[i] = (1-alpha) * sum_j (M_k o A_hat)_ij * Zin[j]  +  alpha * H[i]
//
// Replaces the dense propagation product of the reference, model.py:63
// (`self.ppr[idx] @ self.encoder(X)`), by its K-truncated Neumann series.
//
// The contraction is sparse, so the roofline is HBM (gather) bandwidth, not MFMA.  Layout:
// a row of Z is F contiguous elements (row-major, leading dim ld); each lane owns V
// consecutive features (16-byte vectors where F and ld allow) and a "group" of G lanes covers
// one row slab of G*V features (blockIdx.y selects the slab when F > 64*V).
//
// Two kernel shapes:
//   wide   (G >= 16): one wavefront per row.  The wave loads the row's (col, val) pairs 64 at
//          a time with one coalesced load per lane, stages them in a per-wave LDS tile, and its
//          P = 64/G sub-groups walk the tile interleaved (entry t goes to sub-group t % P),
//          each lane gathering V features of Zin[col] per entry, U entries in flight.
//          Sub-group partial sums are combined with a butterfly (fixed order, deterministic).
//   narrow (G <= 8):  one G-lane group per row, P rows per wave (small F: 3/7/15 features).
// Both fuse the dropout mask, the (1-alpha) scale and the alpha*H AXPBY into the epilogue, so
// every iteration is a single launch that reads CSR + Zin gathers + H and writes Zout once.
#include <algorithm>
#include <cstdlib>

#include "appnp_internal.h"

namespace appnp {

namespace {

// ---- row fragments: V consecutive elements at p.  With TAIL, a lane whose fragment crosses
// the end of the row (rem = f - col0 < V valid elements) WRITES exactly those rem elements,
// in descending power-of-two pieces at compile-time offsets (no runtime register indexing).
// It READS a full vector whenever that stays inside the buffer -- every row but the buffer's
// last, since ld >= roundup(F, V) puts the over-read inside the next row -- so a gather stays
// one load instruction (one set of line requests); only the last row is read piecewise.
// Padding values read that way land in accumulator slots that are never stored.  All tail
// lanes of a wave share rem, so the switches are wave-uniform.
template <typename T, int N, int O, int V>
__device__ __forceinline__ void ld_at(const T* p, float (&x)[V]) {
  float t[N];
  Io<T, N>::load(p + O, t);
#pragma unroll
  for (int i = 0; i < N; ++i) x[O + i] = t[i];
}

template <typename T, int N, int O, int V>
__device__ __forceinline__ void st_at(T* p, const float (&x)[V]) {
  float t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = x[O + i];
  Io<T, N>::store(p + O, t);
}

template <typename T, int V, bool TAIL>
__device__ __forceinline__ void frag_load(const T* p, float (&x)[V], int rem, bool full_ok,
                                          bool nt = false) {
  if (!TAIL || rem >= V || full_ok) {
    if (nt)
      Io<T, V>::load_nt(p, x);
    else
      Io<T, V>::load(p, x);
    return;
  }
#pragma unroll
  for (int v = 0; v < V; ++v) x[v] = 0.0f;
  if constexpr (V == 8) {
    switch (rem) {
      case 1: ld_at<T, 1, 0>(p, x); break;
      case 2: ld_at<T, 2, 0>(p, x); break;
      case 3: ld_at<T, 2, 0>(p, x); ld_at<T, 1, 2>(p, x); break;
      case 4: ld_at<T, 4, 0>(p, x); break;
      case 5: ld_at<T, 4, 0>(p, x); ld_at<T, 1, 4>(p, x); break;
      case 6: ld_at<T, 4, 0>(p, x); ld_at<T, 2, 4>(p, x); break;
      case 7: ld_at<T, 4, 0>(p, x); ld_at<T, 2, 4>(p, x); ld_at<T, 1, 6>(p, x); break;
      default: break;
    }
  } else if constexpr (V == 4) {
    switch (rem) {
      case 1: ld_at<T, 1, 0>(p, x); break;
      case 2: ld_at<T, 2, 0>(p, x); break;
      case 3: ld_at<T, 2, 0>(p, x); ld_at<T, 1, 2>(p, x); break;
      default: break;
    }
  } else if constexpr (V == 2) {
    if (rem == 1) ld_at<T, 1, 0>(p, x);
  }
}

template <typename T, int V, bool TAIL>
__device__ __forceinline__ void frag_store(T* p, const float (&x)[V], int rem, bool nt = false) {
  if (!TAIL || rem >= V) {
    if (nt)
      Io<T, V>::store_nt(p, x);
    else
      Io<T, V>::store(p, x);
    return;
  }
  if constexpr (V == 8) {
    switch (rem) {
      case 1: st_at<T, 1, 0>(p, x); break;
      case 2: st_at<T, 2, 0>(p, x); break;
      case 3: st_at<T, 2, 0>(p, x); st_at<T, 1, 2>(p, x); break;
      case 4: st_at<T, 4, 0>(p, x); break;
      case 5: st_at<T, 4, 0>(p, x); st_at<T, 1, 4>(p, x); break;
      case 6: st_at<T, 4, 0>(p, x); st_at<T, 2, 4>(p, x); break;
      case 7: st_at<T, 4, 0>(p, x); st_at<T, 2, 4>(p, x); st_at<T, 1, 6>(p, x); break;
      default: break;
    }
  } else if constexpr (V == 4) {
    switch (rem) {
      case 1: st_at<T, 1, 0>(p, x); break;
      case 2: st_at<T, 2, 0>(p, x); break;
      case 3: st_at<T, 2, 0>(p, x); st_at<T, 1, 2>(p, x); break;
      default: break;
    }
  } else if constexpr (V == 2) {
    if (rem == 1) st_at<T, 1, 0>(p, x);
  }
}

template <typename T, int V, int EPI, bool TAIL>
__device__ __forceinline__ void epilogue(const StepArgs& a, int64_t row, int col0,
                                         const float (&acc)[V], const float (&hv)[V],
                                         const float (&pv)[V], int rem) {
  float y[V];
#pragma unroll
  for (int v = 0; v < V; ++v) y[v] = a.scale * acc[v];
  if constexpr (EPI == EPI_FWD) {
#pragma unroll
    for (int v = 0; v < V; ++v) y[v] = fmaf(a.alpha, hv[v], y[v]);
    frag_store<T, V, TAIL>(static_cast<T*>(a.out) + row * a.ld_out + col0, y, rem,
                           a.nt & 4);
  } else if constexpr (EPI == EPI_BWD) {
    if (a.out) frag_store<T, V, TAIL>(static_cast<T*>(a.out) + row * a.ld_out + col0, y, rem);
    float dv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) dv[v] = fmaf(a.alpha, y[v], pv[v]);
    frag_store<T, V, TAIL>(static_cast<T*>(a.aux) + row * a.ld_aux + col0, dv, rem);
  } else if constexpr (EPI == EPI_PARTIAL) {
    frag_store<float, V, TAIL>(static_cast<float*>(a.out) + row * a.ld_out + col0, y, rem);
  } else if constexpr (EPI == EPI_ACCUM) {
#pragma unroll
    for (int v = 0; v < V; ++v) y[v] += pv[v];
    frag_store<float, V, TAIL>(static_cast<float*>(a.out) + row * a.ld_out + col0, y, rem);
  } else {  // EPI_FINISH
#pragma unroll
    for (int v = 0; v < V; ++v) y[v] = fmaf(a.alpha, hv[v], y[v] + pv[v]);
    frag_store<T, V, TAIL>(static_cast<T*>(a.out) + row * a.ld_out + col0, y, rem);
  }
}

// The row's epilogue operands, loaded when the row starts so their latency hides under the
// gathers: H (forward, finish), dH (adjoint, in `aux`) and the fp32 partial of the
// row-partition steps (accumulate: the partial in `out`; finish: the one in `aux`).
template <typename T, int V, int EPI, bool TAIL>
__device__ __forceinline__ void load_h(const StepArgs& a, int64_t row, int col0, float (&hv)[V],
                                       float (&pv)[V], int rem) {
  if constexpr (EPI == EPI_FWD || EPI == EPI_FINISH) {
    frag_load<T, V, TAIL>(static_cast<const T*>(a.h) + row * a.ld_h + col0, hv, rem,
                          row + 1 < a.n_rows, a.nt & 2);
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) hv[v] = 0.0f;
  }
  if constexpr (EPI == EPI_BWD) {
    frag_load<T, V, TAIL>(static_cast<const T*>(a.aux) + row * a.ld_aux + col0, pv, rem,
                          row + 1 < a.n_rows);
  } else if constexpr (EPI == EPI_ACCUM) {
    frag_load<float, V, TAIL>(static_cast<const float*>(a.out) + row * a.ld_out + col0, pv, rem,
                              row + 1 < a.n_rows);
  } else if constexpr (EPI == EPI_FINISH) {
    frag_load<float, V, TAIL>(static_cast<const float*>(a.aux) + row * a.ld_aux + col0, pv, rem,
                              row + 1 < a.n_rows);
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) pv[v] = 0.0f;
  }
}

// ------------------------------------------------------------------------------------------
// one wavefront on one row: P = 64/G sub-groups split the row's entries
// ------------------------------------------------------------------------------------------
template <typename T, int V, int G, int EPI, int U, bool TAIL>
__device__ __forceinline__ void wave_row(const StepArgs& a, int64_t row, int lane, int2* tile,
                                         int col0, int rem) {
  constexpr int P = kWave / G;
  const int sub = lane / G;
  const bool fact = rem > 0;
  const T* __restrict__ zin = static_cast<const T*>(a.zin);
  const int beg = a.row_ptr[row];
  const int end = row_end_of(a, row);
  float hv[V], pv[V];
  if (sub == 0 && fact) load_h<T, V, EPI, TAIL>(a, row, col0, hv, pv, rem);
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.0f;

  for (int cb = beg; cb < end; cb += kWave) {
    const int n = min(kWave, end - cb);
    int c = 0;
    float w = 0.0f;
    if (lane < n) {
      float v = 1.0f;
      if (a.nt & 1) {
        c = ld_nt<int32_t>(a.col + cb + lane);
        if (a.val) v = ld_nt<float>(a.val + cb + lane);
      } else {
        c = a.col[cb + lane];
        if (a.val) v = a.val[cb + lane];
      }
      w = edge_weight(v, a.row_lo + row, c, a);
    }
    tile[lane] = make_int2(c, __float_as_int(w));
    __builtin_amdgcn_wave_barrier();
    for (int t = sub; t < n; t += P * U) {
      int2 e[U];
      float z[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = t + u * P;
        e[u] = idx < n ? tile[idx] : make_int2(0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (fact && t + u * P < n) {
          frag_load<T, V, TAIL>(zin + (int64_t)e[u].x * a.ld_in + col0, z[u], rem,
                                e[u].x + 1 < a.zin_rows);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) z[u][v] = 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float wu = __int_as_float(e[u].y);
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = fmaf(wu, z[u][v], acc[v]);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  // combine the P sub-group partial sums (butterfly, fixed order)
#pragma unroll
  for (int off = G; off < kWave; off <<= 1) {
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] += __shfl_xor(acc[v], off);
  }
  if (sub == 0 && fact) epilogue<T, V, EPI, TAIL>(a, row, col0, acc, hv, pv, rem);
}

// ------------------------------------------------------------------------------------------
// wide: one wavefront per row
// ------------------------------------------------------------------------------------------
template <typename T, int V, int G, int EPI, int U, bool TAIL>
__global__ __launch_bounds__(kBlock) void k_step_wide(StepArgs a) {
  __shared__ int2 stage[kWavesPerBlock][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col0 = blockIdx.y * (G * V) + (lane % G) * V;
  const int rem = a.f - col0;  // valid features of this lane's fragment (>= V: full)
  const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
  // Longest-first dispatch: virtual rows [0, n_hub) are the hub rows (> kHubRow entries), so
  // the longest waves start first and do not become the launch's tail; the regular pass
  // skips them.  Pure scheduling: each row is still computed by exactly one wave.
  const int64_t total = a.n_rows + a.n_hub;
  for (int64_t v = (int64_t)blockIdx.x * kWavesPerBlock + wave; v < total; v += nwaves) {
    int64_t row;
    if (v < a.n_hub) {
      row = a.hub[v];
    } else {
      row = v - a.n_hub;
      if (a.hub && a.row_ptr[row + 1] - a.row_ptr[row] > kHubRow) continue;
    }
    wave_row<T, V, G, EPI, U, TAIL>(a, row, lane, stage[wave], col0, rem);
  }
}

// ------------------------------------------------------------------------------------------
// narrow: one G-lane group per row, P = 64/G rows per wave.  Rows longer than a.heavy_thr
// (listed in a.heavy at graph creation) are skipped here and processed by the trailing
// blocks (blockIdx.x >= a.light_blocks), one whole wavefront per row (wave_row), so a hub row
// of a power-law graph does not serialise on G lanes while the rest of the launch waits.
// ------------------------------------------------------------------------------------------
template <typename T, int V, int G, int EPI, int U, bool TAIL>
__global__ __launch_bounds__(kBlock) void k_step_narrow(StepArgs a) {
  constexpr int P = kWave / G;
  __shared__ int2 stage[kWavesPerBlock][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int sub = lane / G;
  const int gl = lane % G;
  const int col0 = blockIdx.y * (G * V) + gl * V;
  const int rem = a.f - col0;  // valid features of this lane's fragment (>= V: full)
  const bool fact = rem > 0;
  const T* __restrict__ zin = static_cast<const T*>(a.zin);

  if ((int64_t)blockIdx.x >= a.light_blocks) {  // heavy rows: a wavefront each
    const int64_t hw = ((int64_t)blockIdx.x - a.light_blocks) * kWavesPerBlock + wave;
    const int64_t hstride = ((int64_t)gridDim.x - a.light_blocks) * kWavesPerBlock;
    for (int64_t h = hw; h < a.n_heavy; h += hstride)
      wave_row<T, V, G, EPI, U, TAIL>(a, a.heavy[h], lane, stage[wave], col0, rem);
    return;
  }
  const int64_t stride = a.light_blocks * kWavesPerBlock * P;
  for (int64_t rb = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * P; rb < a.n_rows;
       rb += stride) {
    const int64_t row = rb + sub;
    if (row >= a.n_rows) continue;
    const int beg = a.row_ptr[row];
    const int end = row_end_of(a, row);
    if (a.heavy && end - beg > a.heavy_thr) continue;
    float hv[V], pv[V];
    if (fact) load_h<T, V, EPI, TAIL>(a, row, col0, hv, pv, rem);
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.0f;
    for (int e = beg; e < end; e += U) {
      int c[U];
      float w[U];
      float z[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (e + u < end) {
          float v = 1.0f;
          if (a.nt & 1) {
            c[u] = ld_nt<int32_t>(a.col + e + u);
            if (a.val) v = ld_nt<float>(a.val + e + u);
          } else {
            c[u] = a.col[e + u];
            if (a.val) v = a.val[e + u];
          }
          w[u] = edge_weight(v, a.row_lo + row, c[u], a);
        } else {
          c[u] = 0;
          w[u] = 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (fact && e + u < end) {
          frag_load<T, V, TAIL>(zin + (int64_t)c[u] * a.ld_in + col0, z[u], rem,
                                c[u] + 1 < a.zin_rows);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) z[u][v] = 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = fmaf(w[u], z[u][v], acc[v]);
      }
    }
    if (fact) epilogue<T, V, EPI, TAIL>(a, row, col0, acc, hv, pv, rem);
  }
}

template <typename T, int V, int EPI, bool TAIL, int U>
hipError_t launch_wide(int G, dim3 grid, const StepArgs& a, hipStream_t s) {
  const dim3 block(kBlock);
  switch (G) {
    case 1: hipLaunchKernelGGL((k_step_wide<T, V, 1, EPI, U, TAIL>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_step_wide<T, V, 2, EPI, U, TAIL>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((k_step_wide<T, V, 4, EPI, U, TAIL>), grid, block, 0, s, a); break;
    case 8: hipLaunchKernelGGL((k_step_wide<T, V, 8, EPI, U, TAIL>), grid, block, 0, s, a); break;
    case 16: hipLaunchKernelGGL((k_step_wide<T, V, 16, EPI, U, TAIL>), grid, block, 0, s, a); break;
    case 32: hipLaunchKernelGGL((k_step_wide<T, V, 32, EPI, U, TAIL>), grid, block, 0, s, a); break;
    case 64: hipLaunchKernelGGL((k_step_wide<T, V, 64, EPI, U, TAIL>), grid, block, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T, int V, int EPI, bool TAIL, int UN>
hipError_t launch_narrow(int G, dim3 grid, const StepArgs& a, hipStream_t s) {
  const dim3 block(kBlock);
  switch (G) {
    case 1: hipLaunchKernelGGL((k_step_narrow<T, V, 1, EPI, UN, TAIL>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_step_narrow<T, V, 2, EPI, UN, TAIL>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((k_step_narrow<T, V, 4, EPI, UN, TAIL>), grid, block, 0, s, a); break;
    case 8: hipLaunchKernelGGL((k_step_narrow<T, V, 8, EPI, UN, TAIL>), grid, block, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// entries in flight: uw per sub-group of the wide kernels, un per row of the narrow ones
template <typename T, int V, int EPI, bool TAIL>
hipError_t launch_g(int G, bool wide, int uw, int un, dim3 grid, const StepArgs& a,
                    hipStream_t s) {
  if (wide) {
    if (uw == 8) return launch_wide<T, V, EPI, TAIL, 8>(G, grid, a, s);
    if (uw == 4) return launch_wide<T, V, EPI, TAIL, 4>(G, grid, a, s);
    if (uw == 2) return launch_wide<T, V, EPI, TAIL, 2>(G, grid, a, s);
    return launch_wide<T, V, EPI, TAIL, 1>(G, grid, a, s);
  }
  if constexpr (V <= 2) {
    if (un == 8) return launch_narrow<T, V, EPI, TAIL, 8>(G, grid, a, s);
  }
  return launch_narrow<T, V, EPI, TAIL, 4>(G, grid, a, s);
  return hipGetLastError();
}

template <typename T, int EPI>
hipError_t launch_v(int V, int G, bool wide, int uw, int un, dim3 grid, const StepArgs& a,
                    hipStream_t s) {
  const bool tail = (a.f % V) != 0;
  switch (V) {
    case 1: return launch_g<T, 1, EPI, false>(G, wide, uw, un, grid, a, s);
    case 2: return tail ? launch_g<T, 2, EPI, true>(G, wide, uw, un, grid, a, s)
                        : launch_g<T, 2, EPI, false>(G, wide, uw, un, grid, a, s);
    case 4: return tail ? launch_g<T, 4, EPI, true>(G, wide, uw, un, grid, a, s)
                        : launch_g<T, 4, EPI, false>(G, wide, uw, un, grid, a, s);
    case 8:
      if constexpr (sizeof(T) == 2)
        return tail ? launch_g<T, 8, EPI, true>(G, wide, uw, un, grid, a, s)
                    : launch_g<T, 8, EPI, false>(G, wide, uw, un, grid, a, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// Largest vector width (elements) valid for every operand: all leading dims and all base
// pointers must be multiples of V elements.  F need not be: the lane holding the last
// fragment of a row then touches only the valid elements (TAIL kernels).  A vector wider
// than F itself is never chosen.
int pick_vec(int dtype, int64_t f, const int64_t* lds, int n_ld, const void* const* ptrs,
             int n_ptr) {
  const int es = dtype == 0 ? 4 : 2;
  int v = dtype == 0 ? 4 : 8;
  for (; v > 1; v >>= 1) {
    bool ok = v <= f || (f % v) == 0;
    for (int i = 0; i < n_ld && ok; ++i) ok = (lds[i] % v) == 0;
    for (int i = 0; i < n_ptr && ok; ++i)
      ok = ptrs[i] == nullptr || (reinterpret_cast<uintptr_t>(ptrs[i]) % (uintptr_t)(v * es)) == 0;
    if (ok) break;
  }
  return v;
}

hipError_t launch_step(int dtype, int epi, int V, const StepArgs& a_in, hipStream_t s) {
  StepArgs a = a_in;
  if (a.n_rows <= 0 || a.f <= 0) return hipSuccess;
  // lanes per row slab: smallest power of two covering min(F, 64V) features
  auto lanes_for = [&](int v) {
    const int64_t need = (std::min<int64_t>(a.f, 64LL * v) + v - 1) / v;
    int g = 1;
    while (g < need) g <<= 1;
    return g;
  };
  // Small graphs are latency-bound: there a wavefront per row (its entries staged once and
  // gathered in one round by 64/G sub-groups) beats G-lane rows that walk their entries a
  // few at a time; large graphs keep G-lane rows for narrow F (fewer instructions per byte).
  // Latency regime (<= 64k rows, measured on pubmed/ms-academic/cora-sized graphs): one
  // feature per lane (V = 1 while F <= 64) -- more lanes per row and a short sub-group
  // reduction -- and a wavefront per row only when the graph has hub rows.
  constexpr int64_t kLatencyRows = 1 << 16;
  const bool latency = a.n_rows <= kLatencyRows;
  const int v_max = V;  // widest vector every operand allows (pick_vec)
  const bool heavy_rows = a.heavy && a.n_heavy > 0;
  if (latency && !heavy_rows) {
    int v = 1;
    while (v < V && (int64_t)64 * v < a.f) v <<= 1;
    V = v;
  }
  // latency regime with hub rows (a wavefront per row): the widest vector, so a row needs the
  // fewest lanes and the most sub-groups walk the longest row at once (Cora-ML 5.94 -> 5.21 us
  // per iteration with V = 4 instead of 1; Citeseer 4.06 -> 3.89 us with V = 2)
  static const int v_env = tuning_env("APPNP_VEC", -1);  // tuning override (<= pick_vec's)
  if (v_env > 0 && v_env <= v_max) V = v_env;
  const int G = lanes_for(V);
  // Bandwidth regime: a wavefront per row also for narrow F once rows are long on average
  // (products-synth slabs of 4-25 features, 51.5 entries a row: 6-10 % faster than G-lane
  // rows; uniform and power-law; arxiv-synth, 14.8 a row: G-lane rows 20-50 % faster).
  const bool long_rows = a.nnz >= (int64_t)kWideAvgRow * a.n_rows;
  static const int wide_env = tuning_env("APPNP_WIDE", -1);  // tuning override
  const bool wide = wide_env >= 0 ? wide_env != 0
                                  : (G >= 16 || (latency && heavy_rows) || (!latency && long_rows));
  const int64_t slabs = (a.f + (int64_t)G * V - 1) / ((int64_t)G * V);
  const int64_t rows_per_block = wide ? kWavesPerBlock : (int64_t)kWavesPerBlock * (kWave / G);
  // one wave per row (wide) by default: measured best on products-synth (tools/tune.sh)
  // gridDim.x * 256 must stay below 2^32: cap at 4M blocks (grid-stride loops take the rest;
  // products-synth needs 612k, i.e. one wave per row)
  static const int max_blocks = std::min(tuning_env("APPNP_MAX_BLOCKS", 1 << 22), 1 << 22);
  if (!wide || !a.hub) {
    a.hub = nullptr;
    a.n_hub = 0;
  }
  int64_t blocks = (a.n_rows + a.n_hub + rows_per_block - 1) / rows_per_block;
  if (blocks > max_blocks) blocks = max_blocks;
  a.light_blocks = blocks;
  if (!wide && a.heavy && a.n_heavy > 0) {
    const int64_t hb = std::min<int64_t>((a.n_heavy + kWavesPerBlock - 1) / kWavesPerBlock, 4096);
    blocks += hb;
  } else {
    a.heavy = nullptr;
    a.n_heavy = 0;
  }
  const dim3 grid((unsigned)blocks, (unsigned)slabs);
  // entries in flight per sub-group of the wide kernel (tools/sweep_uw_bw.sh,
  // tools/sweep_uw.sh).  Bandwidth regime with long rows (>= kWideAvgRow on average): 2 --
  // products-synth fp32 F = 96 8.20 -> 7.32 ms, F = 100 9.76 -> 9.57, products-powerlaw
  // 9.84 -> 9.06, bf16 and F = 128 +0.4-1 %; 4 is no better and costs VGPRs.  Short rows
  // (arxiv-synth, 14.8 a row): 1, 3 % faster than 2.  Small graphs with hub rows (latency
  // regime, wave per row because of them): 8, so the longest row -- which sets the launch
  // time -- takes few dependent rounds (Cora-ML 9.4 -> 5.8 us, Citeseer 5.4 -> 3.9 us).
  // Short rows keep 1 when they are whole rows, but not when they are a range of long rows (the
  // LOCAL half of a row-partitioned step, the shard groups of a pipelined one: 6-26 entries a
  // row of products-synth's 51.5): there 2 is 3-10 % faster (profiles/r6_row8_pipeline.txt,
  // h3_*), while arxiv-synth's whole 14.8-entry rows keep 1 (2 % faster; h4_*).
  const int64_t whole = a.nnz_rows > 0 ? a.nnz_rows : a.nnz;
  const bool long_whole = whole >= (int64_t)kWideAvgRow * a.n_rows;
  static const int uw_env = tuning_env("APPNP_UW", -1);  // tuning override (1, 2, 4, 8)
  const int uw = uw_env > 0                ? uw_env
                 : (latency && heavy_rows) ? 8
                 : (!latency && (long_rows || long_whole)) ? 2
                                                           : 1;
  // cache policy of the streams (StepArgs::nt); APPNP_NT overrides for measurement
  // entries in flight per row of the narrow kernels: 8 in the latency regime, where a row's
  // dependent rounds set the launch time (pubmed-synth 5.77 -> 5.24 us, cora-sized uniform
  // 6.01 -> 5.45 us per iteration; tools/sweep_uw.sh), else 4
  static const int un_env = tuning_env("APPNP_UN", -1);  // tuning override (4, 8)
  const int un = un_env > 0 ? un_env : latency ? 8 : 4;
  static const int nt_env = tuning_env("APPNP_NT", -1);
  a.nt = nt_env >= 0 ? nt_env : (latency ? 0 : 1);
  if (dtype == 0) {
    switch (epi) {
      case EPI_FWD: return launch_v<float, EPI_FWD>(V, G, wide, uw, un, grid, a, s);
      case EPI_BWD: return launch_v<float, EPI_BWD>(V, G, wide, uw, un, grid, a, s);
      case EPI_PARTIAL: return launch_v<float, EPI_PARTIAL>(V, G, wide, uw, un, grid, a, s);
      case EPI_FINISH: return launch_v<float, EPI_FINISH>(V, G, wide, uw, un, grid, a, s);
      case EPI_ACCUM: return launch_v<float, EPI_ACCUM>(V, G, wide, uw, un, grid, a, s);
    }
  } else {
    switch (epi) {
      case EPI_FWD: return launch_v<uint16_t, EPI_FWD>(V, G, wide, uw, un, grid, a, s);
      case EPI_BWD: return launch_v<uint16_t, EPI_BWD>(V, G, wide, uw, un, grid, a, s);
    }
  }
  return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------
// small helpers: dst[i, :f] = alpha * src[i, :f]   (dH init of the adjoint; K = 0 copy)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_scale_rows(const T* __restrict__ src, int64_t ld_src,
                                                       T* __restrict__ dst, int64_t ld_dst,
                                                       int64_t n, int64_t f, float alpha) {
  const int64_t total = n * f;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / f, c = i - r * f;
    float x[1];
    Io<T, 1>::load(src + r * ld_src + c, x);
    x[0] *= alpha;
    Io<T, 1>::store(dst + r * ld_dst + c, x);
  }
}

hipError_t launch_scale_rows(int dtype, const void* src, int64_t ld_src, void* dst,
                             int64_t ld_dst, int64_t n, int64_t f, float alpha, hipStream_t s) {
  const int64_t total = n * f;
  if (total <= 0) return hipSuccess;
  int64_t blocks = (total + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (dtype == 0)
    hipLaunchKernelGGL(k_scale_rows<float>, dim3((unsigned)blocks), dim3(kBlock), 0, s,
                       static_cast<const float*>(src), ld_src, static_cast<float*>(dst), ld_dst,
                       n, f, alpha);
  else
    hipLaunchKernelGGL(k_scale_rows<uint16_t>, dim3((unsigned)blocks), dim3(kBlock), 0, s,
                       static_cast<const uint16_t*>(src), ld_src, static_cast<uint16_t*>(dst),
                       ld_dst, n, f, alpha);
  return hipGetLastError();
}

}  // namespace appnp
