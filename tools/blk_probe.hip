// blk_probe.hip -- measured prototype: the persistent L2-blocked pass of appnp_blocks.hip
// (k_rem_persist, 16-B rows) widened to W = 4 * LPE fp32 columns.  Not part of the library.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/blk_probe.hip -o tools/bin/blk_probe
//   [BLK_N=n BLK_DEG=d] tools/bin/blk_probe W:br:U[:em] [...]   (W in 4, 8, 16, 32; br = log2 source rows
//                                                 per block; U = chunks in flight per wave)
//
// Question: the random-gather SpMM is bound by ~56 G line requests/s from
// HBM / Infinity Cache; L2-resident rows are served ~2.5x faster, but reuse in L2 needs the
// destination sums on chip: a line brought into an XCD's L2 is reused r = a d / N times,
// a = destination rows the XCD holds on chip (LDS: 5 MB per XCD / (4 W) bytes per row).
//   W = 32 (one line per row):  a = 41 k rows, r = 0.86 -- tools/tile2d_probe.hip, rejected.
//   W = 16 (half line):         a = 82 k rows, r = 1.7, and the [n, 16] table (157 MB)
//                               stays in the 256 MB Infinity Cache across the row passes.
// The kernel is k_rem_persist with LPE = W / 4 lanes per entry, laid out quarter-major:
// lane = q * CH + e (entry e of a chunk of CH = 64 / LPE entries, 16-B piece q of its row),
// so each 16-lane DPP row holds one piece of up to 16 consecutive entries and the segmented
// scan over entries is the same row_shr 1/2/4/8 (+ row_bcast15 for CH = 32, + row_bcast31
// for CH = 64) with the compare key (row, q).
//
// Workload: products-synth's shape (n = 2,449,029, 51 uniform random columns + the diagonal
// per row, 127.3 M nonzeros), Y = A Z with A's values 1/52, one W-column slab; the direct
// gather (a wavefront per destination row, LPE lanes per entry) is the baseline and the
// reference for the values.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kWaves = 16, kThreads = kWaves * 64;
constexpr int kLds = 160 * 1024;
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kColBits = 20;

template <int LPE>
__global__ __launch_bounds__(256) void k_direct(const int* __restrict__ rp,
                                                const int* __restrict__ col, float w,
                                                const f4* __restrict__ z, f4* __restrict__ y,
                                                int n) {
  constexpr int CH = 64 / LPE;
  const int lane = threadIdx.x & 63;
  const int e8 = lane / LPE, q = lane % LPE;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += gridDim.x * 4) {
    const int beg = rp[row], end = rp[row + 1];
    f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int e = beg + e8; e < end; e += 2 * CH) {
      const int c0 = __builtin_nontemporal_load(col + e);
      const bool has1 = e + CH < end;
      const int c1 = has1 ? __builtin_nontemporal_load(col + e + CH) : 0;
      const f4 a = z[(int64_t)c0 * LPE + q];
      const f4 b = has1 ? z[(int64_t)c1 * LPE + q] : f4{0.0f, 0.0f, 0.0f, 0.0f};
      acc += a + b;
    }
    for (int o = LPE; o < 64; o <<= 1)
      acc += f4{__shfl_xor(acc.x, o), __shfl_xor(acc.y, o), __shfl_xor(acc.z, o),
                __shfl_xor(acc.w, o)};
    if (lane < LPE) y[(int64_t)row * LPE + q] = acc * w;
  }
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void seg_step(int key, f4& v) {
  const int src = __builtin_amdgcn_update_dpp(0, key, CTRL, ROW_MASK, 0xf, true);
  const float ux = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.x), CTRL, ROW_MASK, 0xf, true));
  const float uy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.y), CTRL, ROW_MASK, 0xf, true));
  const float uz = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.z), CTRL, ROW_MASK, 0xf, true));
  const float uw = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.w), CTRL, ROW_MASK, 0xf, true));
  if (src == key) {
    v.x += ux;
    v.y += uy;
    v.z += uz;
    v.w += uw;
  }
}

// segmented inclusive scan over runs of equal key along the lanes of each piece q (lanes
// q*CH .. q*CH+CH-1), running only the steps some run needs
template <int CH>
__device__ __forceinline__ void seg_scan(int key, f4& v, unsigned long long heads) {
  // lanes at distance >= 1 from their run head (a piece's first lane is always a head)
  unsigned long long m = ~(heads | 0x0001000100010001ull);
  if (m) {
    seg_step<0x111, 0xf>(key, v);
    m &= m << 1;
    if (CH > 2 && m) {
      seg_step<0x112, 0xf>(key, v);
      m &= m << 2;
      if (CH > 4 && m) {
        seg_step<0x114, 0xf>(key, v);
        if (CH > 8 && (m & (m << 4))) seg_step<0x118, 0xf>(key, v);
      }
    }
  }
  if constexpr (CH >= 32) {
    if (~heads & ((1ull << 16) | (1ull << 48))) seg_step<0x142, 0xa>(key, v);
  }
  if constexpr (CH == 64) {
    if (~heads & (1ull << 32)) seg_step<0x143, 0xc>(key, v);
  }
}

template <int LPE, int U>
__global__ __launch_bounds__(kThreads) void k_blk(const int* __restrict__ off,
                                                  const uint32_t* __restrict__ ent,
                                                  const int* __restrict__ cblk, int br_log2,
                                                  int nb, int slots, int rg, int passes, float w,
                                                  const f4* __restrict__ z, f4* __restrict__ y,
                                                  int n) {
  constexpr int CH = 64 / LPE;
  extern __shared__ f4 acc_all[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane / CH, e = lane % CH;
  f4* acc = acc_all + (int64_t)wv * rg * LPE;
  const uint32_t cmask = (1u << kColBits) - 1u;
  // a piece's first lane always starts a run
  unsigned long long first = 0;
  for (int t = 0; t < LPE; ++t) first |= 1ull << (t * CH);
  for (int p = 0; p < passes; ++p) {
    const int64_t g = (int64_t)p * slots + (int64_t)blockIdx.x * kWaves + wv;
    const int64_t r0 = g * rg;
    const int64_t left = n - r0;
    const int rows = left <= 0 ? 0 : (left < rg ? (int)left : rg);
    for (int i = lane; i < rows * LPE; i += 64) acc[i] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const int c_end = off[(g + 1) * nb] / CH;
    for (int c = off[g * nb] / CH; c < c_end; c += U) {
      const int nch = c_end - c < U ? c_end - c : U;
      uint32_t en[U];
      int cb[U];
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        en[u] = kNone;
        cb[u] = 0;
        if (u < nch) {
          en[u] = __builtin_nontemporal_load(ent + (int64_t)(c + u) * CH + e);
          cb[u] = cblk[c + u] << br_log2;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = en[u] != kNone ? z[(int64_t)(cb[u] + (int)(en[u] & cmask)) * LPE + q]
                              : f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u >= nch) break;
        const bool act = en[u] != kNone;
        const int row = (int)(en[u] >> kColBits);
        const int key = (row << 3) | q;
        const int prev = __builtin_amdgcn_update_dpp(-1, key, 0x138, 0xf, 0xf, false);
        const unsigned long long heads = __ballot(prev != key || !act) | first;
        f4 s = v[u];
        seg_scan<CH>(key, s, heads);
        const bool tail = e == CH - 1 || ((heads >> (lane + 1)) & 1ull);
        if (act && tail) {
          const f4 a = acc[row * LPE + q];
          acc[row * LPE + q] = a + s;
        }
      }
    }
    for (int i = lane; i < rows * LPE; i += 64) y[r0 * LPE + i] = acc[i] * w;
  }
}

// Entry-major variant: lane = e * LPE + q, so the LPE lanes of one entry read its row's
// W * 4 contiguous bytes in one go (one L1 tag lookup / L2 request instead of LPE); the
// gathered pieces (and entry words) are then moved to the quarter-major order of k_blk by
// ds_bpermute, and the scan and LDS update are k_blk's.
template <int LPE, int U>
__global__ __launch_bounds__(kThreads) void k_blk_em(const int* __restrict__ off,
                                                     const uint32_t* __restrict__ ent,
                                                     const int* __restrict__ cblk, int br_log2,
                                                     int nb, int slots, int rg, int passes,
                                                     float w, const f4* __restrict__ z,
                                                     f4* __restrict__ y, int n) {
  constexpr int CH = 64 / LPE;
  extern __shared__ f4 acc_all[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane / CH, e = lane % CH;          // quarter-major position (scan, LDS)
  const int le = lane / LPE, lq = lane % LPE;      // entry-major position (gather)
  const int src = (e * LPE + q) * 4;               // bpermute byte address of my piece
  f4* acc = acc_all + (int64_t)wv * rg * LPE;
  const uint32_t cmask = (1u << kColBits) - 1u;
  unsigned long long first = 0;
  for (int t = 0; t < LPE; ++t) first |= 1ull << (t * CH);
  for (int p = 0; p < passes; ++p) {
    const int64_t g = (int64_t)p * slots + (int64_t)blockIdx.x * kWaves + wv;
    const int64_t r0 = g * rg;
    const int64_t left = n - r0;
    const int rows = left <= 0 ? 0 : (left < rg ? (int)left : rg);
    for (int i = lane; i < rows * LPE; i += 64) acc[i] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const int c_end = off[(g + 1) * nb] / CH;
    for (int c = off[g * nb] / CH; c < c_end; c += U) {
      const int nch = c_end - c < U ? c_end - c : U;
      uint32_t en[U];
      int cb[U];
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        en[u] = kNone;
        cb[u] = 0;
        if (u < nch) {
          en[u] = __builtin_nontemporal_load(ent + (int64_t)(c + u) * CH + le);
          cb[u] = cblk[c + u] << br_log2;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = en[u] != kNone ? z[(int64_t)(cb[u] + (int)(en[u] & cmask)) * LPE + lq]
                              : f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u >= nch) break;
        const uint32_t ew = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)en[u]);
        f4 s;
        s.x = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[u].x)));
        s.y = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[u].y)));
        s.z = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[u].z)));
        s.w = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v[u].w)));
        const bool act = ew != kNone;
        const int row = (int)(ew >> kColBits);
        const int key = (row << 3) | q;
        const int prev = __builtin_amdgcn_update_dpp(-1, key, 0x138, 0xf, 0xf, false);
        const unsigned long long heads = __ballot(prev != key || !act) | first;
        seg_scan<CH>(key, s, heads);
        const bool tail = e == CH - 1 || ((heads >> (lane + 1)) & 1ull);
        if (act && tail) {
          const f4 a = acc[row * LPE + q];
          acc[row * LPE + q] = a + s;
        }
      }
    }
    for (int i = lane; i < rows * LPE; i += 64) y[r0 * LPE + i] = acc[i] * w;
  }
}

struct Graph {
  int n;
  int64_t nnz;
  std::vector<int> rp, col;
};

template <int LPE>
float run_direct(const Graph& G, const int* d_rp, const int* d_col, const f4* d_z, f4* d_y,
                 float w, hipEvent_t a, hipEvent_t b) {
  const int n = G.n;
  auto body = [&] {
    hipLaunchKernelGGL(k_direct<LPE>, dim3((n + 3) / 4), dim3(256), 0, 0, d_rp, d_col, w, d_z,
                       d_y, n);
  };
  for (int i = 0; i < 2; ++i) body();
  CHECK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) body();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int LPE, int U, bool EM>
float run_blk(const Graph& G, int br, const f4* d_z, f4* d_y, float w, hipEvent_t a,
              hipEvent_t b, double* pad, int cus) {
  constexpr int CH = 64 / LPE;
  const int n = G.n;
  const int slots = cus * kWaves;
  const int max_rg = kLds / (kWaves * 16 * LPE);
  const int passes = (int)((n + (int64_t)slots * max_rg - 1) / ((int64_t)slots * max_rg));
  const int rg = (int)((n + (int64_t)passes * slots - 1) / ((int64_t)passes * slots));
  const int64_t groups = (int64_t)passes * slots;
  const int nb = (n + (1 << br) - 1) >> br;
  std::vector<int> cnt(groups * nb, 0);
  for (int64_t g = 0; g < groups; ++g)
    for (int64_t i = g * rg; i < std::min<int64_t>(n, g * rg + rg); ++i)
      for (int e = G.rp[i]; e < G.rp[i + 1]; ++e) ++cnt[g * nb + (G.col[e] >> br)];
  std::vector<int> off(groups * nb + 1, 0);
  int64_t tot = 0;
  for (int64_t s = 0; s < groups * nb; ++s) {
    off[s] = (int)tot;
    tot += (cnt[s] + CH - 1) / CH * CH;
  }
  off[groups * nb] = (int)tot;
  std::vector<uint32_t> ent(tot, kNone);
  std::vector<int> cblk(tot / CH);
  std::vector<int> cur(off.begin(), off.end() - 1);
  for (int64_t g = 0; g < groups; ++g)
    for (int64_t i = g * rg; i < std::min<int64_t>(n, g * rg + rg); ++i)
      for (int e = G.rp[i]; e < G.rp[i + 1]; ++e) {
        const int bb = G.col[e] >> br;
        ent[cur[g * nb + bb]++] = ((uint32_t)(i - g * rg) << kColBits) |
                                  (uint32_t)(G.col[e] & ((1 << br) - 1));
      }
  for (int64_t s = 0; s < groups * nb; ++s)
    for (int c = off[s] / CH; c < off[s + 1] / CH; ++c) cblk[c] = (int)(s % nb);
  *pad = (double)(tot - G.nnz) / G.nnz;
  int *d_off, *d_cblk;
  uint32_t* d_ent;
  CHECK(hipMalloc(&d_off, off.size() * 4));
  CHECK(hipMalloc(&d_ent, tot * 4));
  CHECK(hipMalloc(&d_cblk, std::max<size_t>(1, cblk.size()) * 4));
  CHECK(hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ent, ent.data(), tot * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_cblk, cblk.data(), cblk.size() * 4, hipMemcpyHostToDevice));
  auto kern = EM ? k_blk_em<LPE, U> : k_blk<LPE, U>;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  const size_t lds = (size_t)kWaves * rg * LPE * 16;
  auto body = [&] {
    hipLaunchKernelGGL(kern, dim3(cus), dim3(kThreads), lds, 0, d_off, d_ent, d_cblk,
                       br, nb, slots, rg, passes, w, d_z, d_y, n);
  };
  for (int i = 0; i < 2; ++i) body();
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) body();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipFree(d_off));
  CHECK(hipFree(d_ent));
  CHECK(hipFree(d_cblk));
  printf("#   W=%d: %d passes of %d groups x %d rows, %d blocks, %lld padded entries\n",
         LPE * 4, passes, slots, rg, nb, (long long)tot);
  return ms / 10;
}

int main(int argc, char** argv) {
  Graph G;
  // BLK_N / BLK_DEG: another graph shape (arxiv-synth: BLK_N=169343 BLK_DEG=14)
  const int n = getenv("BLK_N") ? atoi(getenv("BLK_N")) : 2449029;
  const int deg = getenv("BLK_DEG") ? atoi(getenv("BLK_DEG")) : 51;
  G.n = n;
  G.nnz = (int64_t)n * (deg + 1);
  const float w = 1.0f / (deg + 1);
  G.rp.resize(n + 1);
  G.col.resize(G.nnz);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  auto rnd = [&] {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
  };
  for (int i = 0; i < n; ++i) {
    G.rp[i] = (int)((int64_t)i * (deg + 1));
    int* c = G.col.data() + G.rp[i];
    c[0] = i;
    for (int k = 1; k <= deg; ++k) c[k] = (int)(rnd() % n);
    std::sort(c, c + deg + 1);
  }
  G.rp[n] = (int)G.nnz;
  const int Wmax = 32;
  std::vector<float> zh((size_t)n * Wmax);
  for (auto& x : zh) x = (float)((int)(rnd() % 2001) - 1000) / 1000.0f;
  int *d_rp, *d_col;
  f4 *d_z, *d_y0, *d_y1;
  CHECK(hipMalloc(&d_rp, (n + 1) * 4));
  CHECK(hipMalloc(&d_col, G.nnz * 4));
  CHECK(hipMalloc(&d_z, (size_t)n * Wmax * 4));
  CHECK(hipMalloc(&d_y0, (size_t)n * Wmax * 4));
  CHECK(hipMalloc(&d_y1, (size_t)n * Wmax * 4));
  CHECK(hipMemcpy(d_rp, G.rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_col, G.col.data(), G.nnz * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_z, zh.data(), (size_t)n * Wmax * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("# one W-column fp32 slab: n = %d, %d uniform columns + the diagonal per row, nnz = %lld, %d CUs\n", n, deg,
         (long long)G.nnz, cus);
  printf("variant      W  block_rows  U  ms_per_pass  G_nonzeros_per_s  padding  max|diff|\n");
  std::vector<float> y0, y1;
  for (int ai = 1; ai < argc; ++ai) {
    int W = 16, br = 14, U = 2, em = 0;
    if (sscanf(argv[ai], "%d:%d:%d:%d", &W, &br, &U, &em) < 1) continue;
    const size_t ny = (size_t)n * W;
    y0.assign(ny, 0.0f);
    y1.assign(ny, 0.0f);
    float td = 0.0f;
    switch (W) {
      case 4: td = run_direct<1>(G, d_rp, d_col, d_z, d_y0, w, a, b); break;
      case 8: td = run_direct<2>(G, d_rp, d_col, d_z, d_y0, w, a, b); break;
      case 16: td = run_direct<4>(G, d_rp, d_col, d_z, d_y0, w, a, b); break;
      case 32: td = run_direct<8>(G, d_rp, d_col, d_z, d_y0, w, a, b); break;
      default: fprintf(stderr, "W must be 4, 8, 16 or 32\n"); return 1;
    }
    CHECK(hipMemcpy(y0.data(), d_y0, ny * 4, hipMemcpyDeviceToHost));
    printf("direct     %3d           -  -  %11.3f  %16.1f        -          -\n", W, td,
           G.nnz / (td * 1e6));
    fflush(stdout);
    if (br <= 0) continue;
    CHECK(hipMemset(d_y1, 0, ny * 4));
    double pad = 0.0;
    float t = 0.0f;
#define BLK(L, UU) t = em ? run_blk<L, UU, true>(G, br, d_z, d_y1, w, a, b, &pad, cus) \
                            : run_blk<L, UU, false>(G, br, d_z, d_y1, w, a, b, &pad, cus)
    if (W == 4) { if (U == 1) BLK(1, 1); else if (U == 2) BLK(1, 2); else BLK(1, 4); }
    if (W == 8) { if (U == 1) BLK(2, 1); else if (U == 2) BLK(2, 2); else BLK(2, 4); }
    if (W == 16) { if (U == 1) BLK(4, 1); else if (U == 2) BLK(4, 2); else BLK(4, 4); }
    if (W == 32) { if (U == 1) BLK(8, 1); else if (U == 2) BLK(8, 2); else BLK(8, 4); }
#undef BLK
    CHECK(hipMemcpy(y1.data(), d_y1, ny * 4, hipMemcpyDeviceToHost));
    double err = 0.0, mx = 0.0;
    for (size_t i = 0; i < ny; ++i) {
      err = std::max(err, (double)std::fabs(y0[i] - y1[i]));
      mx = std::max(mx, (double)std::fabs(y0[i]));
    }
    printf("%s %3d  %10d  %d  %11.3f  %16.1f  %6.1f %%  %.2e of %.2e\n",
           em ? "blocked-em" : "blocked   ", W, 1 << br, U, t, G.nnz / (t * 1e6), 100.0 * pad, err, mx);
    fflush(stdout);
  }
  return 0;
}
