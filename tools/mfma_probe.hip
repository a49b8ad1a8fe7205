// mfma_probe.hip -- measured prototype, not part of the library: a source-blocked pass over a
// 16-column fp32 slab whose destination sums live in MFMA accumulator tiles instead of LDS.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mfma_probe.hip -o tools/bin/mfma_probe
//   [BLK_N=n BLK_DEG=d] tools/bin/mfma_probe T:WPC:U:br [...]
//      T = 16-row tiles per wave, WPC = waves per CU, U = quads in flight, br = log2 source
//      rows per block
//
// Why (profiles/r2_blk_probe.txt): the LDS-accumulator pass (blk_probe
// k_blk, W = 16) needs 4 row passes on products-synth (160 KB of LDS per CU holds 2,400 rows of
// 64 B), and every row pass re-fetches the whole [n, 16] table into every XCD's L2: 1.89 ms
// per pass against 0.68 ms for the one-pass W = 4 form.  The register file is 3.2x the LDS
// (512 KB per CU), but a segmented-scan tail lane cannot add into another lane's register.
// An MFMA can: C[16 x 16] += A[16 x 4] B[4 x 16] with A the one-hot row selector of 4 entries
// (A[i][k] = (row_k == i)) and B their gathered rows adds each entry's row into its tile row
// -- v_mfma_f32_16x16x4_f32 is bitwise a k-ordered fmaf chain (cdna_hip_programming.md 3), so
// a one-hot A gives exact sequential fp32 adds.  The tile is wave-uniform (one scalar switch
// per quad of entries), the accumulators stay in registers for the whole sweep, and 12 waves
// per CU x 32 tiles x 16 rows cover 1.57 M rows per pass: 2 passes on products-synth.
//
// Layout: per wave group (T tiles = 16 T destination rows), per source block, per tile: its
// entries padded to a multiple of 4 (a quad).  Entry word: tile (6 bits) << 26 | row in tile
// (4 bits) << 22 | global source column (22 bits; all ones = padding).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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
constexpr uint32_t kPadCol = 0x3fffffu;
constexpr uint32_t kPad = kPadCol;

// direct gather (blk_probe k_direct<4>): a wavefront per row, 4 lanes per entry
__global__ __launch_bounds__(256) void k_direct(const int* __restrict__ rp,
                                                const int* __restrict__ col, float w,
                                                const f4* __restrict__ z, f4* __restrict__ y,
                                                int n) {
  constexpr int LPE = 4, CH = 16;
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

template <int T>
struct Acc {
  f4 t[T];
};

// acc.t[tile] = mfma(a, b, acc.t[tile]) with a compile-time register set per leaf: a binary
// search on the wave-uniform tile (scalar branches), log2 T levels
template <int T, int LO, int HI>
__device__ __forceinline__ void mfma_into(Acc<T>& acc, int tile, float a, float b) {
  if constexpr (HI - LO == 1) {
    acc.t[LO] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc.t[LO], 0, 0, 0);
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (tile < MID)
      mfma_into<T, LO, MID>(acc, tile, a, b);
    else
      mfma_into<T, MID, HI>(acc, tile, a, b);
  }
}

template <int T, int U, int WPC>
__global__ __launch_bounds__(WPC * 64) void k_mfma(const int* __restrict__ qoff,
                                                    const uint32_t* __restrict__ ent,
                                                    const float* __restrict__ z,
                                                    float* __restrict__ y, int n, int slots,
                                                    int passes, float w) {
  const int lane = threadIdx.x & 63;
  const int k = lane >> 4, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int R = 16 * T;
  for (int p = 0; p < passes; ++p) {
    const int g = p * slots + (int)blockIdx.x * WPC + wv;
    Acc<T> acc;
#pragma unroll
    for (int t = 0; t < T; ++t) acc.t[t] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const int q0 = qoff[g], q1 = qoff[g + 1];
    uint32_t e[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      e[u] = q0 + u < q1 ? __builtin_nontemporal_load(ent + (q0 + u) * 4 + k) : kPad;
    for (int q = q0; q < q1; q += U) {
      float b[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t c = e[u] & kPadCol;
        b[u] = c == kPadCol ? 0.0f : z[(int)c * 16 + j];
      }
      uint32_t en[U];  // the next round's entries, in flight under this round's gathers
#pragma unroll
      for (int u = 0; u < U; ++u)
        en[u] = q + U + u < q1 ? __builtin_nontemporal_load(ent + (q + U + u) * 4 + k) : kPad;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (q + u >= q1) break;
        const int tile = __builtin_amdgcn_readfirstlane((int)(e[u] >> 26));
        const float a = (int)((e[u] >> 22) & 15u) == j && (e[u] & kPadCol) != kPadCol ? 1.0f
                                                                                    : 0.0f;
        mfma_into<T, 0, T>(acc, tile, a, b[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) e[u] = en[u];
    }
    // C layout: lane holds C[4 k + r][j], r = 0..3
    const int rbase = g * R + 4 * k;
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + 16 * t + r;
        if (row < n) y[row * 16 + j] = acc.t[t][r] * w;
      }
    }
  }
}

struct Graph {
  int n;
  int64_t nnz;
  std::vector<int> rp, col;
};

float run_direct(const Graph& G, const int* d_rp, const int* d_col, const f4* d_z, f4* d_y,
                 float w, hipEvent_t a, hipEvent_t b) {
  const int n = G.n;
  auto body = [&] {
    hipLaunchKernelGGL(k_direct, dim3((n + 3) / 4), dim3(256), 0, 0, d_rp, d_col, w, d_z, d_y,
                       n);
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

template <int T, int U, int WPC>
float run_mfma(const Graph& G, int br, const float* d_z, float* d_y, float w,
               hipEvent_t a, hipEvent_t b, double* pad, int cus, int* passes_out) {
  const int n = G.n;
  const int R = 16 * T;
  const int wpc = WPC;
  const int slots = cus * wpc;
  const int passes = (int)((n + (int64_t)slots * R - 1) / ((int64_t)slots * R));
  const int64_t groups = (int64_t)passes * slots;
  const int nb = (n + (1 << br) - 1) >> br;
  // count entries per (group, block, tile)
  std::vector<int> qoff(groups + 1, 0);
  std::vector<std::vector<int>> cnt(1);
  int64_t tot_q = 0;
  std::vector<int> c(nb * T);
  std::vector<uint32_t> ent;
  ent.reserve((size_t)(G.nnz * 1.2));
  std::vector<std::vector<uint32_t>> bucket(nb * T);
  for (int64_t g = 0; g < groups; ++g) {
    qoff[g] = (int)tot_q;
    for (auto& v : bucket) v.clear();
    const int64_t r0 = g * R, r1 = std::min<int64_t>(n, r0 + R);
    for (int64_t i = r0; i < r1; ++i) {
      const int t = (int)((i - r0) / 16), r = (int)((i - r0) % 16);
      for (int e = G.rp[i]; e < G.rp[i + 1]; ++e) {
        const int cc = G.col[e];
        bucket[(cc >> br) * T + t].push_back(((uint32_t)t << 26) | ((uint32_t)r << 22) |
                                             (uint32_t)cc);
      }
    }
    for (int bl = 0; bl < nb; ++bl)
      for (int t = 0; t < T; ++t) {
        auto& v = bucket[bl * T + t];
        if (v.empty()) continue;
        for (auto x : v) ent.push_back(x);
        while (v.size() % 4) {
          v.push_back(0);
          ent.push_back(((uint32_t)t << 26) | kPadCol);
        }
        tot_q += (int64_t)v.size() / 4;
      }
  }
  qoff[groups] = (int)tot_q;
  *pad = (double)(tot_q * 4 - G.nnz) / G.nnz;
  int* d_qoff;
  uint32_t* d_ent;
  CHECK(hipMalloc(&d_qoff, qoff.size() * 4));
  CHECK(hipMalloc(&d_ent, std::max<size_t>(4, ent.size() * 4)));
  CHECK(hipMemcpy(d_qoff, qoff.data(), qoff.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice));
  auto body = [&] {
    hipLaunchKernelGGL((k_mfma<T, U, WPC>), dim3(cus), dim3(wpc * 64), 0, 0, d_qoff, d_ent,
                       d_z, d_y, n, slots, passes, w);
  };
  for (int i = 0; i < 2; ++i) body();
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) body();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipFree(d_qoff));
  CHECK(hipFree(d_ent));
  *passes_out = passes;
  return ms / 10;
}

int main(int argc, char** argv) {
  Graph G;
  const int n = getenv("BLK_N") ? atoi(getenv("BLK_N")) : 2449029;
  const int deg = getenv("BLK_DEG") ? atoi(getenv("BLK_DEG")) : 51;
  if (n >= (1 << 22)) {
    fprintf(stderr, "n must be < 2^22 (22-bit columns)\n");
    return 1;
  }
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
    int* cc = G.col.data() + G.rp[i];
    cc[0] = i;
    for (int kk = 1; kk <= deg; ++kk) cc[kk] = (int)(rnd() % n);
    std::sort(cc, cc + deg + 1);
  }
  G.rp[n] = (int)G.nnz;
  std::vector<float> zh((size_t)n * 16);
  for (auto& x : zh) x = (float)((int)(rnd() % 2001) - 1000) / 1000.0f;
  int *d_rp, *d_col;
  float *d_z, *d_y0, *d_y1;
  CHECK(hipMalloc(&d_rp, (n + 1) * 4));
  CHECK(hipMalloc(&d_col, G.nnz * 4));
  CHECK(hipMalloc(&d_z, (size_t)n * 16 * 4));
  CHECK(hipMalloc(&d_y0, (size_t)n * 16 * 4));
  CHECK(hipMalloc(&d_y1, (size_t)n * 16 * 4));
  CHECK(hipMemcpy(d_rp, G.rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_col, G.col.data(), G.nnz * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_z, zh.data(), (size_t)n * 16 * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("# one 16-column fp32 slab: n = %d, %d uniform columns + the diagonal per row, nnz = "
         "%lld, %d CUs\n", n, deg, (long long)G.nnz, cus);
  const size_t ny = (size_t)n * 16;
  std::vector<float> y0(ny), y1(ny);
  const float td = run_direct(G, d_rp, d_col, reinterpret_cast<const f4*>(d_z),
                              reinterpret_cast<f4*>(d_y0), w, a, b);
  CHECK(hipMemcpy(y0.data(), d_y0, ny * 4, hipMemcpyDeviceToHost));
  printf("direct (a wavefront per row, 4 lanes per entry): %.3f ms\n", td);
  printf("variant  T  WPC  U  block_rows  passes  ms_per_pass_total  padding  max|diff|\n");
  fflush(stdout);
  for (int ai = 1; ai < argc; ++ai) {
    int T = 32, wpc = 12, U = 8, br = 15;
    if (sscanf(argv[ai], "%d:%d:%d:%d", &T, &wpc, &U, &br) < 1) continue;
    CHECK(hipMemset(d_y1, 0, ny * 4));
    double pad = 0.0;
    float t = 0.0f;
    int passes = 0;
#define RUN(TT, UU, WW) t = run_mfma<TT, UU, WW>(G, br, d_z, d_y1, w, a, b, &pad, cus, &passes)
    if (T == 32 && U == 8 && wpc == 12) RUN(32, 8, 12);
    else if (T == 32 && U == 4 && wpc == 12) RUN(32, 4, 12);
    else if (T == 40 && U == 8 && wpc == 8) RUN(40, 8, 8);
    else if (T == 40 && U == 16 && wpc == 8) RUN(40, 16, 8);
    else if (T == 20 && U == 8 && wpc == 16) RUN(20, 8, 16);
    else if (T == 20 && U == 4 && wpc == 16) RUN(20, 4, 16);
    else if (T == 16 && U == 4 && wpc == 16) RUN(16, 4, 16);
    else if (T == 16 && U == 8 && wpc == 16) RUN(16, 8, 16);
    else {
      fprintf(stderr, "unsupported T:WPC:U %d:%d:%d\n", T, wpc, U);
      continue;
    }
#undef RUN
    CHECK(hipMemcpy(y1.data(), d_y1, ny * 4, hipMemcpyDeviceToHost));
    double err = 0.0, mx = 0.0;
    for (size_t i = 0; i < ny; ++i) {
      err = std::max(err, (double)std::fabs(y0[i] - y1[i]));
      mx = std::max(mx, (double)std::fabs(y0[i]));
    }
    printf("mfma    %2d  %3d  %2d  %10d  %6d  %17.3f  %6.1f %%  %.2e of %.2e\n", T, wpc, U,
           1 << br, passes, t, 100.0 * pad, err, mx);
    fflush(stdout);
  }
  return 0;
}
