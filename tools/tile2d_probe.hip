// tile2d_probe.hip -- measured prototype of 2-D (destination tile x source block) tiling for
// the random-gather SpMM ("L2 blocking").  Not part of the library.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/tile2d_probe.hip -o tools/bin/tile2d_probe
//
// Workload: products-synth's shape on one 32-column fp32 slab of Z (128-B rows, one cache
// line each): n = 2,449,029 rows, 51 uniformly random columns + the diagonal per row
// (127.4 M nonzeros), Y = A Z with A's values 1/52.
//
// direct  a wavefront per destination row, 8 lanes per entry (one 128-B line), 8 entries per
//         wave instruction, two instructions in flight: one line request per nonzero, served
//         from the Infinity Cache / HBM (the library's k_step_wide shape for F = 32).
// tile2d  the 2-D pass: a persistent 1024-thread workgroup per CU; each wave owns a group of
//         80 destination rows whose 128-B sums stay in its LDS slice (16 x 80 x 128 B =
//         160 KiB) while it streams its entries source block by source block (blocks of
//         2^br rows of Z, 2^br x 128 B, meant to be L2-resident), 8 entries per chunk, two
//         chunks in flight; equal rows are combined by a segmented scan over the entry slots
//         and their tail adds into LDS.  The entries are regrouped on the host, each
//         (group, block) segment padded to whole chunks.  A line brought into an XCD's L2 is
//         reused only by the destination rows that XCD holds on chip at the time:
//         32 CUs x 1,280 rows x 51.5 / 2.45 M = 0.86 uses -- the prototype measures whether
//         the L2 turns that into any saving.
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
constexpr int kWaves = 16, kThreads = kWaves * 64, kRG = 80;  // 16 x 80 x 128 B = 160 KiB
constexpr uint32_t kNone = 0xffffffffu;

__device__ __forceinline__ f4 shfl_up4(f4 v, int d) {
  return f4{__shfl_up(v.x, d), __shfl_up(v.y, d), __shfl_up(v.z, d), __shfl_up(v.w, d)};
}
__device__ __forceinline__ f4 shfl_xor4(f4 v, int d) {
  return f4{__shfl_xor(v.x, d), __shfl_xor(v.y, d), __shfl_xor(v.z, d), __shfl_xor(v.w, d)};
}

__global__ __launch_bounds__(256) void k_direct(const int* __restrict__ rp,
                                                const int* __restrict__ col, float w,
                                                const f4* __restrict__ z, f4* __restrict__ y,
                                                int n) {
  const int lane = threadIdx.x & 63;
  const int e8 = lane >> 3, q = lane & 7;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += gridDim.x * 4) {
    const int beg = rp[row], end = rp[row + 1];
    f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int e = beg + e8; e < end; e += 16) {
      const int c0 = __builtin_nontemporal_load(col + e);
      const bool has1 = e + 8 < end;
      const int c1 = has1 ? __builtin_nontemporal_load(col + e + 8) : 0;
      const f4 a = z[(int64_t)c0 * 8 + q];
      const f4 b = has1 ? z[(int64_t)c1 * 8 + q] : f4{0.0f, 0.0f, 0.0f, 0.0f};
      acc += a + b;
    }
    for (int o = 8; o < 64; o <<= 1) acc += shfl_xor4(acc, o);
    if (lane < 8) y[(int64_t)row * 8 + q] = acc * w;
  }
}

template <int U>
__global__ __launch_bounds__(kThreads) void k_tile2d(const int* __restrict__ off,
                                                     const uint32_t* __restrict__ ent,
                                                     const int* __restrict__ cblk, int br_log2,
                                                     int nb, int slots, int passes, float w,
                                                     const f4* __restrict__ z,
                                                     f4* __restrict__ y, int n) {
  extern __shared__ f4 acc_all[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int e8 = lane >> 3, q = lane & 7;
  f4* acc = acc_all + wv * kRG * 8;
  for (int p = 0; p < passes; ++p) {
    const int64_t g = (int64_t)p * slots + (int64_t)blockIdx.x * kWaves + wv;
    const int64_t r0 = g * kRG;
    const int64_t left = n - r0;
    const int rows = left <= 0 ? 0 : (left < kRG ? (int)left : kRG);
    for (int i = lane; i < rows * 8; i += 64) acc[i] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const int c_end = off[(g + 1) * nb] / 8;
    for (int c = off[g * nb] / 8; c < c_end; c += U) {
      uint32_t en[U];
      int64_t cb[U];
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        en[u] = kNone;
        cb[u] = 0;
        if (c + u < c_end) {
          en[u] = ent[(int64_t)(c + u) * 8 + e8];
          cb[u] = (int64_t)cblk[c + u] << br_log2;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = en[u] != kNone ? z[(cb[u] + (en[u] & 0xfffffu)) * 8 + q] : f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (c + u >= c_end) break;
        const int row = (int)(en[u] >> 20);
        f4 s = v[u];
        for (int d = 8; d < 64; d <<= 1) {
          const f4 su = shfl_up4(s, d);
          const int ru = __shfl_up(row, d);
          if (lane >= d && ru == row) s += su;
        }
        const int rn = __shfl_down(row, 8);
        const bool tail = e8 == 7 || rn != row;
        if (en[u] != kNone && tail) acc[row * 8 + q] += s;
      }
    }
    for (int i = lane; i < rows * 8; i += 64) y[(r0 + i / 8) * 8 + (i & 7)] = acc[i] * w;
  }
}

int main() {
  const int n = 2449029, deg = 51;
  const int64_t nnz = (int64_t)n * (deg + 1);
  const float w = 1.0f / (deg + 1);
  // CSR: 51 uniform random columns + the diagonal per row, sorted
  std::vector<int> rp(n + 1), col(nnz);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  auto rnd = [&] {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return st;
  };
  for (int i = 0; i < n; ++i) {
    rp[i] = (int)((int64_t)i * (deg + 1));
    int* c = col.data() + rp[i];
    c[0] = i;
    for (int k = 1; k <= deg; ++k) c[k] = (int)(rnd() % n);
    std::sort(c, c + deg + 1);
  }
  rp[n] = (int)nnz;
  std::vector<float> zh((size_t)n * 32);
  for (auto& x : zh) x = (float)((int)(rnd() % 2001) - 1000) / 1000.0f;
  int *d_rp, *d_col;
  f4 *d_z, *d_y0, *d_y1;
  CHECK(hipMalloc(&d_rp, (n + 1) * 4));
  CHECK(hipMalloc(&d_col, nnz * 4));
  CHECK(hipMalloc(&d_z, (size_t)n * 128));
  CHECK(hipMalloc(&d_y0, (size_t)n * 128));
  CHECK(hipMalloc(&d_y1, (size_t)n * 128));
  CHECK(hipMemcpy(d_rp, rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_col, col.data(), nnz * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_z, zh.data(), (size_t)n * 128, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto time_ms = [&](auto body) {
    for (int i = 0; i < 2; ++i) body();
    CHECK(hipEventRecord(a));
    const int reps = 10;
    for (int i = 0; i < reps; ++i) body();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
  };
  const float t_direct = time_ms([&] {
    hipLaunchKernelGGL(k_direct, dim3((n + 3) / 4), dim3(256), 0, 0, d_rp, d_col, w, d_z, d_y0, n);
  });
  printf("# one 32-column fp32 slab of products-synth's shape: n = %d, nnz = %lld\n", n,
         (long long)nnz);
  printf("variant            block_rows  ms_per_pass  G_nonzeros_per_s  padding\n");
  printf("direct (1 line/nz)          -  %11.3f  %16.1f        -\n", t_direct,
         nnz / (t_direct * 1e6));
  std::vector<f4> y0((size_t)n * 8), y1((size_t)n * 8);
  CHECK(hipMemcpy(y0.data(), d_y0, (size_t)n * 128, hipMemcpyDeviceToHost));

  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int slots = cus * kWaves;
  const int passes = (int)((n + (int64_t)slots * kRG - 1) / ((int64_t)slots * kRG));
  const int64_t groups = (int64_t)passes * slots;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_tile2d<2>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  for (int br : {12, 13, 14, 15}) {
    const int nb = (n + (1 << br) - 1) >> br;
    std::vector<int64_t> cnt(groups * nb, 0);
    for (int64_t g = 0; g < groups; ++g)
      for (int64_t i = g * kRG; i < std::min<int64_t>(n, g * kRG + kRG); ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e) ++cnt[g * nb + (col[e] >> br)];
    std::vector<int> off(groups * nb + 1, 0);
    int64_t tot = 0;
    for (int64_t s = 0; s < groups * nb; ++s) {
      off[s] = (int)tot;
      tot += (cnt[s] + 7) / 8 * 8;
    }
    off[groups * nb] = (int)tot;
    std::vector<uint32_t> ent(tot, kNone);
    std::vector<int> cblk(tot / 8);
    std::vector<int> cur(off.begin(), off.end() - 1);
    for (int64_t g = 0; g < groups; ++g)
      for (int64_t i = g * kRG; i < std::min<int64_t>(n, g * kRG + kRG); ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e) {
          const int bb = col[e] >> br;
          ent[cur[g * nb + bb]++] =
              ((uint32_t)(i - g * kRG) << 20) | (uint32_t)(col[e] & ((1 << br) - 1));
        }
    for (int64_t s = 0; s < groups * nb; ++s)
      for (int c = off[s] / 8; c < off[s + 1] / 8; ++c) cblk[c] = (int)(s % nb);
    int *d_off, *d_cblk;
    uint32_t* d_ent;
    CHECK(hipMalloc(&d_off, off.size() * 4));
    CHECK(hipMalloc(&d_ent, tot * 4));
    CHECK(hipMalloc(&d_cblk, cblk.size() * 4));
    CHECK(hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_ent, ent.data(), tot * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_cblk, cblk.data(), cblk.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(d_y1, 0, (size_t)n * 128));
    const float t = time_ms([&] {
      hipLaunchKernelGGL(k_tile2d<2>, dim3(cus), dim3(kThreads), 160 * 1024, 0, d_off, d_ent,
                         d_cblk, br, nb, slots, passes, w, d_z, d_y1, n);
    });
    CHECK(hipMemcpy(y1.data(), d_y1, (size_t)n * 128, hipMemcpyDeviceToHost));
    double err = 0.0, mx = 0.0;
    for (size_t i = 0; i < y0.size(); ++i)
      for (int k = 0; k < 4; ++k) {
        err = std::max(err, (double)std::fabs(y0[i][k] - y1[i][k]));
        mx = std::max(mx, (double)std::fabs(y0[i][k]));
      }
    printf("tile2d (LDS acc)   %10d  %11.3f  %16.1f  %6.1f %%   max|diff| %.2e of %.2e\n",
           1 << br, t, nnz / (t * 1e6), 100.0 * (tot - nnz) / nnz, err, mx);
    CHECK(hipFree(d_off));
    CHECK(hipFree(d_ent));
    CHECK(hipFree(d_cblk));
  }
  return 0;
}
