// flat_probe.hip -- does a random gather of 384-B rows (3 lines: the split main part of an
// F = 100 fp32 row) run faster when every lane of a wave instruction carries a piece of some
// row (8 lines per instruction: 8 rows per 3 instructions, "flat") than with the SpMM kernel's
// mapping (32-lane groups of which 24 lanes are active: 2 rows = 6 lines per instruction)?
// Design input for k_step_wide.  Not part of the library.
//
//   hipcc -O3 --offload-arch=gfx950 tools/flat_probe.hip -o tools/bin/flat_probe
//   tools/bin/flat_probe [table_MB]
#include <hip/hip_runtime.h>

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

constexpr int kPieces = 24;  // 16-B pieces of a 384-B row

// the SpMM mapping: G = 32 lanes per row (24 active), 2 rows per instruction, U instructions in
// flight per wave
template <int U>
__global__ __launch_bounds__(256) void k_grouped(const float4* __restrict__ table,
                                                 const int* __restrict__ idx, int64_t n_idx,
                                                 float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int sub = lane / 32, gl = lane % 32;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t base = wave * 2 * U; base < n_idx; base += nw * 2 * U) {
    float4 z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + u * 2 + sub;
      z[u] = (gl < kPieces && e < n_idx) ? table[(int64_t)idx[e] * kPieces + gl]
                                         : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += z[u].x; acc.y += z[u].y; acc.z += z[u].z; acc.w += z[u].w;
    }
  }
  if (acc.x == 12345.f) sink[0] = acc.y + acc.z + acc.w;
}

// flat: 8 rows per group of 3 instructions, every lane active; lane l of instruction j takes
// piece (64 j + l) % 24 of row (64 j + l) / 24; U groups in flight per wave
template <int U>
__global__ __launch_bounds__(256) void k_flat(const float4* __restrict__ table,
                                              const int* __restrict__ idx, int64_t n_idx,
                                              float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t base = wave * 8 * U; base < n_idx; base += nw * 8 * U) {
    float4 z[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int p = 64 * j + lane;
        const int64_t e = base + u * 8 + p / kPieces;
        z[u][j] = e < n_idx ? table[(int64_t)idx[e] * kPieces + p % kPieces]
                            : make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        acc.x += z[u][j].x; acc.y += z[u][j].y; acc.z += z[u][j].z; acc.w += z[u][j].w;
      }
    }
  }
  if (acc.x == 12345.f) sink[0] = acc.y + acc.z + acc.w;
}

template <typename F>
float time_it(F launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) launch();
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t table_mb = argc > 1 ? atoll(argv[1]) : 940;
  const int64_t n_idx = 64ll << 20;  // 64 M row gathers = 192 M lines
  const int64_t rows = (table_mb << 20) / 384;
  int* idx;
  float4* table;
  float* sink;
  CHECK(hipMalloc(&idx, n_idx * 4));
  CHECK(hipMalloc(&table, rows * 384));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(table, 0, rows * 384));
  std::vector<int> h(n_idx);
  uint64_t s = 88172645463325252ull;
  for (int64_t i = 0; i < n_idx; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (int)(s % (uint64_t)rows);
  }
  CHECK(hipMemcpy(idx, h.data(), n_idx * 4, hipMemcpyHostToDevice));
  const double lines = (double)n_idx * 3;
  printf("# 384-B rows, %lld MB table, 64 M random rows (192 M lines), 256-thread blocks\n",
         (long long)table_mb);
  printf("mapping   U  blocks   ms     G_lines_s\n");
  for (int blocks : {2048, 8192}) {
#define RUN(KERNEL, U)                                                                         \
  {                                                                                            \
    const float ms = time_it([&] {                                                             \
      hipLaunchKernelGGL((KERNEL<U>), dim3(blocks), dim3(256), 0, 0, table, idx, n_idx, sink); \
    });                                                                                        \
    printf("%-8s %2d %6d %7.3f %8.1f\n", #KERNEL, U, blocks, ms, lines / (ms * 1e-3) / 1e9);   \
    fflush(stdout);                                                                            \
  }
    RUN(k_grouped, 2) RUN(k_grouped, 4) RUN(k_grouped, 8)
    RUN(k_flat, 1) RUN(k_flat, 2) RUN(k_flat, 3)
  }
  return 0;
}
