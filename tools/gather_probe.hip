// gather_probe.hip -- microbenchmark: random row-gather throughput on MI355X vs table size and
// row size (where the rows are served from: L2 / Infinity Cache / HBM).  Design input for the
// APPNP SpMM (its cost is dominated by gathers of Z rows).  Not part of the library.
//
//   hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o tools/bin/gather_probe
//   tools/bin/gather_probe
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

// G lanes x 16 B per row; 64/G rows per wave instruction; U instructions in flight.
template <int G, int U, bool NT>
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ table, int64_t ld4,
                                                int lanes_used, const int* __restrict__ idx,
                                                int64_t n_idx, float* __restrict__ sink) {
  constexpr int P = 64 / G;
  const int lane = threadIdx.x & 63;
  const int sub = lane / G, gl = lane % G;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float4 acc = make_float4(0, 0, 0, 0);
  const bool act = gl < lanes_used;
  for (int64_t base = wave * P * U; base < n_idx; base += nw * P * U) {
    float4 z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + u * P + sub;
      if (act && e < n_idx) {
        const int r = idx[e];
        const float4* p = table + (int64_t)r * ld4 + gl;
        typedef float f4 __attribute__((ext_vector_type(4)));
        if (NT) {
          const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
          z[u] = make_float4(t.x, t.y, t.z, t.w);
        } else {
          z[u] = *p;
        }
      } else {
        z[u] = make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += z[u].x; acc.y += z[u].y; acc.z += z[u].z; acc.w += z[u].w;
    }
  }
  if (acc.x == 12345.f) sink[0] = acc.y + acc.z + acc.w;
}

template <int G, bool NT>
float run(const float4* table, int64_t ld4, int lanes, const int* idx, int64_t n_idx, float* sink,
          int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((k_gather<G, 8, NT>), dim3(blocks), dim3(256), 0, 0, table, ld4, lanes, idx,
                       n_idx, sink);
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_gather<G, 8, NT>), dim3(blocks), dim3(256), 0, 0, table, ld4, lanes, idx,
                       n_idx, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t n_idx = 64ll << 20;  // 64M gathers
  int blocks = argc > 1 ? atoi(argv[1]) : 2048;
  int* idx;
  float4* table;
  float* sink;
  const int64_t max_table = 4ll << 30;
  CHECK(hipMalloc(&idx, n_idx * 4));
  CHECK(hipMalloc(&table, max_table));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(table, 0, max_table));
  std::vector<int> h(n_idx);
  const int64_t table_mb[] = {16, 64, 128, 192, 256, 384, 1024, 4096};
  const int row_bytes[] = {64, 128, 256, 384, 400, 512};
  printf("table_MB row_B  ms   gathered_GB/s  (nt: the same with non-temporal loads)\n");
  uint64_t s = 88172645463325252ull;
  for (int rb : row_bytes) {
    for (int64_t tmb : table_mb) {
      const int64_t ld_bytes = rb;  // dense rows
      const int64_t rows = (tmb << 20) / ld_bytes;
      if (rows <= 0) continue;
      for (int64_t i = 0; i < n_idx; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = (int)(s % (uint64_t)rows);
      }
      CHECK(hipMemcpy(idx, h.data(), n_idx * 4, hipMemcpyHostToDevice));
      const int lanes = rb / 16;
      const int64_t ld4 = rb / 16;
      float ms = 0, ms_nt = 0;
      switch (rb) {
        case 64: ms = run<4, false>(table, ld4, lanes, idx, n_idx, sink, blocks);
                 ms_nt = run<4, true>(table, ld4, lanes, idx, n_idx, sink, blocks); break;
        case 128: ms = run<8, false>(table, ld4, lanes, idx, n_idx, sink, blocks);
                  ms_nt = run<8, true>(table, ld4, lanes, idx, n_idx, sink, blocks); break;
        case 256: ms = run<16, false>(table, ld4, lanes, idx, n_idx, sink, blocks);
                  ms_nt = run<16, true>(table, ld4, lanes, idx, n_idx, sink, blocks); break;
        case 384: ms = run<32, false>(table, ld4, lanes, idx, n_idx, sink, blocks);
                  ms_nt = run<32, true>(table, ld4, lanes, idx, n_idx, sink, blocks); break;
        case 400: ms = run<32, false>(table, ld4, lanes, idx, n_idx, sink, blocks);
                  ms_nt = run<32, true>(table, ld4, lanes, idx, n_idx, sink, blocks); break;
        case 512: ms = run<32, false>(table, ld4, lanes, idx, n_idx, sink, blocks);
                  ms_nt = run<32, true>(table, ld4, lanes, idx, n_idx, sink, blocks); break;
      }
      const double gb = (double)n_idx * rb / 1e9;
      printf("%6lld %5d %7.3f %8.0f  (nt %8.0f)\n", (long long)tmb, rb, ms, gb / (ms * 1e-3),
             gb / (ms_nt * 1e-3));
      fflush(stdout);
    }
  }
  return 0;
}
