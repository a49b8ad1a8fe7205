// xcd_probe.hip -- round-5 measurement probe, not part of the library: the chip's random-line
// rate when only some XCDs issue the gathers.  Question: could the remainder pass run on ONE
// XCD (its L2 private to it) concurrently with the main SpMM on the other seven, or does the
// main SpMM need every XCD to reach the fabric's random-line rate?
//
// k_lines: random 128-B lines of a table (8 lanes x 16 B per line, 8 lines per wave
// instruction, 8 instructions in flight: the library's appnp_line_rate_probe shape).  Every
// workgroup reads its XCD (s_getreg XCC_ID); a workgroup on an XCD outside `mask` exits at once,
// the others claim chunks of requests from a device counter until all are taken, so the same
// number of lines is gathered whatever the mask.  Optionally a second kernel, k_l2, runs
// concurrently on another stream: gathers confined to a small (L2-resident) table by the
// workgroups of the XCDs in its own mask -- the remainder pass's shape.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/xcd_probe.hip -o tools/bin/xcd_probe
//   tools/bin/xcd_probe [table_MB]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int kChunk = 1 << 14;  // requests per claim

// gather `requests` random lines of table[n_lines * 8] (f4 units), chunks claimed from ctr[0]
__global__ __launch_bounds__(256) void k_lines(const f4* __restrict__ table, uint32_t n_lines,
                                               int64_t requests, uint32_t mask, uint64_t seed,
                                               unsigned long long* ctr, float* sink) {
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;
  if (!((mask >> xcc) & 1u)) return;
  __shared__ long long chunk;
  const int lane = threadIdx.x & 63, sub = lane / 8, gl = lane % 8, w = threadIdx.x >> 6;
  f4 acc = {0, 0, 0, 0};
  for (;;) {
    if (threadIdx.x == 0) chunk = (long long)atomicAdd(ctr, 1ull);
    __syncthreads();
    const int64_t c0 = chunk * kChunk;
    __syncthreads();
    if (c0 >= requests) break;
    // 4 waves x 8 lines x 8 in flight = 256 lines per round
    for (int64_t base = c0 + w * 64; base < c0 + kChunk && base < requests; base += 256) {
      f4 z[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint64_t e = (uint64_t)(base + u * 8 + sub);
        const uint32_t h = (uint32_t)mix(seed + e);
        const uint32_t line = __umulhi(h, n_lines);
        z[u] = table[(int64_t)line * 8 + gl];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += z[u];
    }
  }
  if (acc.x == 1.2345e-30f) sink[0] = acc.y;
}

// gather `requests` random ROWS of 3 lines (384 B, the main SpMM's 96 columns) from
// table[n_rows * 24] (f4 units): 32 lanes per row, 24 active (the SpMM's lane mapping), 2 rows
// per wave instruction, U rows in flight per sub-group; all XCDs
template <int U>
__global__ __launch_bounds__(256) void k_rows3(const f4* __restrict__ table, uint32_t n_rows,
                                               int64_t requests, uint64_t seed,
                                               unsigned long long* ctr, float* sink) {
  __shared__ long long chunk;
  const int lane = threadIdx.x & 63, sub = lane / 32, gl = lane % 32, w = threadIdx.x >> 6;
  f4 acc = {0, 0, 0, 0};
  for (;;) {
    if (threadIdx.x == 0) chunk = (long long)atomicAdd(ctr, 1ull);
    __syncthreads();
    const int64_t c0 = chunk * (kChunk / 4);
    __syncthreads();
    if (c0 >= requests) break;
    for (int64_t base = c0 + w * 2 * U; base < c0 + kChunk / 4 && base < requests;
         base += 4 * 2 * U) {
      f4 z[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t e = (uint64_t)(base + u * 2 + sub);
        const uint32_t h = (uint32_t)mix(seed + e);
        const uint32_t r = __umulhi(h, n_rows);
        z[u] = gl < 24 ? table[(int64_t)r * 24 + gl] : f4{0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += z[u];
    }
  }
  if (acc.x == 1.2345e-30f) sink[0] = acc.y;
}

template <int U>
void run_rows3(const f4* table, uint32_t n_rows, unsigned long long* ctr, float* sink,
               hipStream_t s, hipEvent_t a, hipEvent_t b) {
  const int64_t rows = 1ll << 27;  // 3 x 2^27 lines
  for (int rep = 0; rep < 2; ++rep) {
    CHECK(hipMemset(ctr, 0, sizeof(unsigned long long)));
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_rows3<U>, dim3(2048), dim3(256), 0, s, table, n_rows, rows,
                       99ull + rep, ctr, sink);
    CHECK(hipEventRecord(b, s));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (rep == 1)
      printf("384-B rows, %d rows in flight per sub-group %9.3f ms %8.2f G lines/s\n", U, ms,
             3.0 * rows / (ms * 1e-3) / 1e9);
  }
}

int main(int argc, char** argv) {
  const int64_t table_mb = argc > 1 ? atoll(argv[1]) : 940;
  const uint32_t n_lines = (uint32_t)(table_mb * (1 << 20) / 128);
  const int64_t requests = 1ll << 29;
  f4* table;
  float* sink;
  f4* small;
  unsigned long long* ctr;
  CHECK(hipMalloc(&table, (size_t)n_lines * 128));
  CHECK(hipMemset(table, 0, (size_t)n_lines * 128));
  CHECK(hipMalloc(&small, 1 << 20));  // 1 MB: L2-resident
  CHECK(hipMemset(small, 0, 1 << 20));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMalloc(&ctr, 2 * sizeof(unsigned long long)));
  hipStream_t s0, s1;
  CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t a, b, c, d;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventCreate(&c));
  CHECK(hipEventCreate(&d));
  const unsigned grid = 256 * 8;  // 8 workgroups of 4 waves per CU
  printf("table %lld MB, %lld random 128-B lines per run\n", (long long)table_mb,
         (long long)requests);
  printf("%-34s %9s %12s %12s\n", "case", "ms", "G lines/s", "L2 kernel ms");
  struct Case { const char* name; uint32_t mask; uint32_t l2mask; int64_t l2req; };
  const Case cases[] = {
      {"all 8 XCDs", 0xff, 0, 0},
      {"7 XCDs (not 0)", 0xfe, 0, 0},
      {"6 XCDs", 0xfc, 0, 0},
      {"4 XCDs", 0xf0, 0, 0},
      {"1 XCD", 0x01, 0, 0},
      {"L2 table alone, XCD 0", 0, 0x01, 1ll << 27},
      {"L2 table alone, all XCDs", 0, 0xff, 1ll << 27},
      {"7 XCDs + L2 table on XCD 0", 0xfe, 0x01, 1ll << 27},
      {"8 XCDs + L2 table on all", 0xff, 0xff, 1ll << 27},
      {"all 8 XCDs (again)", 0xff, 0, 0},
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (const Case& k : cases) {
      CHECK(hipMemset(ctr, 0, 2 * sizeof(unsigned long long)));
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a, s0));
      CHECK(hipEventRecord(c, s1));
      if (k.mask)
        hipLaunchKernelGGL(k_lines, dim3(grid), dim3(256), 0, s0, table, n_lines, requests,
                           k.mask, 12345ull + rep, ctr, sink);
      if (k.l2mask)
        hipLaunchKernelGGL(k_lines, dim3(grid), dim3(256), 0, s1, small, 1u << 13, k.l2req,
                           k.l2mask, 777ull + rep, ctr + 1, sink);
      CHECK(hipEventRecord(b, s0));
      CHECK(hipEventRecord(d, s1));
      CHECK(hipDeviceSynchronize());
      float ms = 0, ms2 = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      CHECK(hipEventElapsedTime(&ms2, c, d));
      if (rep == 1)
        printf("%-34s %9.3f %12.2f %12.3f\n", k.name, k.mask ? ms : 0.0,
               k.mask ? requests / (ms * 1e-3) / 1e9 : 0.0, k.l2mask ? ms2 : 0.0);
    }
  }
  // the main SpMM's row shape: 3 consecutive lines per random row, 24 of 32 lanes
  const uint32_t n_rows = (uint32_t)((size_t)n_lines * 128 / 384);
  run_rows3<1>(table, n_rows, ctr, sink, s0, a, b);
  run_rows3<2>(table, n_rows, ctr, sink, s0, a, b);
  run_rows3<4>(table, n_rows, ctr, sink, s0, a, b);
  run_rows3<8>(table, n_rows, ctr, sink, s0, a, b);
  return 0;
}
