// launch_probe.hip -- microbenchmark: per-launch floor of back-to-back dependent kernels on
// MI355X (empty kernels, and kernels with a chain of D dependent global loads), by grid size.
// Design input for the latency regime of the APPNP step (small graphs).  Not part of the library.
//
//   hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o tools/bin/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 0;
}

// D dependent loads per thread through a pointer-chasing table (next = tab[cur]), then a store
template <int D>
__global__ __launch_bounds__(256) void k_chain(const int* __restrict__ tab, int* __restrict__ out,
                                               int n) {
  int i = (blockIdx.x * 256 + threadIdx.x) % n;
#pragma unroll
  for (int d = 0; d < D; ++d) i = tab[i];
  out[blockIdx.x * 256 + threadIdx.x] = i;
}

template <typename F>
float per_launch_us(F launch, int reps = 200) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) launch();
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

int main() {
  const int n = 1 << 20;
  int *tab, *out;
  CHECK(hipMalloc(&tab, n * sizeof(int)));
  CHECK(hipMalloc(&out, 4096 * 256 * sizeof(int)));
  int* h = (int*)malloc(n * sizeof(int));
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (int)(s % n);
  }
  CHECK(hipMemcpy(tab, h, n * sizeof(int), hipMemcpyHostToDevice));
  printf("blocks  empty_us  chain1_us  chain2_us  chain4_us  chain8_us\n");
  for (int blocks : {1, 64, 256, 1024, 4096}) {
    float e = per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, 0, out); });
    float c1 = per_launch_us([&] { hipLaunchKernelGGL(k_chain<1>, dim3(blocks), dim3(256), 0, 0, tab, out, n); });
    float c2 = per_launch_us([&] { hipLaunchKernelGGL(k_chain<2>, dim3(blocks), dim3(256), 0, 0, tab, out, n); });
    float c4 = per_launch_us([&] { hipLaunchKernelGGL(k_chain<4>, dim3(blocks), dim3(256), 0, 0, tab, out, n); });
    float c8 = per_launch_us([&] { hipLaunchKernelGGL(k_chain<8>, dim3(blocks), dim3(256), 0, 0, tab, out, n); });
    printf("%6d  %8.2f  %9.2f  %9.2f  %9.2f  %9.2f\n", blocks, e, c1, c2, c4, c8);
  }
  return 0;
}
