// launch_probe.hip -- microbenchmark of the latency regime (small graphs).
// Not part of the library.
//
//   hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o tools/bin/launch_probe
//
// 1. Per-launch time of back-to-back dependent kernels, eager (host submission included) and
//    replayed from a captured hipGraph (device-side boundary only), by grid size.
// 2. Per-barrier time of a grid barrier inside one persistent launch (one chip-wide arrival
//    counter, agent-scope atomics, release/acquire fences; bounded spins).
// 3. A PubMed-sized APPNP K-loop (19,717 nodes, 44,324 undirected random edges + self loops,
//    F = 3, K = 10, one G = 4-lane group per row, 4 entries in flight): K captured launches
//    against ONE persistent launch whose iterations are separated by the grid barrier.
//    Both write the same Z (checked bitwise).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

typedef __attribute__((address_space(1))) unsigned gu32;

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 0;
}

hipStream_t g_stream;

template <typename F>
float time_us(F body, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) body();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a, g_stream));
  for (int i = 0; i < reps; ++i) body();
  CHECK(hipEventRecord(b, g_stream));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

// ---- grid barrier: one chip-wide arrival counter (agent-scope atomics), each workgroup waits
// until gen * gridDim.x arrivals.  Generations continue across launches (gen0 = barriers
// already passed), so nothing is reset between timed launches.  Bounded: a spin that runs out
// sets *fail (reported) instead of hanging.
__device__ __forceinline__ void grid_barrier(gu32* cnt, unsigned gen, gu32* fail) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains first
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = gen * gridDim.x;
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 16)) {
        __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__global__ void k_barriers(gu32* cnt, int n_bar, gu32* fail, unsigned gen0) {
  for (int i = 1; i <= n_bar; ++i) grid_barrier(cnt, gen0 + i, fail);
}

// ---- one APPNP iteration, G = 4 lanes per row (F = 3: lane 3 idle), 4 entries in flight
__device__ __forceinline__ void appnp_rows(const int* __restrict__ rp, const int* __restrict__ col,
                                           const float* __restrict__ val,
                                           const float* __restrict__ zin,
                                           const float* __restrict__ h, float* __restrict__ zout,
                                           int n, int f, float alpha, int row0, int stride) {
  const int sub = threadIdx.x >> 2, gl = threadIdx.x & 3;
  for (int row = row0 + sub; row < n; row += stride) {
    const int beg = rp[row], end = rp[row + 1];
    float acc = 0.0f;
    for (int e = beg; e < end; e += 4) {
      int c[4];
      float w[4], z[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[u] = e + u < end ? col[e + u] : 0;
        w[u] = e + u < end ? val[e + u] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) z[u] = (e + u < end && gl < f) ? zin[(int64_t)c[u] * 4 + gl] : 0.0f;
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = fmaf(w[u], z[u], acc);
    }
    if (gl < f) zout[(int64_t)row * 4 + gl] = fmaf(alpha, h[(int64_t)row * 4 + gl], (1.0f - alpha) * acc);
  }
}

__global__ __launch_bounds__(256) void k_step(const int* rp, const int* col, const float* val,
                                              const float* zin, const float* h, float* zout,
                                              int n, int f, float alpha) {
  appnp_rows(rp, col, val, zin, h, zout, n, f, alpha, blockIdx.x * 64, gridDim.x * 64);
}

__global__ __launch_bounds__(256) void k_loop(const int* rp, const int* col, const float* val,
                                              const float* h, float* z0, float* z1, int n, int f,
                                              float alpha, int K, gu32* cnt, gu32* fail,
                                              unsigned gen0) {
  const float* src = h;
  for (int k = 0; k < K; ++k) {
    float* dst = ((K - 1 - k) % 2 == 0) ? z0 : z1;
    appnp_rows(rp, col, val, src, h, dst, n, f, alpha, blockIdx.x * 64, gridDim.x * 64);
    if (k + 1 < K) grid_barrier(cnt, gen0 + k + 1, fail);
    src = dst;
  }
}

// ---- 4. persistent K-loop shaped for latency: each workgroup keeps ITS rows' CSR in LDS
// (iteration-invariant), every thread issues all the gathers of its rows before it sums them
// (one dependent round per iteration instead of row_ptr -> col -> gather), and Z crosses
// workgroups by write-through (sc1) stores and sc1 loads, so the barrier needs no fences:
// every storing wave drains (vmcnt 0), the workgroup barrier, one agent-scope arrival, a
// relaxed poll (MI355X_MICROARCH.md, valid forms, first row).
constexpr int kSlots = 8;  // entries per row issued together; longer rows finish in a loop
template <int J>           // rows per 4-lane group: 64 groups x J rows per block
__global__ __launch_bounds__(256) void k_loop_lds(const int* rp, const int* col, const float* val,
                                                  const float* h, float* z0, float* z1, int n,
                                                  int f, float alpha, int K, gu32* cnt,
                                                  gu32* fail, unsigned gen0) {
  extern __shared__ int lds_i[];
  constexpr int rows_per_block = 64 * J;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(n, r0 + rows_per_block);
  const int e0 = rp[r0], e1 = rp[r1];
  int* lrp = lds_i;                                   // rows_per_block + 1
  int* lcol = lds_i + rows_per_block + 1;             // entries of the block
  float* lval = reinterpret_cast<float*>(lcol + (e1 - e0));
  for (int i = threadIdx.x; i <= r1 - r0; i += 256) lrp[i] = rp[r0 + i] - e0;
  for (int e = threadIdx.x; e < e1 - e0; e += 256) {
    lcol[e] = col[e0 + e];
    lval[e] = val[e0 + e];
  }
  __syncthreads();
  const int sub = threadIdx.x >> 2, gl = threadIdx.x & 3;
  const bool on = gl < f;
  const float* src = h;
  for (int k = 0; k < K; ++k) {
    float* dst = ((K - 1 - k) % 2 == 0) ? z0 : z1;
    float v[J][kSlots];
    int b[J], e[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int lr = sub + 64 * j;
      const bool live = lr < r1 - r0 && on;
      b[j] = live ? lrp[lr] : 0;
      e[j] = live ? lrp[lr + 1] : 0;
#pragma unroll
      for (int t = 0; t < kSlots; ++t)
        v[j][t] = b[j] + t < e[j]
                      ? __hip_atomic_load(src + (int64_t)lcol[b[j] + t] * 4 + gl,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      float acc = 0.0f;
#pragma unroll
      for (int t = 0; t < kSlots; ++t)
        if (b[j] + t < e[j]) acc = fmaf(lval[b[j] + t], v[j][t], acc);
      for (int t = b[j] + kSlots; t < e[j]; ++t)
        acc = fmaf(lval[t],
                   __hip_atomic_load(src + (int64_t)lcol[t] * 4 + gl, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT),
                   acc);
      const int lr = sub + 64 * j;
      if (lr < r1 - r0 && on) {
        const int64_t o = (int64_t)(r0 + lr) * 4 + gl;
        __hip_atomic_store(dst + o, fmaf(alpha, h[o], (1.0f - alpha) * acc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (k + 1 < K) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
      __syncthreads();
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (gen0 + k + 1) * gridDim.x;
        unsigned spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1u << 16)) {
            __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __syncthreads();
    }
    src = dst;
  }
}

int main() {
  int* out;
  CHECK(hipMalloc(&out, 4096 * sizeof(int)));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  g_stream = s;

  printf("# 1. dependent empty kernels, per launch (us)\n");
  printf("blocks  eager  graph\n");
  const int chain = 200;
  for (int blocks : {1, 64, 256, 1024, 4096}) {
    auto launch = [&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, out); };
    const float eager = time_us(launch, chain);
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < chain; ++i) launch();
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const float graph = time_us([&] { CHECK(hipGraphLaunch(ge, s)); }, 20) / chain;
    printf("%6d  %5.2f  %5.2f\n", blocks, eager, graph);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }

  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned *cnt, *fail;
  CHECK(hipMalloc(&cnt, 64));
  CHECK(hipMalloc(&fail, 64));
  CHECK(hipMemset(fail, 0, 64));
  auto reset = [&] { CHECK(hipMemsetAsync(cnt, 0, 64, s)); };

  printf("# 2. grid barrier inside one launch (one chip counter), per barrier (us)\n");
  printf("grid  per_barrier\n");
  for (int grid : {cus / 4, cus, 2 * cus}) {
    const int nbar = 200;
    unsigned gen0 = 0;
    reset();
    const float t0 = time_us([&] {
      hipLaunchKernelGGL(k_barriers, dim3(grid), dim3(256), 0, s, (gu32*)cnt, 0, (gu32*)fail,
                         gen0);
    }, 20);
    const float t1 = time_us([&] {
      hipLaunchKernelGGL(k_barriers, dim3(grid), dim3(256), 0, s, (gu32*)cnt, nbar,
                         (gu32*)fail, gen0);
      gen0 += nbar;
    }, 20);
    printf("%4d  %6.2f\n", grid, (t1 - t0) / nbar);
  }

  // ---- 3. PubMed-sized K-loop
  const int n = 19717, m = 44324, f = 3, K = 10;
  const float alpha = 0.1f;
  std::vector<std::vector<int>> adj(n);
  uint64_t st = 88172645463325252ull;
  auto rnd = [&] {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return st;
  };
  for (int e = 0; e < m; ++e) {
    const int a = (int)(rnd() % n), b = (int)(rnd() % n);
    if (a == b) continue;
    adj[a].push_back(b);
    adj[b].push_back(a);
  }
  std::vector<int> rp(n + 1, 0), cl;
  std::vector<float> vl;
  std::vector<double> deg(n);
  for (int i = 0; i < n; ++i) {
    adj[i].push_back(i);
    std::sort(adj[i].begin(), adj[i].end());
    adj[i].erase(std::unique(adj[i].begin(), adj[i].end()), adj[i].end());
    deg[i] = (double)adj[i].size();
  }
  for (int i = 0; i < n; ++i) {
    for (int j : adj[i]) {
      cl.push_back(j);
      vl.push_back((float)(1.0 / std::sqrt(deg[i]) / std::sqrt(deg[j])));
    }
    rp[i + 1] = (int)cl.size();
  }
  std::vector<float> hh((size_t)n * 4, 0.0f);
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < f; ++c) hh[(size_t)i * 4 + c] = (float)((int)(rnd() % 2001) - 1000) / 1000.0f;
  int *d_rp, *d_col;
  float *d_val, *d_h, *z0, *z1, *w0, *w1;
  CHECK(hipMalloc(&d_rp, rp.size() * 4));
  CHECK(hipMalloc(&d_col, cl.size() * 4));
  CHECK(hipMalloc(&d_val, vl.size() * 4));
  CHECK(hipMalloc(&d_h, hh.size() * 4));
  for (float** p : {&z0, &z1, &w0, &w1}) {
    CHECK(hipMalloc(p, hh.size() * 4));
    CHECK(hipMemset(*p, 0, hh.size() * 4));
  }
  CHECK(hipMemcpy(d_rp, rp.data(), rp.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_col, cl.data(), cl.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_val, vl.data(), vl.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_h, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
  const int steps_grid = (n + 63) / 64;
  // K dependent launches, captured
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  const float* src = d_h;
  for (int k = 0; k < K; ++k) {
    float* dst = ((K - 1 - k) % 2 == 0) ? z0 : z1;
    hipLaunchKernelGGL(k_step, dim3(steps_grid), dim3(256), 0, s, d_rp, d_col, d_val, src, d_h,
                       dst, n, f, alpha);
    src = dst;
  }
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  const float t_launches = time_us([&] { CHECK(hipGraphLaunch(ge, s)); }, 200);
  printf("# 3. pubmed-sized APPNP, K = %d, F = %d, nnz = %zu\n", K, f, cl.size());
  printf("variant                         grid  us_per_propagation  us_per_iteration\n");
  printf("captured K launches            %5d  %18.2f  %16.2f\n", steps_grid, t_launches,
         t_launches / K);
  std::vector<float> ref(hh.size()), got(hh.size());
  CHECK(hipMemcpy(ref.data(), z0, ref.size() * 4, hipMemcpyDeviceToHost));
  for (int grid : {cus / 4, cus / 2, cus}) {
    unsigned gen0 = 0;
    reset();
    auto run = [&] {
      hipLaunchKernelGGL(k_loop, dim3(grid), dim3(256), 0, s, d_rp, d_col, d_val, d_h, w0, w1, n,
                         f, alpha, K, (gu32*)cnt, (gu32*)fail, gen0);
      gen0 += K - 1;
    };
    const float t = time_us(run, 200);
    CHECK(hipMemcpy(got.data(), w0, got.size() * 4, hipMemcpyDeviceToHost));
    const bool same = got == ref;
    printf("persistent launch + barriers   %5d  %18.2f  %16.2f  %s\n", grid, t, t / K,
           same ? "bitwise equal" : "MISMATCH");
  }
  // variant 4: CSR in LDS, all gathers of a thread's rows in flight, write-through hand-off
  auto variant4 = [&](auto kern, int J) {
    const int rows_per_block = 64 * J;
    const int grid4 = (n + rows_per_block - 1) / rows_per_block;
    int max_e = 0;
    for (int b = 0; b < grid4; ++b) {
      const int lo = b * rows_per_block, hi = std::min(n, lo + rows_per_block);
      max_e = std::max(max_e, rp[hi] - rp[lo]);
    }
    const size_t lds4 = (size_t)(rows_per_block + 1 + 2 * max_e) * 4;
    unsigned gen0 = 0;
    reset();
    CHECK(hipMemset(w0, 0, hh.size() * 4));
    auto run = [&] {
      hipLaunchKernelGGL(kern, dim3(grid4), dim3(256), lds4, s, d_rp, d_col, d_val, d_h, w0, w1,
                         n, f, alpha, K, (gu32*)cnt, (gu32*)fail, gen0);
      gen0 += K - 1;
    };
    const float t = time_us(run, 200);
    CHECK(hipMemcpy(got.data(), w0, got.size() * 4, hipMemcpyDeviceToHost));
    double err = 0.0;
    for (size_t i = 0; i < got.size(); ++i)
      err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    printf("LDS CSR + sc1, %d rows/group   %5d  %18.2f  %16.2f  max|diff| %.2e (LDS %zu B)\n", J,
           grid4, t, t / K, err, lds4);
  };
  variant4(k_loop_lds<1>, 1);
  variant4(k_loop_lds<2>, 2);
  variant4(k_loop_lds<4>, 4);
  variant4(k_loop_lds<8>, 8);
  unsigned hfail = 0;
  CHECK(hipMemcpy(&hfail, fail, 4, hipMemcpyDeviceToHost));
  printf("barrier spin give-ups: %u\n", hfail);
  return 0;
}
