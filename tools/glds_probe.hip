// glds_probe.hip -- measured question: do LDS-DMA gathers (global_load_lds_dwordx4) of random
// 384-B rows from a ~1 GB table (the split main part of products-synth: 2.45 M rows x 96 fp32)
// move more bytes per second than the register gathers the SpMM uses?  Not part of the library.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/glds_probe.hip -o tools/bin/glds_probe
//
// reg   a wave gathers 2 rows per instruction (24 lanes x 16 B each, 16 lanes idle), U
//       instructions in flight, into registers (tools/gather_probe.hip's shape for 384-B rows).
// glds  a wave gathers 8 rows = 3 KB = 3 wave-instructions of global_load_lds_dwordx4 (1 KB
//       each, lane l of instruction i moves bytes i*1024 + 16 l of the 8-row slot) into a ring
//       of S slots in LDS; the 8 row indices of a slot come in by one scalar load (lgkm counter),
//       so the DMAs are the only vector-memory instructions and a counted vmcnt(3 (S - 1))
//       keeps S - 1 slots in flight while the oldest is summed from LDS.
#include <hip/hip_runtime.h>

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
constexpr int kRowB = 384, kRowF4 = kRowB / 16;  // 24 pieces of 16 B per row

template <int U>
__global__ __launch_bounds__(256) void k_reg(const f4* __restrict__ table,
                                             const int* __restrict__ idx, int64_t n_idx,
                                             float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int sub = lane / kRowF4, q = lane % kRowF4;  // sub 0, 1 active; lanes 48..63 idle
  const bool act = sub < 2;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int64_t base = wave * 2 * U; base < n_idx; base += nw * 2 * U) {
    f4 z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + 2 * u + sub;
      z[u] = (act && e < n_idx) ? table[(int64_t)idx[e] * kRowF4 + q] : f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += z[u];
  }
  if (acc.x == 12345.0f) sink[0] = acc.y + acc.z + acc.w;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  // s_waitcnt vmcnt(N), expcnt / lgkmcnt left at their maxima (gfx9 encoding)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xf) | ((N >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

// slot of 8 rows: lane l of DMA instruction i moves bytes t = i*1024 + 16 l, i.e. piece
// (t % 384) / 16 of row t / 384
template <int S>
__global__ __launch_bounds__(256) void k_glds(const f4* __restrict__ table,
                                              const int* __restrict__ idx, int64_t n_slots,
                                              float* __restrict__ sink) {
  extern __shared__ f4 ring_all[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f4* ring = ring_all + (size_t)wv * S * 192;  // 3 KB = 192 f4 per slot
  const int64_t wave = (int64_t)blockIdx.x * 4 + wv;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int row_of[3], piece_of[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int t = i * 1024 + 16 * lane;
    row_of[i] = t / kRowB;
    piece_of[i] = (t % kRowB) / 16;
  }
  const int64_t my_slots = wave < n_slots ? (n_slots - 1 - wave) / nw + 1 : 0;
  auto issue = [&](int64_t j, int r) {  // j-th slot of this wave into ring position r
    const int64_t s = wave + j * nw;
    const int4* ip = reinterpret_cast<const int4*>(idx + s * 8);
    const int4 a = ip[0], b = ip[1];  // wave-uniform: scalar loads
    const int ix[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      int r8 = ix[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) r8 = row_of[i] == k ? ix[k] : r8;
      const f4* src = table + (int64_t)r8 * kRowF4 + piece_of[i];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src),
          (__attribute__((address_space(3))) void*)(ring + r * 192 + i * 64), 16, 0, 0);
    }
  };
  f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t pro = my_slots < S ? my_slots : S;
  for (int64_t j = 0; j < pro; ++j) issue(j, (int)j);
  for (int64_t j = 0; j < my_slots; ++j) {
    const int r = (int)(j % S);
    // slot j is done when at most the DMAs of the slots after it are outstanding
    const int64_t after = (my_slots - 1 - j) < (S - 1) ? (my_slots - 1 - j) : (S - 1);
    if (after >= S - 1) wait_vm<3 * (S - 1)>();
    else wait_vm<0>();
#pragma unroll
    for (int i = 0; i < 3; ++i) acc += ring[r * 192 + i * 64 + lane];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the reads are done before the refill
    if (j + S < my_slots) issue(j + S, r);
  }
  if (acc.x == 12345.0f) sink[0] = acc.y + acc.z + acc.w;
}

int main() {
  const int64_t n = 2449029;                  // rows of the table (940 MB)
  const int64_t n_idx = 32LL << 20;           // gathers per launch (12.9 GB)
  std::vector<int> hidx(n_idx);
  uint64_t st = 0x2545F4914F6CDD1Dull;
  for (auto& v : hidx) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    v = (int)(st % (uint64_t)n);
  }
  f4* table;
  int* idx;
  float* sink;
  CHECK(hipMalloc(&table, n * kRowB));
  CHECK(hipMemset(table, 0, n * kRowB));
  CHECK(hipMalloc(&idx, n_idx * 4));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemcpy(idx, hidx.data(), n_idx * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto time_ms = [&](auto body) {
    for (int i = 0; i < 2; ++i) body();
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < 5; ++i) body();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
  };
  const double bytes = (double)n_idx * kRowB;
  printf("# random 384-B rows from a %.0f MB table, %lld gathers per launch, %d CUs\n",
         n * kRowB / 1e6, (long long)n_idx, cus);
  printf("variant               blocks  lds_KB/CU  ms      GB/s   G_lines/s\n");
  auto report = [&](const char* name, int blocks, int lds_kb, float ms) {
    printf("%-20s  %6d  %9d  %6.3f  %6.0f  %6.1f\n", name, blocks, lds_kb, ms,
           bytes / (ms * 1e6), 3.0 * n_idx / (ms * 1e6));
    fflush(stdout);
  };
  for (int bpc : {8, 16}) {
    const int blocks = cus * bpc;
    report("reg U=2", blocks, 0, time_ms([&] {
             hipLaunchKernelGGL(k_reg<2>, dim3(blocks), dim3(256), 0, 0, table, idx, n_idx, sink);
           }));
    report("reg U=4", blocks, 0, time_ms([&] {
             hipLaunchKernelGGL(k_reg<4>, dim3(blocks), dim3(256), 0, 0, table, idx, n_idx, sink);
           }));
  }
  const int64_t n_slots = n_idx / 8;
#define GLDS(SS, BPC)                                                                         \
  do {                                                                                        \
    const size_t lds = (size_t)4 * SS * 3072;                                                 \
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_glds<SS>),                       \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));          \
    const int blocks = cus * BPC;                                                             \
    char nm[32];                                                                              \
    snprintf(nm, sizeof nm, "glds S=%d", SS);                                                 \
    report(nm, blocks, (int)(lds * BPC / 1024), time_ms([&] {                                 \
             hipLaunchKernelGGL(k_glds<SS>, dim3(blocks), dim3(256), lds, 0, table, idx,      \
                                n_slots, sink);                                               \
           }));                                                                               \
  } while (0)
  GLDS(2, 4);
  GLDS(3, 4);
  GLDS(4, 3);
  GLDS(6, 2);
  GLDS(8, 1);
  GLDS(12, 1);
  return 0;
}
