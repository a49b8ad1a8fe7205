// appnp_probe.hip -- the box's random-line gather rate, measured in-library (gfx950).
//
// The SpMM on a uniform random graph is bound by the rate at which the chip serves random
// 128-B line requests beyond L2 (53-60 G lines/s from 64 MB-1 GB tables,
// tools/gather_probe.hip).  Boxes and even processes differ in that rate ("two
// timing states"), so bench.py runs this probe on the bench's own H buffer right before its
// timed region and prints the rate next to the result (roofline.box_line_rate): a slow line
// then says whether the box served lines slowly or the kernel did.
//
// Shape: the gather_probe kernel's -- G = 8 lanes x 16 B per line, 8 lines per wave
// instruction, U = 8 instructions in flight -- with the line indices hashed in-kernel
// (splitmix64 of the request number), so no index stream competes with the gathers.  The sum of
// the gathered values feeds a store that never happens (unless the sum equals a sentinel), so
// the loads stay.
#include <algorithm>

#include "appnp_internal.h"
#include "../../include/ppnp_amd.h"

namespace appnp {
namespace {

constexpr int kProbeG = 8;                 // lanes per 128-B line
constexpr int kProbeLines = kWave / kProbeG;  // lines per wave instruction
constexpr int kProbeU = 8;                 // instructions in flight per wave
constexpr int kProbeThreads = 256;

__global__ __launch_bounds__(kProbeThreads) void k_line_probe(const f32x4* __restrict__ table,
                                                              int64_t n_lines, int64_t requests,
                                                              uint64_t seed,
                                                              float* __restrict__ sink) {
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane / kProbeG, gl = lane % kProbeG;
  const int64_t wave = (int64_t)blockIdx.x * (kProbeThreads / kWave) + (threadIdx.x >> 6);
  const int64_t waves = (int64_t)gridDim.x * (kProbeThreads / kWave);
  constexpr int64_t step = (int64_t)kProbeLines * kProbeU;
  f32x4 acc = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int64_t base = wave * step; base < requests; base += waves * step) {
    f32x4 z[kProbeU];
#pragma unroll
    for (int u = 0; u < kProbeU; ++u) {
      const int64_t e = base + u * kProbeLines + sub;
      z[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (e < requests) {
        // a 32-bit hash scaled to [0, n_lines) by a high multiply (no 64-bit division)
        const uint32_t h = (uint32_t)splitmix64(seed + (uint64_t)e);
        const int64_t line = (int64_t)__umulhi(h, (uint32_t)n_lines);
        z[u] = table[line * kProbeG + gl];
      }
    }
#pragma unroll
    for (int u = 0; u < kProbeU; ++u) acc += z[u];
  }
  if (acc.x == 1.2345e-30f) sink[0] = acc.y + acc.z + acc.w;
}

}  // namespace
}  // namespace appnp

extern "C" int appnp_line_rate_probe(const void* table, int64_t table_bytes, int64_t lines,
                                     uint64_t seed, float* sink, void* stream) {
  using namespace appnp;
  if (table_bytes < 128 || lines < 0 || !table || !sink) return APPNP_EINVAL;
  if (reinterpret_cast<uintptr_t>(table) % 128 != 0) return APPNP_EINVAL;
  if (lines == 0) return APPNP_OK;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return APPNP_EDEVICE;
  // 8 workgroups of 4 waves per CU (32 waves: the SpMM kernels' occupancy), grid-stride
  const int64_t per_wg = (int64_t)(kProbeThreads / kWave) * kProbeLines * kProbeU;
  const int64_t blocks = std::min<int64_t>((int64_t)cus * 8, (lines + per_wg - 1) / per_wg);
  hipLaunchKernelGGL(k_line_probe, dim3((unsigned)std::max<int64_t>(1, blocks)),
                     dim3(kProbeThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const f32x4*>(table),
                     std::min<int64_t>(table_bytes / 128, UINT32_MAX), lines, seed, sink);
  return hipGetLastError() == hipSuccess ? APPNP_OK : APPNP_EDEVICE;
}
