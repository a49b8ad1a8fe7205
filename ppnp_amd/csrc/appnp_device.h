// appnp_device.h -- shared device-side definitions for the gfx950 APPNP propagation path.
//
// Internal to libppnp_amd.so.  The public ABI is include/ppnp_amd.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace appnp {

constexpr int kWave = 64;           // CDNA wavefront
constexpr int kBlock = 256;         // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;

// Epilogue of one propagation step (y = scale * sum_j w_ij Zin[j]):
//   FWD      out = y + alpha * H                    (forward iteration)
//   BWD      out = y (if out != null); aux += alpha * y   (adjoint iteration; aux = dH)
//   PARTIAL  out(fp32) = y                          (local-column half of a split step; the
//                                                    first shard group of a pipelined one)
//   FINISH   out = y + aux(fp32) + alpha * H        (remote-column half of a split step; the
//                                                    last shard group of a pipelined one)
//   ACCUM    out(fp32) += y                         (a middle shard group of a pipelined step)
enum Epi { EPI_FWD = 0, EPI_BWD = 1, EPI_PARTIAL = 2, EPI_FINISH = 3, EPI_ACCUM = 4 };

struct StepArgs {
  const int32_t* row_ptr;  // local rows, row_ptr[0] == 0
  const int32_t* row_end;  // null: row i's entries end at row_ptr[i + 1]; else at row_end[i]
                           // (a shard range of the held rows: appnp_step_shards)
  const int32_t* col;      // global column index
  const float* val;        // A_hat values (fp32)
  const void* zin;         // all n rows (global index)
  const void* h;           // held rows (local index)
  void* out;               // held rows (local index)
  void* aux;               // BWD: dH (storage dtype); FINISH: fp32 partial
  int64_t ld_in, ld_h, ld_out, ld_aux;
  int64_t n_rows;          // rows held
  int64_t nnz;             // entries of those rows (< 0: unknown); picks the row shape
  int64_t nnz_rows;        // entries of the whole rows when nnz counts a part of them (a shard
                           // range, the LOCAL / REMOTE half); 0: nnz
  int64_t zin_rows;        // rows of zin (its last row is never over-read)
  int64_t row_lo;          // global index of local row 0 (hash key only)
  uint64_t mkey;           // per-iteration dropout key = splitmix64(seed + (k+1)*golden)
  int32_t f;               // features
  uint32_t drop_thr;       // 24-bit drop threshold (edge dropped iff hash24 < drop_thr)
  int32_t drop_on;         // 1 when p_drop > 0
  float scale;             // 1 - alpha
  float alpha;             // weight of H (FWD/FINISH) or of y into aux (BWD)
  float drop_scale;        // 1 / (1 - p)
  int32_t tkey;            // 1: hash key of entry (row i, col j) is (j, i)  (transposed operator)
  const int32_t* heavy;    // rows longer than heavy_thr (narrow kernels give them a wave)
  int64_t n_heavy;
  int32_t heavy_thr;
  int64_t light_blocks;    // set by launch_step: blocks [light_blocks, grid) take heavy rows
  const int32_t* hub;      // rows longer than kHubRow: the wide kernels dispatch them first
  int64_t n_hub;
  int32_t nt;              // cache policy of the streams (set by launch_step): bit 0 col/val,
                           // bit 1 H, bit 2 Zout -- non-temporal, so they do not evict the
                           // gathered rows of Zin from the Infinity Cache
  float* rem_dh;           // remainder pass, adjoint: dH's remainder columns (rows x ld_rem_dh)
  int64_t ld_rem_dh;
};

// End of row i's entries in the step's CSR (StepArgs::row_end)
__device__ __forceinline__ int32_t row_end_of(const StepArgs& a, int64_t i) {
  return a.row_end ? a.row_end[i] : a.row_ptr[i + 1];
}

constexpr int kHeavyRow = 32;   // a row longer than this gets a whole wavefront (narrow)
constexpr int kHubRow = 512;    // ... and one longer than this is dispatched first (wide)
constexpr int kWideAvgRow = 24; // mean row length from which large graphs take a wave per row
constexpr int kSourceBlockLog2 = 15;  // source rows per block of the remainder pass: 2^15
                                     // (512 KB of 16-B remainders; the waves of an XCD drift
                                     // over a few blocks, which must share its 4 MB L2:
                                     // products-synth 2^14 / 2^15 / 2^16 / 2^17 rows
                                     // 8.00 / 7.97 / 8.22 / 8.27 ms per iteration)
#ifndef APPNP_REM_WAVES
#define APPNP_REM_WAVES 16  // -DAPPNP_REM_WAVES=n: measurement variants (tools/build_variant.sh)
#endif
constexpr int kRemWaves = APPNP_REM_WAVES;  // waves per workgroup of the persistent remainder pass
constexpr int kRemColBits = 20;      // column-in-block bits of a packed remainder entry
constexpr int kRemRowBits = 12;      // row-in-group bits (the rest of the 32)
constexpr int kNearRows = 1 << 14;  // "near" entry: |col - row| below this (gather locality)

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Edge dropout: counter hash of (key, row, col); identical to oracle/ppnp_oracle.py
// edge_keep_mask.  Independent of the partition and of the visiting order.
__device__ __forceinline__ float edge_weight(float w, int64_t grow, int32_t c,
                                             const StepArgs& a) {
  if (!a.drop_on) return w;
  const uint64_t r = (uint32_t)grow, cc = (uint32_t)c;
  const uint64_t key = a.tkey ? ((cc << 32) | r) : ((r << 32) | cc);
  const uint64_t h = splitmix64(key ^ a.mkey);
  return ((uint32_t)(h >> 40) >= a.drop_thr) ? w * a.drop_scale : 0.0f;
}

// ---- storage traits: V consecutive elements <-> V fp32 registers -------------------------

__device__ __forceinline__ float bf16_to_f32(uint32_t b) { return __uint_as_float(b << 16); }

// round-to-nearest-even, NaN stays NaN
__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

template <typename T, int V>
struct Io;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// non-temporal accesses for the streams (touched once per launch)
template <typename W>
__device__ __forceinline__ W ld_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const W*>(p));
}
template <typename W>
__device__ __forceinline__ void st_nt(void* p, W w) {
  __builtin_nontemporal_store(w, reinterpret_cast<W*>(p));
}

template <int V>
struct Io<float, V> {
  static __device__ __forceinline__ void load(const float* p, float (&x)[V]) {
    if constexpr (V == 4) {
      const float4 t = *reinterpret_cast<const float4*>(p);
      x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
    } else if constexpr (V == 2) {
      const float2 t = *reinterpret_cast<const float2*>(p);
      x[0] = t.x; x[1] = t.y;
    } else {
      x[0] = *p;
    }
  }
  static __device__ __forceinline__ void store(float* p, const float (&x)[V]) {
    if constexpr (V == 4) {
      *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
    } else if constexpr (V == 2) {
      *reinterpret_cast<float2*>(p) = make_float2(x[0], x[1]);
    } else {
      *p = x[0];
    }
  }
  static __device__ __forceinline__ void load_nt(const float* p, float (&x)[V]) {
    if constexpr (V == 4) {
      const f32x4 t = ld_nt<f32x4>(p);
      x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
    } else if constexpr (V == 2) {
      const f32x2 t = ld_nt<f32x2>(p);
      x[0] = t.x; x[1] = t.y;
    } else {
      x[0] = ld_nt<float>(p);
    }
  }
  static __device__ __forceinline__ void store_nt(float* p, const float (&x)[V]) {
    if constexpr (V == 4) {
      st_nt<f32x4>(p, f32x4{x[0], x[1], x[2], x[3]});
    } else if constexpr (V == 2) {
      st_nt<f32x2>(p, f32x2{x[0], x[1]});
    } else {
      st_nt<float>(p, x[0]);
    }
  }
};

template <int V>
struct Io<uint16_t, V> {  // bf16 storage
  static __device__ __forceinline__ void load(const uint16_t* p, float (&x)[V]) {
    if constexpr (V == 8) {
      const uint4 t = *reinterpret_cast<const uint4*>(p);
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[2 * i] = __uint_as_float(w[i] << 16);
        x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    } else if constexpr (V == 4) {
      const uint2 t = *reinterpret_cast<const uint2*>(p);
      x[0] = __uint_as_float(t.x << 16); x[1] = __uint_as_float(t.x & 0xffff0000u);
      x[2] = __uint_as_float(t.y << 16); x[3] = __uint_as_float(t.y & 0xffff0000u);
    } else if constexpr (V == 2) {
      const uint32_t t = *reinterpret_cast<const uint32_t*>(p);
      x[0] = __uint_as_float(t << 16); x[1] = __uint_as_float(t & 0xffff0000u);
    } else {
      x[0] = bf16_to_f32(*p);
    }
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float (&x)[V]) {
    if constexpr (V == 8) {
      uint4 t;
      t.x = f32_to_bf16(x[0]) | (f32_to_bf16(x[1]) << 16);
      t.y = f32_to_bf16(x[2]) | (f32_to_bf16(x[3]) << 16);
      t.z = f32_to_bf16(x[4]) | (f32_to_bf16(x[5]) << 16);
      t.w = f32_to_bf16(x[6]) | (f32_to_bf16(x[7]) << 16);
      *reinterpret_cast<uint4*>(p) = t;
    } else if constexpr (V == 4) {
      uint2 t;
      t.x = f32_to_bf16(x[0]) | (f32_to_bf16(x[1]) << 16);
      t.y = f32_to_bf16(x[2]) | (f32_to_bf16(x[3]) << 16);
      *reinterpret_cast<uint2*>(p) = t;
    } else if constexpr (V == 2) {
      *reinterpret_cast<uint32_t*>(p) = f32_to_bf16(x[0]) | (f32_to_bf16(x[1]) << 16);
    } else {
      *p = (uint16_t)f32_to_bf16(x[0]);
    }
  }
  static __device__ __forceinline__ void load_nt(const uint16_t* p, float (&x)[V]) {
    if constexpr (V == 8) {
      const u32x4 t = ld_nt<u32x4>(p);
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[2 * i] = __uint_as_float(w[i] << 16);
        x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    } else if constexpr (V == 4) {
      const u32x2 t = ld_nt<u32x2>(p);
      x[0] = __uint_as_float(t.x << 16); x[1] = __uint_as_float(t.x & 0xffff0000u);
      x[2] = __uint_as_float(t.y << 16); x[3] = __uint_as_float(t.y & 0xffff0000u);
    } else {
      load(p, x);
    }
  }
  static __device__ __forceinline__ void store_nt(uint16_t* p, const float (&x)[V]) {
    if constexpr (V == 8) {
      st_nt<u32x4>(p, u32x4{f32_to_bf16(x[0]) | (f32_to_bf16(x[1]) << 16),
                            f32_to_bf16(x[2]) | (f32_to_bf16(x[3]) << 16),
                            f32_to_bf16(x[4]) | (f32_to_bf16(x[5]) << 16),
                            f32_to_bf16(x[6]) | (f32_to_bf16(x[7]) << 16)});
    } else if constexpr (V == 4) {
      st_nt<u32x2>(p, u32x2{f32_to_bf16(x[0]) | (f32_to_bf16(x[1]) << 16),
                            f32_to_bf16(x[2]) | (f32_to_bf16(x[3]) << 16)});
    } else {
      store(p, x);
    }
  }
};

}  // namespace appnp
