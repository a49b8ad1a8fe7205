// appnp_blocks.hip -- remainder columns of a row through one persistent, L2-resident pass
// per iteration (gfx950).
//
// Why.  The SpMM is bound by random 128-B line requests: every nonzero
// gathers one row of Z.  An fp32 row of F = 32q + r features (1 <= r <= 4: F = 100 is
// 96 + 4) spans q + 1 lines, and the last one carries only r * 4 <= 16 useful bytes -- a
// quarter of products-synth's line requests.  Those r columns are taken out of the gather:
//
//   * Z between iterations is kept "split": Z_main [n, 32q] (rows of whole lines, so a
//     gather is exactly q lines) and Z_rem [n, 4] (16 B per row).
//   * The remainder product  R = (M_k o A_hat) Z_rem  runs as ONE launch per iteration that
//     sweeps A_hat by SOURCE block: block b holds the entries whose column lies in
//     [b * 2^15, (b+1) * 2^15), i.e. 512 KB of Z_rem, which sits in every XCD's 4 MB L2 while
//     the chip gathers from it.  Every wave walks the blocks in the same order at about the
//     same rate, so the blocks live in L2 at one time are the few between the slowest and
//     the fastest wave.  For this one-row-pass W4 pass, pacing measured slower every way it was
//     tried: per-block counters with a workgroup barrier (8.33 against 8.15 ms per
//     products-synth iteration), per-wave signals with bounded waits inside groups of
//     co-located workgroups, leading by 1, 2 or 4 blocks (8.6 to 16.9 against 8.2 ms),
//     an in-workgroup progress window, barriers every 8-32 blocks (profiles/r4_sync_ab.txt)
//     and XCD-wide arrival counters (profiles/r5_pace_ab.txt).  The wider
//     passes, whose 2-4 row passes let the waves drift much further, take a barrier every 32
//     blocks (k_rem_persist).
//
// The accumulators never leave the chip.  The launch is persistent -- one 1024-thread
// workgroup per CU, each of its 16 waves owning a group of <= 640 destination rows whose
// 16-B sums live in that wave's slice of LDS (16 x 640 x 16 B = 160 KiB) across all blocks.
// (The round-1 form launched once per block and re-read / re-wrote a [n, 4] accumulator in
// HBM every launch: 19 launches and ~2.7 GB of streams per products-synth iteration.)
//
// Work inside a wave is entry-parallel, so hub rows and ragged groups cost no idle lanes:
// the wave streams its entries -- block after block, one contiguous run per wave, each
// block's segment padded to whole chunks of 64 so a chunk never mixes blocks -- one entry per
// lane, sorted by (row, column); gathers Z_rem[column] from L2; and combines the products
// of equal rows with a segmented inclusive scan over the lanes (DPP row shifts + row
// broadcasts, fixed order); each segment's last lane adds the sum into its row's LDS slot.
// U = 2 chunks (128 entries; APPNP_REM_U at compile time) are in flight per wave: fewer chunks
// keep the waves of an XCD close together in the block sweep, so fewer blocks share its L2
// (92 % hits at U = 2, 66 % at U = 8).  The order of every addition is fixed by
// the layout: bitwise deterministic run to run.
//
// The regrouped copy of A_hat (APPNP_GRAPH_SOURCE_BLOCKS / _SB_W8 / _SB_W16) is built at graph
// creation: the entries of wave group g's block b are the segment off[g * nb + b] ..
// off[g * nb + b + 1], each packed into 32 bits as (row in group << kRemColBits | column in
// block), kRemColBits = 20, with their fp32 value (none on a unit graph, below); padding
// entries are kRemNone (all ones) with value 0.  A wave group holds 640 / LPE rows.  off holds
// passes x (CUs x 16) x blocks + 1 ints: linear in n (one int per (640 / LPE)-row x 2^15-column
// tile of A_hat, ~1.2 MB on products-synth at LPE = 1).
//
// A unit graph (unweighted A without self loops: every entry of A+I is 1, so A_hat_ij =
// dl_i dr_j with sym: dl = dr = dinv, rw: dl = dinv, dr = 1) stores NO values: the remainder
// buffers hold dr o Z_rem, the pass sums the gathered rows and the epilogue scales by dl_i.
// The entry stream halves (4 B per entry): 0.91 -> 0.81 ms per products-synth launch.
//
// Wider remainders (APPNP_GRAPH_SB_W8 / APPNP_GRAPH_SB_W16): the same pass over rows of
// W = 4 LPE fp32 columns, LPE = 2 or 4 lanes per entry, laid out piece-major (lane = piece * CH +
// entry, CH = 64 / LPE entries per chunk), so every 16-lane DPP row holds one 16-B piece of up to
// 16 consecutive entries and the segmented scan compares (row, piece).  A wave group holds
// 640 / LPE rows.  It takes 5-8 remainder columns (F = 32q + r) and narrow rows (F <= W) out
// of the random gather: on products-synth F = 16 takes 2.01 against 2.40 ms per iteration and
// F = 40 = 32 + 8 3.68 against 4.44 ms (profiles/r2_wide_remainder.txt).
// LPE = 1 is the pass above, unchanged.
//
// The sums of a wave group live in LDS piece-major: piece q of row r at slot q rg + r.  The tails
// of one piece in an 8-lane group of a 16-B LDS access are then consecutive slots for
// consecutive rows; row-major (a 64-B row stride on a W16 copy) put every row of one parity in
// the same 4 banks: 2.2e8 bank-conflict cycles per launch of the 8-rank column slab's pass
// (SQ_LDS_BANK_CONFLICT), 5.2e7 piece-major; W16 1.825 -> 1.817 ms, W8 0.977 -> 0.970 ms
// (profiles/r6_w16_ab.txt).
#include <algorithm>
#include <cstdlib>

#include "appnp_internal.h"
#include "../../include/ppnp_amd.h"

namespace appnp {
namespace {

constexpr int kRemThreads = kRemWaves * kWave;  // 1024 at 16 waves
constexpr int kRemLdsBytes = 160 * 1024;        // LDS per CU on gfx950
constexpr int kRemMaxRg = kRemLdsBytes / (kRemWaves * 16);  // 640 rows per wave group at 16
constexpr uint32_t kRemNone = 0xffffffffu;      // packed entry of an idle lane (row 4095)
constexpr int kWalkWaves = kWavesPerBlock;      // build walk: one wave per group
constexpr int kWalkMaxBlocks = 4096;            // LDS cursors of the build walk: 64 KiB
constexpr int kRemChunk = kWave;                // entries per chunk; segments padded to it
#ifndef APPNP_REM_U
#define APPNP_REM_U 2
#endif
constexpr int kRemU = APPNP_REM_U;              // chunks in flight per wave (-DAPPNP_REM_U: measurement)
// The W16 pass (16 entries per chunk) keeps 4 chunks in flight: the 13-column slab of
// products-synth took 1.93 ms at 4, 1.94 at 8, 2.01 at 2 and 2.25 at 1; the W8 pass (F = 40)
// 1.212 ms at 4 against 1.205 at 2 (profiles/r4_w16_ab.txt, r4_sync_ab.txt)
#ifndef APPNP_REM_U_W16
#define APPNP_REM_U_W16 4
#endif
constexpr int kRemUW16 = APPNP_REM_U_W16;

static_assert(kRemMaxRg < (1 << kRemRowBits), "row in group must fit the packed entry");
static_assert(kRemRowBits + kRemColBits == 32, "packed entry is 32 bits");

struct RemLayout {
  const int32_t* off;   // segment starts, [(pass * slots + slot) * nb + block]
  const uint32_t* ent;  // packed (row in group, column in block); padding: kRemNone
  const float* val;     // entry values; null for a unit graph (VF kernels)
  const int32_t* cblk;  // source block of each chunk of 64 entries
  const float* dl;      // VF: row scale of A_hat (fp32 dinv) of the held rows (local index)
  const float* dr;      // VF: column scale (sym: fp32 dinv; rw: null) of all n rows (global
                        // index).  Z_rem buffers hold dr o Z_rem, so a gathered row needs no
                        // value
  int32_t nb, br_log2, slots, rg, passes;
  int32_t scale_out;    // VF: the output is the next remainder buffer (store dr o y)
  int32_t sync;         // > 0: workgroup barrier after every `sync` source blocks (k_rem_persist)
};

// ---- segmented inclusive scan over the 64 lanes (rows non-decreasing across lanes) --------
// DPP (gfx9 family): row_shr:n shifts within each 16-lane row; row_bcast:15 / row_bcast:31
// feed lane 15 of a row / lane 31 to the rows above.  A lane adds the moved partial only when
// it comes from a lane of the same row index (segment); rows are sorted, so equality of the
// two end points means every lane between belongs to the segment too.
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114,
              kDppRowShr8 = 0x118, kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143,
              kDppWaveShr1 = 0x138;  // whole-wave shift by one lane (GFX9 family)

// bound_ctrl: a lane whose source lane is out of its row (or outside ROW_MASK's rows) reads 0
// for both the row and the partial.  A spurious match on row 0 then adds 0.0, so no 'old'
// operand needs initialising (five fewer moves per step).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void seg_step(int row, f32x4& v) {
  const int src_row = __builtin_amdgcn_update_dpp(0, row, CTRL, ROW_MASK, 0xf, true);
  const float ux = __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v.x), CTRL, ROW_MASK, 0xf, true));
  const float uy = __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v.y), CTRL, ROW_MASK, 0xf, true));
  const float uz = __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v.z), CTRL, ROW_MASK, 0xf, true));
  const float uw = __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v.w), CTRL, ROW_MASK, 0xf, true));
  if (src_row == row) {
    v.x += ux;
    v.y += uy;
    v.z += uz;
    v.w += uw;
  }
}

// Segmented inclusive scan of v over runs of equal `row` (Hillis-Steele over DPP: row_shr 1,
// 2, 4, 8 within each 16-lane row, then row_bcast15 / row_bcast31 across rows), running only
// the steps some run needs.  `heads` (wave-uniform) marks the first lane of every run.  An
// in-row step of shift d is a no-op unless some lane sits >= d places after its run's head
// within its 16-lane row, and a broadcast is a no-op unless lane 16 / 48 (bcast15) or lane 32
// (bcast31) continues a run.  So the result is the full six-step scan's, bit for bit.  Runs in
// a chunk are short (a group's row has ~0.7 entries per source block), so most chunks need
// two or three steps.
template <int CH>
__device__ __forceinline__ void seg_scan(int row, f32x4& v, unsigned long long heads) {
  unsigned long long m = ~(heads | 0x0001000100010001ull);  // lanes >= 1 after their head
  if (m) {
    seg_step<kDppRowShr1, 0xf>(row, v);
    m &= m << 1;  // >= 2 after
    if (m) {
      seg_step<kDppRowShr2, 0xf>(row, v);
      m &= m << 2;  // >= 4 after
      if (m) {
        seg_step<kDppRowShr4, 0xf>(row, v);
        if (m & (m << 4)) seg_step<kDppRowShr8, 0xf>(row, v);
      }
    }
  }
  // runs cross 16-lane rows only where a piece spans several of them (CH = 32, 64)
  if constexpr (CH >= 32) {
    if (~heads & ((1ull << 16) | (1ull << 48)))
      seg_step<kDppRowBcast15, 0xa>(row, v);  // rows 1, 3 <- lanes 15, 47
  }
  if constexpr (CH == 64) {
    if (~heads & (1ull << 32)) seg_step<kDppRowBcast31, 0xc>(row, v);  // rows 2, 3 <- lane 31
  }
}

// Epilogue of one row of the iteration: FWD out[i, :nv] = (1-alpha) R[i] + alpha H_rem[i]
// (a.h = H_rem, a.out / a.ld_out, a.f = nv valid columns: 4 into the next Z_rem, 1-4 into Z's
// last columns); BWD G_k = (1-alpha) R into the next remainder buffer (none at k = 0) and
// dH[:, fs:f] += alpha' G_k (a.rem_dh / a.ld_rem_dh).
template <int EPI, bool VF>
__device__ __forceinline__ void rem_finish(const StepArgs& a, const RemLayout& L, int64_t i,
                                           f32x4 acc) {
  float so = 1.0f;  // VF: scale of a stored remainder row (dr_i), 1 for Z itself
  if constexpr (VF) {
    const float dl = L.dl[i];
    acc = f32x4{dl * acc.x, dl * acc.y, dl * acc.z, dl * acc.w};
    if (L.scale_out && L.dr) so = L.dr[a.row_lo + i];  // dr: all n rows (global index)
  }
  if constexpr (EPI == EPI_BWD) {
    const float y[4] = {a.scale * acc.x, a.scale * acc.y, a.scale * acc.z, a.scale * acc.w};
    if (a.out)
      static_cast<f32x4*>(a.out)[i] = f32x4{so * y[0], so * y[1], so * y[2], so * y[3]};
    const int nv = a.f;
    float* d = a.rem_dh + i * a.ld_rem_dh;
    if (nv == 4) {
      f32x4 v = *reinterpret_cast<f32x4*>(d);
      v = f32x4{fmaf(a.alpha, y[0], v.x), fmaf(a.alpha, y[1], v.y), fmaf(a.alpha, y[2], v.z),
                fmaf(a.alpha, y[3], v.w)};
      *reinterpret_cast<f32x4*>(d) = v;
    } else {
      for (int v = 0; v < nv; ++v) d[v] = fmaf(a.alpha, y[v], d[v]);
    }
  } else {
    // H rows are 16-B aligned with ld_h >= roundup(f, 4): the 16 B at H_rem stay inside the
    // row's storage, except possibly on the buffer's last row (read exactly nv there)
    const int nv = a.f;
    const float* hp = static_cast<const float*>(a.h) + i * a.ld_h;
    f32x4 h = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (nv == 4 || i + 1 < a.n_rows) {
      h = *reinterpret_cast<const f32x4*>(hp);
    } else {
      h.x = hp[0];
      if (nv > 1) h.y = hp[1];
      if (nv > 2) h.z = hp[2];
    }
    const float y[4] = {fmaf(a.alpha, h.x, a.scale * acc.x),
                        fmaf(a.alpha, nv > 1 ? h.y : 0.0f, a.scale * acc.y),
                        fmaf(a.alpha, nv > 2 ? h.z : 0.0f, a.scale * acc.z),
                        fmaf(a.alpha, nv > 3 ? h.w : 0.0f, a.scale * acc.w)};
    float* o = static_cast<float*>(a.out) + i * a.ld_out;
    if (nv == 4) {
      *reinterpret_cast<f32x4*>(o) = f32x4{so * y[0], so * y[1], so * y[2], so * y[3]};
    } else {
      for (int v = 0; v < nv; ++v) o[v] = y[v];
    }
  }
}

// The epilogue of piece q (columns 4q .. 4q+3 of the remainder) of one row for LPE > 1.
// a.f = nv: the valid remainder columns (f - fs), on every iteration; L.scale_out: the output
// is the next remainder buffer (rows of 4 LPE floats, a.ld_out = 4 LPE; unit graph: dr o y)
// rather than Z (only the valid columns).  FWD reads H_rem's valid columns only; BWD adds
// alpha' G_k into dH's valid columns.
template <int EPI, bool VF, int LPE>
__device__ __forceinline__ void rem_finish_piece(const StepArgs& a, const RemLayout& L, int64_t i,
                                                 int q, f32x4 acc) {
  const int nv = a.f - 4 * q;  // valid columns of this piece (may be <= 0)
  float so = 1.0f;
  if constexpr (VF) {
    const float dl = L.dl[i];
    acc = f32x4{dl * acc.x, dl * acc.y, dl * acc.z, dl * acc.w};
    if (L.scale_out && L.dr) so = L.dr[a.row_lo + i];
  }
  float y[4] = {a.scale * acc.x, a.scale * acc.y, a.scale * acc.z, a.scale * acc.w};
  if constexpr (EPI == EPI_BWD) {
    if (a.out)
      static_cast<f32x4*>(a.out)[i * LPE + q] = f32x4{so * y[0], so * y[1], so * y[2], so * y[3]};
    float* d = a.rem_dh + i * a.ld_rem_dh + 4 * q;
    for (int v = 0; v < 4 && v < nv; ++v) d[v] = fmaf(a.alpha, y[v], d[v]);
  } else {
    const float* hp = static_cast<const float*>(a.h) + i * a.ld_h + 4 * q;
#pragma unroll
    for (int v = 0; v < 4; ++v) y[v] = v < nv ? fmaf(a.alpha, hp[v], y[v]) : y[v];
    if (L.scale_out) {
      static_cast<f32x4*>(a.out)[i * LPE + q] = f32x4{so * y[0], so * y[1], so * y[2], so * y[3]};
    } else {
      float* o = static_cast<float*>(a.out) + i * a.ld_out + 4 * q;
      for (int v = 0; v < 4 && v < nv; ++v) o[v] = y[v];
    }
  }
}

// The wave's LDS sums of a row group, piece-major (see the file comment): piece q of row `row`
// is acc[q * rg + row].
#ifdef APPNP_REM_ROW_MAJOR  // measurement variant: the round-5 row-major sums
#define REM_SLOT(q, row) ((row) * LPE + (q))
#else
#define REM_SLOT(q, row) ((q) * L.rg + (row))
#endif

// Chunks [c_begin, c_end) of a wave's entry stream: gather, weight, segmented scan, and the
// run tails' adds into the wave's LDS rows.  U chunks in flight; the source block of chunk c is
// cblk[c].
template <int U, bool VF, int LPE>
__device__ __forceinline__ void rem_walk(const StepArgs& a, const RemLayout& L,
                                         const f32x4* __restrict__ z, f32x4* acc, int64_t r0,
                                         int32_t c_begin, int32_t c_end) {
  constexpr int CH = kWave / LPE;  // entries per chunk; piece q of entry e on lane q * CH + e
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane / CH, le = lane % CH;
  const uint32_t cmask = (1u << kRemColBits) - 1u;
  // the entries of chunks [c0, c0 + U): first source row of each chunk's block (wave-uniform:
  // scalar loads), packed entry, value
  auto fetch = [&](int32_t c0, int32_t (&cbx)[U], uint32_t (&enx)[U], float (&wtx)[U]) {
    const int n = min(U, c_end - c0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cbx[u] = 0;
      enx[u] = kRemNone;
      wtx[u] = 1.0f;
      if (u < n) {
        const int64_t e = (int64_t)(c0 + u) * CH + le;
        cbx[u] = L.cblk[c0 + u] << L.br_log2;
        enx[u] = ld_nt<uint32_t>(L.ent + e);
        if constexpr (!VF) wtx[u] = ld_nt<float>(L.val + e);
      }
    }
  };
  int32_t cb[U];
  uint32_t en[U];
  float wt[U];
#ifdef APPNP_REM_PREFETCH
  fetch(c_begin, cb, en, wt);
#endif
  for (int32_t c = c_begin; c < c_end; c += U) {
    const int nch = min(U, c_end - c);
#ifndef APPNP_REM_PREFETCH
    fetch(c, cb, en, wt);
#endif
    f32x4 zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (LPE == 1) {
        zv[u] = en[u] != kRemNone ? z[cb[u] + (int32_t)(en[u] & cmask)]
                                  : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      } else {
        // a piece wholly past the valid remainder columns (a.f) holds zeros in every buffer:
        // no request for it (a 4-column remainder on a W8 / W16 copy gathers one piece)
        zv[u] = (en[u] != kRemNone && 4 * q < a.f)
                    ? z[(int64_t)(cb[u] + (int32_t)(en[u] & cmask)) * LPE + q]
                    : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
    }
#ifdef APPNP_REM_PREFETCH
    // measurement variant: the next chunks' entries load under this iteration's gathers
    int32_t cbn[U];
    uint32_t enn[U];
    float wtn[U];
    fetch(c + U, cbn, enn, wtn);
#endif
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= nch) break;  // wave-uniform
      const bool act = en[u] != kRemNone;
      const int row = (int)(en[u] >> kRemColBits);
      // scan key: the row, and for LPE > 1 the piece (runs never cross pieces)
      const int key = LPE == 1 ? row : ((row << 3) | q);
      f32x4 v = zv[u];
      if (!VF || a.drop_on) {
        const float w = act ? edge_weight(wt[u], a.row_lo + r0 + row,
                                          cb[u] + (int32_t)(en[u] & cmask), a)
                            : 0.0f;
        v = f32x4{w * v.x, w * v.y, w * v.z, w * v.w};
      }
      // the previous lane's row (lane 0: none), by DPP rather than an LDS permute
      const int prev = __builtin_amdgcn_update_dpp(-1, key, kDppWaveShr1, 0xf, 0xf, false);
      const unsigned long long heads = __ballot(lane == 0 || prev != key || !act);
      seg_scan<CH>(key, v, heads);
      const bool tail = le == CH - 1 || ((heads >> (lane + 1)) & 1ull);
      if (act && tail) {
        f32x4& t = acc[REM_SLOT(q, row)];
        t = f32x4{t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w};
      }
    }
#ifdef APPNP_REM_PREFETCH
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cb[u] = cbn[u];
      en[u] = enn[u];
      wt[u] = wtn[u];
    }
#endif
  }
}

// One iteration of the remainder columns over all source blocks (see the file comment).
// a.zin = Z_rem (n x 4 fp32; VF: dr o Z_rem); U chunks of 64 entries in flight per wave.
// VF (unit graph): entries carry no value -- the sum of the gathered dr_j Z_j is scaled by
// dl_i in the epilogue, so the entry stream is 4 B per entry instead of 8 (0.91 -> 0.81 ms
// per products-synth launch).
// L.sync > 0 (the W8 / W16 passes, rem_sync_blocks): the waves of a workgroup walk the source
// blocks in step, with a workgroup barrier after every L.sync blocks and at the end of every row
// pass.  Without it a wave streams its segments back to back, and the CU's oldest-first
// arbitration spreads its waves over ~12 % of a sweep (profiles/r3_rem_timeline.txt), and
// further over the 2-4 row passes of a wide pass: the span of blocks in use must share the
// XCD's 4 MB L2, which a W4 table's 512-KB blocks do (92 % hits) and a W16 table's 2-MB blocks
// do not (28 %; profiles/r4_w16_ab.txt).  A barrier after every block lifts the W16 pass to
// 58 % hits but leaves waves idle at every block; every 32 blocks keeps 52 % and wins
// (profiles/r4_sync_ab.txt).  A softer per-block progress window (a wave ahead of its
// workgroup's slowest by more than D blocks sleeps; LDS counters) lost at every width and D.
template <int EPI, int U, bool VF, int LPE>
__global__ __launch_bounds__(kRemThreads) void k_rem_persist(StepArgs a, RemLayout L) {
  constexpr int CH = kWave / LPE;
  extern __shared__ f32x4 rem_acc[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4* acc = rem_acc + (int64_t)wv * L.rg * LPE;  // this wave's rg rows x LPE pieces
  const f32x4* __restrict__ z = static_cast<const f32x4*>(a.zin);
  const int64_t slot = (int64_t)blockIdx.x * kRemWaves + wv;
  for (int p = 0; p < L.passes; ++p) {
    const int64_t g = (int64_t)p * L.slots + slot;
    const int64_t r0 = g * L.rg;
    const int rows = (int)max<int64_t>(0, min<int64_t>(L.rg, a.n_rows - r0));
    for (int r = lane; r < L.rg * LPE; r += kWave) acc[r] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (L.sync > 0) {
      // every wave runs the same nb blocks (an empty segment is 0 chunks) in the same steps,
      // so every wave reaches every barrier; a wave's segments are contiguous in its stream
      for (int b = 0; b < L.nb; b += L.sync) {
        rem_walk<U, VF, LPE>(a, L, z, acc, r0, L.off[g * L.nb + b] / CH,
                             L.off[g * L.nb + min(b + L.sync, L.nb)] / CH);
        __syncthreads();
      }
    } else {
      // this wave's stream: blocks 0..nb-1 back to back, each a whole number of chunks
      rem_walk<U, VF, LPE>(a, L, z, acc, r0, L.off[g * L.nb] / CH, L.off[(g + 1) * L.nb] / CH);
    }
    if constexpr (LPE == 1) {
      for (int r = lane; r < rows; r += kWave) rem_finish<EPI, VF>(a, L, r0 + r, acc[r]);
    } else {
      // row-major over (row, piece), so a wave's stores cover whole rows of the output (a
      // piece-major order here, 16-B stores 16 LPE B apart, measured 5 % slower at W16)
      for (int r = lane; r < rows * LPE; r += kWave)
        rem_finish_piece<EPI, VF, LPE>(a, L, r0 + r / LPE, r % LPE,
                                       acc[REM_SLOT(r % LPE, r / LPE)]);
    }
  }
}

// Build walk: one wave per group, walking the group's rows in order with one cursor per
// source block in LDS.  COUNT: the number of entries of each (group, block) segment, padded
// to whole chunks, into cnt, plus the off-diagonal entries within kNearRows of their row
// (gather locality).  FILL: cursors start at the segment offsets; every entry is written to
// its slot (the padding stays as preset).  A row's columns are sorted, so its entries of one
// block are a run of consecutive lanes.
template <bool FILL>
__global__ __launch_bounds__(kBlock) void k_rb_walk(const int32_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const float* __restrict__ val, int64_t n,
                                                    int64_t row_lo, int rg, int nb, int br_log2,
                                                    int chunk,
                                                    int64_t n_groups, int32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ off,
                                                    uint32_t* __restrict__ ent,
                                                    float* __restrict__ bval,
                                                    unsigned long long* __restrict__ near) {
  extern __shared__ int32_t walk_cur[];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = threadIdx.x >> 6;
  int32_t* cur = walk_cur + (int64_t)w * nb;
  const int64_t g = (int64_t)blockIdx.x * kWalkWaves + w;
  if (g >= n_groups) return;  // no workgroup barrier in this kernel
  for (int b = lane; b < nb; b += kWave) cur[b] = FILL ? off[g * nb + b] : 0;
  const int64_t r0 = g * rg, r1 = min<int64_t>(n, r0 + rg);
  unsigned long long nr = 0;
  for (int64_t i = r0; i < r1; ++i) {
    const int32_t beg = rp[i], end = rp[i + 1];
    for (int32_t e0 = beg; e0 < end; e0 += kWave) {
      const int32_t e = e0 + lane;
      const bool act = e < end;
      const int32_t c = act ? col[e] : 0;
      const int b = act ? (c >> br_log2) : INT32_MAX;
      const int bprev = __shfl_up(b, 1);
      const unsigned long long heads = __ballot(act && (lane == 0 || bprev != b));
      const unsigned long long upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1ull);
      const int head = 63 - __clzll(heads & upto);  // first lane of this lane's run
      const int bnext = __shfl_down(b, 1);
      const bool tail = act && (lane == kWave - 1 || bnext != b);
      int32_t base = 0;
      if (act) base = cur[b];
      if constexpr (FILL) {
        if (act) {
          const int32_t pos = base + (lane - head);
          ent[pos] = ((uint32_t)(i - r0) << kRemColBits) | ((uint32_t)c & ((1u << br_log2) - 1u));
          if (bval) bval[pos] = val[e];
        }
      } else {
        const int64_t d = (int64_t)c - (row_lo + i);  // global row vs global column
        nr += (act && d != 0 && d < kNearRows && d > -kNearRows) ? 1 : 0;
      }
      if (tail) cur[b] = base + (lane - head + 1);
    }
  }
  if constexpr (!FILL) {
    for (int b = lane; b < nb; b += kWave)
      cnt[g * nb + b] = (cur[b] + chunk - 1) / chunk * chunk;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) nr += __shfl_xor(nr, o);
    if (lane == 0 && nr) atomicAdd(near, nr);
  }
}

// Off-diagonal entries of A within kNearRows of their row, over ALL n rows (the gather-locality
// measure of a row-partitioned graph: every rank computes the same value from the same A, so
// every rank takes the same split decision).  Thread per row, grid-stride.
__global__ __launch_bounds__(kBlock) void k_near_all(const int32_t* __restrict__ rp,
                                                     const int32_t* __restrict__ col, int64_t n,
                                                     unsigned long long* __restrict__ near) {
  unsigned long long nr = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    for (int32_t e = rp[i]; e < rp[i + 1]; ++e) {
      const int64_t d = (int64_t)col[e] - i;
      nr += (d != 0 && d < kNearRows && d > -kNearRows) ? 1 : 0;
    }
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) nr += __shfl_xor(nr, o);
  if ((threadIdx.x & (kWave - 1)) == 0 && nr) atomicAdd(near, nr);
}

// cblk[c] = b for every chunk c of segment (group, block b).  Thread per segment.
__global__ __launch_bounds__(kBlock) void k_rb_chunks(const int32_t* __restrict__ off,
                                                      int64_t cells, int nb, int chunk,
                                                      int32_t* __restrict__ cblk) {
  const int64_t sg = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (sg >= cells) return;
  const int b = (int)(sg % nb);
  for (int32_t c = off[sg] / chunk; c < off[sg + 1] / chunk; ++c) cblk[c] = b;
}

// H [n, ld_h] -> the split layout: main [n, fs] (whole lines per row) and rem [n, 4]
// (columns fs..f-1, zero padded; times rem_scale[row] when given).  Thread per 16-B piece of a row (fs / 4 + 1 pieces).
__global__ __launch_bounds__(kBlock) void k_split_copy(const float* __restrict__ h, int64_t ld_h,
                                                       int64_t n, int f, int fs, int rw,
                                                       float* __restrict__ main,
                                                       float* __restrict__ rem,
                                                       const float* __restrict__ rem_scale) {
  const int rp = rw / 4;  // 16-B pieces per remainder row
  const int pieces = fs / 4 + rp;
  const int64_t total = n * pieces;
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kBlock) {
    const int64_t row = t / pieces;
    const int q = (int)(t - row * pieces);
    const float* p = h + row * ld_h + 4 * q;
    if (q < fs / 4) {
      *reinterpret_cast<f32x4*>(main + row * fs + 4 * q) = ld_nt<f32x4>(p);
    } else {
      // a remainder piece: a full 16-B read stays inside the row's storage except possibly
      // on the buffer's last row, which reads exactly its nv valid columns; a piece wholly
      // past column f (rw > 4 only) reads nothing
      const int j = q - fs / 4;
      const int nv = f - fs - 4 * j;
      f32x4 v = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (nv <= 0) {
      } else if (nv >= 4 || row + 1 < n) {
        v = ld_nt<f32x4>(p);
        if (nv < 4) v.w = 0.0f;
        if (nv < 3) v.z = 0.0f;
        if (nv < 2) v.y = 0.0f;
      } else {
        v.x = p[0];
        if (nv > 1) v.y = p[1];
        if (nv > 2) v.z = p[2];
      }
      if (rem_scale) {  // unit graph: the remainder buffers hold dr o Z_rem
        const float d = rem_scale[row];
        v = f32x4{d * v.x, d * v.y, d * v.z, d * v.w};
      }
      *reinterpret_cast<f32x4*>(rem + row * rw + 4 * j) = v;
    }
  }
}

template <int EPI, bool VF, int LPE>
hipError_t launch_rem(dim3 grid, dim3 block, size_t lds, hipStream_t s, const StepArgs& a,
                      const RemLayout& L) {
  constexpr int U = LPE == 4 ? kRemUW16 : kRemU;
  static const hipError_t attr = hipFuncSetAttribute(  // > 64 KiB of dynamic LDS, once
      reinterpret_cast<const void*>(k_rem_persist<EPI, U, VF, LPE>),
      hipFuncAttributeMaxDynamicSharedMemorySize, kRemLdsBytes);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_rem_persist<EPI, U, VF, LPE>), grid, block, lds, s, a, L);
  return hipGetLastError();
}

template <int EPI, bool VF>
hipError_t launch_rem_lpe(int lpe, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                          const StepArgs& a, const RemLayout& L) {
  switch (lpe) {
    case 1: return launch_rem<EPI, VF, 1>(grid, block, lds, s, a, L);
    case 2: return launch_rem<EPI, VF, 2>(grid, block, lds, s, a, L);
    case 4: return launch_rem<EPI, VF, 4>(grid, block, lds, s, a, L);
    default: return hipErrorInvalidValue;
  }
}

// Source blocks between workgroup barriers of the pass of width 4 lpe (0: none).  The W8 and
// W16 passes sweep the table in 2-4 row passes, and without barriers the CU's oldest-first
// arbitration lets its fast waves run ahead across them; a barrier every 32 blocks (and so at
// every row pass's end) re-aligns the waves: W16 1.94 -> 1.77 ms, W8 1.21 -> 1.10 ms on
// products-synth, L2 hits 28 -> 52 % (W16).  Every block costs more at the barrier than the
// misses save (2.26 ms), and the single-pass W4 pass gains nothing (0.766 against 0.769 ms);
// profiles/r4_sync_ab.txt.  APPNP_REM_SYNC_W4 / _W8 / _W16 (tuning overrides, APPNP_TUNING=1).
int rem_sync_blocks(int lpe) {
  static const int w4 = tuning_env("APPNP_REM_SYNC_W4", 0),
                   w8 = tuning_env("APPNP_REM_SYNC_W8", 32),
                   w16 = tuning_env("APPNP_REM_SYNC_W16", 32);
  return lpe == 1 ? w4 : lpe == 2 ? w8 : w16;
}

// fp32 copy of dinv (the unit graph's row / column scales)
__global__ __launch_bounds__(kBlock) void k_dinv_f32(const double* __restrict__ d, int64_t n,
                                                     float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) out[i] = (float)d[i];
}

#ifdef APPNP_TESTING
// test hooks, compiled into libppnp_amd_test.so only (make test-lib): read at every call
int test_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}
#endif

}  // namespace

// The regrouped copy of A_hat for the persistent remainder pass.  Best-effort at the caller
// (appnp_graph_create_rows): APPNP_ENOTSUP / APPNP_ERANGE / APPNP_ENOMEM leave the graph
// without it, and appnp_propagate gathers whole rows.
int graph_build_source_blocks(appnp_graph* g, int lpe, const int32_t* a_indptr,
                              const int32_t* a_indices, int64_t a_nnz, hipStream_t s) {
  // the held rows [row_lo, row_hi) in row groups; source blocks over all n global columns
  const int64_t rows = g->row_hi - g->row_lo;
  const bool partial = g->row_lo != 0 || rows != g->n;
  if (lpe != 1 && lpe != 2 && lpe != 4) return APPNP_EINVAL;
  const int chunk = kRemChunk / lpe;     // entries per chunk (one per lpe lanes)
  const int max_rg = kRemMaxRg / lpe;    // rows per wave group: 16 x max_rg x 16 lpe B of LDS
  // APPNP_SB_ROWS: tuning override of the block size (a power of two, 2^10..2^20 rows)
  static const int br_log2 = [] {
    const int x = tuning_env("APPNP_SB_ROWS", 1 << kSourceBlockLog2);
    int l = 10;
    while (l < kRemColBits && (1 << l) < x) ++l;
    return l;
  }();
  const int64_t nb = std::max<int64_t>(1, (g->n + (1LL << br_log2) - 1) >> br_log2);
#ifdef APPNP_TESTING
  // APPNP_SB_MAX_BLOCKS (test library): a lower block limit, so a test can take the best-effort
  // fallback on a small graph
  const int max_blocks =
      std::min(kWalkMaxBlocks, std::max(1, test_env("APPNP_SB_MAX_BLOCKS", kWalkMaxBlocks)));
#else
  const int max_blocks = kWalkMaxBlocks;
#endif
  if (nb > max_blocks) return APPNP_ENOTSUP;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return APPNP_EDEVICE;
  const int64_t slots = (int64_t)cus * kRemWaves;
  const int64_t passes = std::max<int64_t>(1, (rows + slots * max_rg - 1) / (slots * max_rg));
  const int64_t rg = std::max<int64_t>(1, (rows + passes * slots - 1) / (passes * slots));
  const int64_t cells = passes * nb * slots;
  if (cells + 1 > INT32_MAX) return APPNP_ERANGE;
  int rc = APPNP_OK;
  int32_t* cnt = nullptr;
  int64_t *bsum = nullptr, *tot = nullptr;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && rc == APPNP_OK)
      rc = (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? APPNP_ENOMEM
                                                                       : APPNP_EDEVICE;
    return rc == APPNP_OK;
  };
  // a unit graph (every entry of A+I is 1) stores no values: A_hat_ij = dl_i dr_j.
  // APPNP_REM_VF=0 keeps the values (tuning override)
  const bool vf = g->unit && tuning_env("APPNP_REM_VF", 1) != 0;
  const int64_t n_groups = passes * slots;
  const unsigned grid = (unsigned)((n_groups + kWalkWaves - 1) / kWalkWaves);
  const size_t lds = (size_t)kWalkWaves * nb * sizeof(int32_t);
  int64_t h_tot[2] = {0, 0};  // padded entries, near entries
  if (ok(hipMalloc(&g->rb_off, (cells + 1) * sizeof(int32_t))) &&
      ok(hipMalloc(&cnt, cells * sizeof(int32_t))) &&
      ok(hipMalloc(&bsum, scan_partials(cells) * sizeof(int64_t))) &&
      ok(hipMalloc(&tot, 2 * sizeof(int64_t))) &&
      ok(hipMemsetAsync(tot, 0, 2 * sizeof(int64_t), s))) {
    hipLaunchKernelGGL(k_rb_walk<false>, dim3(grid), dim3(kBlock), lds, s, g->row_ptr, g->col,
                       g->val, rows, g->row_lo, (int)rg, (int)nb, br_log2, chunk, n_groups, cnt,
                       nullptr, nullptr, nullptr,
                       reinterpret_cast<unsigned long long*>(tot + 1));
    if (partial && a_nnz > 0 && ok(hipGetLastError()) &&
        ok(hipMemsetAsync(tot + 1, 0, sizeof(int64_t), s))) {
      // the near count of the WHOLE A (replacing the held rows' count of the walk)
      const int64_t nblk = std::min<int64_t>((g->n + kBlock - 1) / kBlock, 4096);
      hipLaunchKernelGGL(k_near_all, dim3((unsigned)std::max<int64_t>(1, nblk)), dim3(kBlock), 0,
                         s, a_indptr, a_indices, g->n,
                         reinterpret_cast<unsigned long long*>(tot + 1));
    }
    if (ok(hipGetLastError()) && ok(exclusive_scan(cnt, cells, g->rb_off, bsum, tot, s)) &&
        ok(hipMemcpyAsync(h_tot, tot, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, s)) &&
        ok(hipStreamSynchronize(s))) {
      // padded total: the int32 segment offsets must hold it
      if (h_tot[0] > INT32_MAX) rc = APPNP_ERANGE;
    }
    const int64_t total = std::max<int64_t>(1, h_tot[0]);
#ifdef APPNP_TESTING
    // APPNP_SB_TEST_OOM (test library): ask for an impossible size, so the best-effort ENOMEM
    // path runs with a real failing hipMalloc
    const size_t ent_bytes = test_env("APPNP_SB_TEST_OOM", 0) ? (size_t)1 << 60
                                                              : (size_t)total * sizeof(uint32_t);
#else
    const size_t ent_bytes = (size_t)total * sizeof(uint32_t);
#endif
    if (rc == APPNP_OK && ok(hipMalloc(&g->rb_ent, ent_bytes)) &&
        (vf || ok(hipMalloc(&g->rb_val, total * sizeof(float)))) &&
        ok(hipMemsetAsync(g->rb_ent, 0xff, total * sizeof(uint32_t), s)) &&  // kRemNone
        (vf || ok(hipMemsetAsync(g->rb_val, 0, total * sizeof(float), s))) &&
        (!vf || ok(hipMalloc(&g->rb_dl, std::max<int64_t>(1, rows) * sizeof(float)))) &&
        (!vf || g->mode != APPNP_NORM_SYM ||
         ok(hipMalloc(&g->rb_dr, std::max<int64_t>(1, g->n) * sizeof(float)))) &&
        ok(hipMalloc(&g->rb_cblk, std::max<int64_t>(1, total / chunk) * sizeof(int32_t)))) {
      hipLaunchKernelGGL(k_rb_walk<true>, dim3(grid), dim3(kBlock), lds, s, g->row_ptr, g->col,
                         g->val, rows, g->row_lo, (int)rg, (int)nb, br_log2, chunk, n_groups,
                         nullptr,
                         g->rb_off,
                         g->rb_ent, g->rb_val, nullptr);
      if (vf && ok(hipGetLastError())) {
        // dl: the held rows' scale (local index); dr: every column's (global index)
        if (rows > 0)
          hipLaunchKernelGGL(k_dinv_f32, dim3((unsigned)((rows + kBlock - 1) / kBlock)),
                             dim3(kBlock), 0, s, g->dinv + g->row_lo, rows, g->rb_dl);
        if (g->rb_dr && g->n > 0)
          hipLaunchKernelGGL(k_dinv_f32, dim3((unsigned)((g->n + kBlock - 1) / kBlock)),
                             dim3(kBlock), 0, s, g->dinv, g->n, g->rb_dr);
      }
      if (ok(hipGetLastError()))
        hipLaunchKernelGGL(k_rb_chunks, dim3((unsigned)((cells + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, s, g->rb_off, cells, (int)nb, chunk, g->rb_cblk);
      // near entries per entry of A_hat: the held rows' (full graph) or the whole graph's
      // (row partition: A's off-diagonal entries + the n diagonal ones)
      const double denom = partial ? (double)(a_nnz + g->n) : (double)g->nnz_hat;
      if (ok(hipGetLastError()) && ok(hipStreamSynchronize(s)))
        g->near_frac = denom > 0 ? (double)h_tot[1] / denom : 0.0;
    }
  }
  if (cnt) (void)hipFree(cnt);
  if (bsum) (void)hipFree(bsum);
  if (tot) (void)hipFree(tot);
  if (rc != APPNP_OK) {
    // the graph stays usable without the copy: clear the failed call's error from this
    // thread's last-error slot, or the next hipGetLastError (a launch check here or in the
    // caller's framework) would report it as its own
    (void)hipGetLastError();
    if (g->rb_off) (void)hipFree(g->rb_off);
    if (g->rb_ent) (void)hipFree(g->rb_ent);
    if (g->rb_val) (void)hipFree(g->rb_val);
    if (g->rb_cblk) (void)hipFree(g->rb_cblk);
    if (g->rb_dl) (void)hipFree(g->rb_dl);
    if (g->rb_dr) (void)hipFree(g->rb_dr);
    g->rb_dl = g->rb_dr = nullptr;
    g->rb_off = nullptr;
    g->rb_ent = nullptr;
    g->rb_val = nullptr;
    g->rb_cblk = nullptr;
    return rc;
  }
  g->rb_total = h_tot[0];
  g->rb_nb = (int32_t)nb;
  g->rb_br_log2 = br_log2;
  g->rb_grid = cus;
  g->rb_slots = (int32_t)slots;
  g->rb_rg = (int32_t)rg;
  g->rb_passes = (int32_t)passes;
  g->rb_lpe = lpe;
  return APPNP_OK;
}

// One iteration of the remainder columns: R = (M_k o A_hat) Z_rem over all source blocks in
// one persistent launch (k_rem_persist), epilogue included.  a: the iteration's StepArgs
// (dropout key, n_rows, scale, alpha); z_rem [n, 4]; h_rem = H + fs; out / ld_out / nv: where
// the nv valid columns of Z_{k+1} go.  epi = EPI_BWD (adjoint): h_rem / ld_h are dH's
// remainder columns, accumulated into; out (G_k's remainder) may be null.
hipError_t launch_remainder(const appnp_graph* g, const StepArgs& a_in, int epi,
                            const float* z_rem, const float* h_rem, int64_t ld_h, float* out,
                            int64_t ld_out, int nv, bool to_rem, hipStream_t s) {
  StepArgs a = a_in;
  a.zin = z_rem;
  a.aux = nullptr;
  if (epi == EPI_BWD) {  // h_rem / ld_h: dH's remainder columns, accumulated into
    a.h = nullptr;
    a.rem_dh = const_cast<float*>(h_rem);
    a.ld_rem_dh = ld_h;
  } else {
    a.h = h_rem;
    a.ld_h = ld_h;
  }
  a.out = out;
  a.ld_out = ld_out;
  a.f = nv;
  if (a.n_rows <= 0) return hipSuccess;
  const bool vf = g->rb_val == nullptr;
  const int lpe = g->rb_lpe;
  const int sync = rem_sync_blocks(lpe);
  RemLayout L{g->rb_off, g->rb_ent, g->rb_val, g->rb_cblk, g->rb_dl, g->rb_dr, g->rb_nb,
              g->rb_br_log2, g->rb_slots, g->rb_rg, g->rb_passes, to_rem ? 1 : 0, sync};
  const size_t lds = (size_t)kRemWaves * g->rb_rg * lpe * sizeof(f32x4);
  const dim3 grid((unsigned)g->rb_grid), block(kRemThreads);
  if (epi == EPI_BWD)
    return vf ? launch_rem_lpe<EPI_BWD, true>(lpe, grid, block, lds, s, a, L)
              : launch_rem_lpe<EPI_BWD, false>(lpe, grid, block, lds, s, a, L);
  return vf ? launch_rem_lpe<EPI_FWD, true>(lpe, grid, block, lds, s, a, L)
            : launch_rem_lpe<EPI_FWD, false>(lpe, grid, block, lds, s, a, L);
}

hipError_t launch_split_copy(const float* h, int64_t ld_h, int64_t n, int64_t f, int64_t fs,
                             int64_t rw, float* main, float* rem, const float* rem_scale,
                             hipStream_t s) {
  const int64_t total = n * (fs / 4 + rw / 4);
  if (total <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((total + kBlock - 1) / kBlock, 1 << 20);
  hipLaunchKernelGGL(k_split_copy, dim3((unsigned)blocks), dim3(kBlock), 0, s, h, ld_h, n,
                     (int)f, (int)fs, (int)rw, main, rem, rem_scale);
  return hipGetLastError();
}

}  // namespace appnp
