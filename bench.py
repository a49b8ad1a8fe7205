#!/usr/bin/env python
"""Benchmark of the APPNP propagation hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload products-synth]

A "step" is one full propagation call -- K=10 fused SpMM+AXPBY iterations over the whole
graph (appnp_propagate, or the partitioned multi-GPU loop) -- on synthetic input that is
resident in HBM before the timed region.  value = nodes * F * K * steps / time (whole job).

N > 1 (launched by torch.distributed.run, one rank per GPU): the ranks form an R x C layout
(ppnp_amd/dist.py): C feature slabs need no exchange, R row groups
exchange their Z shards over RCCL every iteration.  --layout auto measures every candidate
layout of ppnp_amd.dist.candidate_layouts with the full protocol (W warm-up steps, then exactly
K timed steps bracketed by barrier + synchronize, max over ranks, parity of the result) and
prints the fastest one whose parity holds.  The candidate without a data-path exchange (the
column layout) is measured first, and every later candidate runs under a deadline
(--candidate-timeout): if an exchange stalls, the RCCL communicators are aborted, rank 0
prints the best line measured so far, and every rank exits -- the scaling run always gets a
line unless the exchange-free layout itself fails.  --run-budget bounds the whole run: no
candidate starts with less than MIN_CANDIDATE_S of it left, and a running one is cut short.

Extra JSON fields:
  roofline      HBM roofline of the iteration's kernels on one rank: algorithmic bytes per
                iteration B_iter = 4(rows+1) + 8 nnz(A_hat rows) + (n + 2 rows) F s (SURVEY.md
                section 8(d), restricted to the rank's share) / the average iteration time,
                measured with HIP events on the launch stream; peak 8 TB/s.  ``ceiling`` is
                the access-pattern floor of the iteration time (line requests beyond L2 at the
                fastest measured random-line rate, the remainder pass's count floor;
                exchange at the xGMI link peak).  ``traffic``: committed PMC bytes of the
                rank's kernels.  ``box_line_rate``: this GPU's random-line rate, probed right
                before the timed region.  ``kernel_ms``: every launch of one untimed
                propagation right after the timed region, timed by the library's per-launch
                timer (appnp_kernel_timer_*), per kind and per launch.
  device        the GPU the line ran on: PCI address, HBM vendor, board id, VBIOS, clocks.
  cpu_baseline  the oracle's torch.sparse.mm CPU loop (oracle/ppnp_oracle.py) on the same
                graph and H, all K iterations, rank 0 (N = 1: after the timed region; N > 1:
                once, before the first candidate).
  parity        the timed Z_K against the CPU loop's Z_K: N = 1 the whole result, N > 1 every
                rank's block (max over ranks; also printed as ``parity_cpu``).
"""

from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "APPNP K=10 propagated node-feats/sec; achieved HBM GB/s vs peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level parameters)
# random row-gather rate: 53-60 G cache-line requests/s for 64-512 B rows from 64 MB-1 GB
# tables, Infinity-Cache hits or not (tools/gather_probe.hip, profiles/r1_gather_probe.txt).
# The ceiling uses the fastest measured rate, so it is a lower bound on the iteration time.
GATHER_LINE_CEILING = 60.0
# xGMI: 7 links per GPU at 76.8 GB/s per direction (153.6 GB/s bidirectional)
XGMI_IN_GBS = 7 * 76.8
# The persistent remainder pass (appnp_blocks.hip): its floor from COUNTS, independent of the
# pass's own timings (round 4 priced it at its own fastest time, so the
# 8-rank column slab's ceiling certified the kernel against itself).  Two terms, the larger wins:
#   * fill: every XCD's L2 must take in the whole remainder table once per row pass --
#     row passes x 8 XCDs x n x 16 LPE bytes / 128-B lines, at the fastest measured random-line
#     rate (GATHER_LINE_CEILING) -- plus the entry stream (4 B per entry: value-free) at the HBM
#     peak, both from beyond L2;
#   * requests: one L2 request per nonzero (an entry's 16 LPE bytes lie in one line) at the rate
#     of the W4 pass with every gather forced to an L2-resident row: 0.665 ms for products-synth's
#     126,165,965 nonzeros, entry stream included = 189.7 G requests/s.
# Row passes: ceil(rows / (CUs x 16 waves x 640 / LPE rows)), as graph_build_source_blocks has it.
REM_L2_REQ_RATE = 126_165_965 / 0.665e-3 / 1e9
REM_L2_REQ_SOURCE = ("DESIGN.md 4.2: the W4 pass with every gather an L2 hit, 0.665 ms for "
                     "126.2 M nonzeros")
XCDS, CUS, REM_WAVES, REM_ROWS_LPE1 = 8, 256, 16, 640
# N > 1: the whole run's wall budget, below the driver's 600 s bench timeout with
# room for the launcher, the first `import torch` of a fresh box and the teardown; a candidate
# is not started with less than MIN_CANDIDATE_S of it left
RUN_BUDGET_S = 420.0
MIN_CANDIDATE_S = 20.0
# N > 1: the largest oracle Z_K (fp32 bytes) rank 0 sends to every rank for the parity check
# (products-synth: 0.98 GB, ~2-4 s over gloo on one host)
PARITY_BCAST_MAX_BYTES = 4 << 30
# The in-library line-rate probe run before the timed region (appnp_line_rate_probe): random
# 128-B lines gathered from the bench's own H buffer, ~20 ms
PROBE_LINES = 1 << 30


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)  # median of >= 20 after 3 warm-ups
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="products-synth")
    p.add_argument("--dtype", default=None, choices=["f32", "bf16"],
                   help="override the workload's storage dtype (non-headline variants)")
    p.add_argument("--features", type=int, default=None,
                   help="override the workload's feature width F (non-headline variants)")
    p.add_argument("--cpu-iters", type=int, default=None,
                   help="iterations of the CPU baseline sample (default K: its Z_K is then the "
                        "parity reference of the GPU result; 0 disables it)")
    p.add_argument("--layout", default="auto",
                   help="multi-GPU layout: auto | row | col | RxC (row groups x column groups)")
    p.add_argument("--emulate", default=None, metavar="P:r",
                   help="single-GPU emulation of rank r of a P-rank --layout (kernel time of "
                        "that rank only, no exchange; NOT a multi-GPU result)")
    p.add_argument("--plan", action="store_true",
                   help="single GPU: replay the K launches as one captured hipGraph "
                        "(appnp_plan_*; for small, launch-bound workloads)")
    p.add_argument("--overlap", action="store_true",
                   help="row layouts: overlap the all-gather with the local-column product")
    p.add_argument("--exchange", default="multipath", choices=["multipath", "group", "native"],
                   help="R x C layouts: relayed exchange over every rank, or one all-gather "
                        "per column group; row layouts: 'native' runs the library's own loop")
    p.add_argument("--pipeline", default="auto", choices=["auto", "on", "off"],
                   help="row layouts with overlap and >= 3 row groups: exchange by one broadcast "
                        "per row shard and run the product per group of arrived shards (auto: "
                        "whenever it applies)")
    p.add_argument("--candidate-timeout", type=float, default=240.0,
                   help="N > 1: seconds one layout candidate (build, warm-up, timed steps, "
                        "parity) may take before the run is ended with the best line so far")
    p.add_argument("--run-budget", type=float, default=RUN_BUDGET_S,
                   help="N > 1: wall seconds, counted from this process's start, after which no "
                        "further candidate starts and a running one is cut short (its deadline "
                        "is the smaller of --candidate-timeout and the budget left); the best "
                        "line so far is printed.  Keep it below the driver's bench timeout "
                        "(600 s); 0 disables it")
    return p.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads(world: int = 1) -> tuple[int, int]:
    """(threads to use, CPUs this process may run on).  BASELINE.md asks for every core; on the
    GPU box the process's share is what OMP_NUM_THREADS names (16 of a much larger machine, whose
    full count os.cpu_count() reports), so that bounds it.  At N > 1 torch.distributed.run sets
    OMP_NUM_THREADS=1 for every rank unless the caller set it; rank 0 runs the CPU leg while the
    other ranks wait at a barrier, so it takes up to 16 of its visible CPUs regardless."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or visible
    if world > 1:
        share = max(share, min(16, visible))
    return max(1, min(visible, share)), visible


def src_digest() -> str:
    """Digest of the HIP sources (ppnp_amd/csrc/srcdigest.py, the same function the Makefile
    compiles into the library): keys the committed PMC traffic to the kernels that made it."""
    import importlib.util

    path = os.path.join(ROOT, "ppnp_amd", "csrc", "srcdigest.py")
    spec = importlib.util.spec_from_file_location("ppnp_srcdigest", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.src_digest(os.path.dirname(path))


def build_info() -> dict:
    """Provenance of the library this process loaded: the source digest
    compiled into it (appnp_build_info) against the digest of the sources in this tree.  A
    library built from other sources reads ``match: false``."""
    from ppnp_amd import _lib

    here = src_digest()
    try:
        lib = _lib.load()
        info = lib.appnp_build_info().decode()
        active = lib.appnp_tuning_overrides().decode()
        names = lib.appnp_tuning_names().decode().split(";")
    except Exception as e:  # noqa: BLE001 -- provenance is reported, never fatal to the line
        return {"library": _lib.LIB_PATH, "info": f"{type(e).__name__}: {e}",
                "library_src": None, "tree_src": here, "match": False, "overrides": None}
    fields = dict(kv.split("=", 1) for kv in info.split(";") if "=" in kv)
    # tuning overrides in effect (APPNP_TUNING=1), and any set but ignored without it
    # (a stray variable must not change kernels silently)
    overrides = dict(kv.split("=", 1) for kv in active.split(";") if "=" in kv)
    ignored = sorted(k for k in names if os.environ.get(k) and k not in overrides)
    return {"library": _lib.LIB_PATH, "info": info, "library_src": fields.get("src"),
            "tree_src": here, "match": fields.get("src") == here,
            "overrides": overrides or None, "overrides_ignored": ignored or None}


def device_info(dev) -> dict:
    """Which GPU this line ran on (round 5, VERDICT r4 #1: the two timing states switch between
    boxes): torch's name / arch / uuid / PCI address, and what the amdgpu driver exposes read-only
    in sysfs for that PCI function -- the HBM vendor, the board's unique id, the VBIOS, and the
    current memory / fabric / shader clock levels -- so lines in the fast and the slow state can be
    told apart by hardware.  Fields that cannot be read are null; never raises."""
    out = {}
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        out = {"name": p.name, "arch": getattr(p, "gcnArchName", None), "pci": bdf,
               "uuid": str(getattr(p, "uuid", "")) or None}
    except Exception as e:  # noqa: BLE001 -- a diagnostic
        return {"error": f"{type(e).__name__}: {e}"}
    base = os.path.join("/sys/bus/pci/devices", out["pci"])
    for key, fname in (("vram_vendor", "mem_info_vram_vendor"), ("unique_id", "unique_id"),
                       ("vbios", "vbios_version"), ("mclk", "pp_dpm_mclk"),
                       ("fclk", "pp_dpm_fclk"), ("sclk", "pp_dpm_sclk")):
        try:
            with open(os.path.join(base, fname)) as fh:
                txt = fh.read().strip()
            if fname.startswith("pp_dpm_"):  # the current level is marked with '*'
                cur = [ln for ln in txt.splitlines() if ln.rstrip().endswith("*")]
                txt = cur[0].split(":", 1)[-1].strip(" *") if cur else txt.replace("\n", "; ")
            out[key] = txt
        except OSError:
            out[key] = None
    return out


def traffic_key(workload, dtype_name, kernel_key, f_local, rows, overlap=False,
                pipeline=False) -> str:
    """Key of the PMC traffic of one rank's iteration: what the rank RUNS -- the workload, the
    dtype, the iteration's kernels, its feature slab width and held rows, the local/remote split
    of overlap mode -- and a digest of the kernel sources.  Not the layout's name: rank r of a
    real P-rank run and ``--emulate P:r`` on one GPU run the same kernels on the same share, so a
    profile of the emulation is the traffic of the real rank (VERDICT r3 missing #3), and a
    profile of other kernels, another share or an older build of them never matches."""
    ov = (":ov" if overlap else "") + (":pipe" if pipeline else "")
    return (f"{workload}:{dtype_name}:{kernel_key}:F{f_local}:rows{rows}{ov}"
            f":src={src_digest()}")


def committed_traffic(key):
    """HBM bytes per iteration from the committed PMC profile of the same command, kernels and
    kernel sources (tools/summarize_profile.py writes profiles/pmc_traffic.json), or None: a
    profile of other kernels or of an older build of them never matches the key."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            return json.load(fh).get(key)
    except (OSError, ValueError):
        return None


def cpu_baseline(graph, H, K, alpha, iters, adj=None, world=1):
    """Time the oracle's CPU torch.sparse.mm APPNP loop on the same operator and H (SURVEY.md
    8(d) CPU baseline (i)); return (the JSON object, Z of the CPU loop).  For N <= 20k also time
    the reference's as-shipped PPNP path, compute_ppr + dense Pi @ H (helpers.py:68-71,
    model.py:63; baseline (ii))."""
    from oracle import ppnp_oracle as O

    threads, visible = cpu_threads(world)
    torch.set_num_threads(threads)
    rp, col, val, _ = graph.csr()
    a_t = torch.sparse_csr_tensor(rp.cpu().long(), col.cpu().long(), val.cpu(),
                                  size=(graph.n, graph.n))
    del rp, col, val
    Hc = H.float().cpu()
    t0 = time.perf_counter()
    Zc = O.appnp_propagate_torch_cpu(a_t, Hc, iters, alpha)
    dt = time.perf_counter() - t0
    n, f = Hc.shape
    res = {
        "value": n * f * iters / dt,
        "unit": "node-feats/s",
        "cores": threads,
        "threads": threads,
        "cpus_visible": visible,
        "cpu_model": cpu_model(),
        "kind": "port",
        "sample": f"full graph, {iters} of K={K} iterations, torch.sparse.mm fp32 CSR "
                  f"(oracle/ppnp_oracle.py appnp_propagate_torch_cpu), {dt:.2f} s",
    }
    if adj is not None and n <= 20000:
        import numpy as np

        t0 = time.perf_counter()
        Pi = O.compute_ppr(adj, alpha)
        t_ppr = time.perf_counter() - t0
        Hn = Hc.double().numpy()
        t0 = time.perf_counter()
        _ = np.asarray(Pi, dtype=np.float32) @ Hn.astype(np.float32)
        t_mm = time.perf_counter() - t0
        res["ppnp_as_shipped"] = {
            "compute_ppr_s": t_ppr,
            "dense_pi_h_s": t_mm,
            "value": n * f / (t_ppr + t_mm),
            "unit": "node-feats/s (one exact propagation, K -> infinity)",
            "sample": "oracle compute_ppr (helpers.py:68-71: dense fp64 inverse) + fp32 Pi @ H",
        }
    return res, Zc


# ---------------------------------------------------------------------------------------------
# roofline of one rank's iteration
# ---------------------------------------------------------------------------------------------


def kernel_plan(F_local, K, remainder_cols, sb):
    """What one iteration runs on this rank: (description, key, fs, r, lpe).  ``remainder_cols``
    is the split the runner actually takes (0: whole rows through the SpMM kernel); ``sb`` the
    graph's source-blocked layout (Graph.source_block_layout)."""
    r = int(remainder_cols) if K >= 2 and sb else 0
    if not r:
        return ("k_step (one fused SpMM launch per iteration)", "k_step", F_local, 0, 1)
    fs = F_local - r
    lpe = sb["width"] // 4
    rem = f"k_rem_persist<W{sb['width']}{',vf' if sb['value_free'] else ''}>"
    if not fs:
        return (f"{rem} on all {F_local} columns (narrow rows: one persistent L2-blocked launch "
                f"per iteration, {sb['row_passes']} row passes)", f"{rem}[0,{F_local})", 0, r,
                lpe)
    return (f"k_step on columns [0, {fs}) + {rem} on the remainder columns [{fs}, {F_local}) "
            "(one persistent L2-blocked launch) per iteration; times are per iteration",
            f"k_step[0,{fs})+{rem}[{fs},{F_local})", fs, r, lpe)


def rank_kernel_plan(runner, K):
    """kernel_plan of what ``runner`` (SingleRunner, PartitionedAPPNP, NativeRowRunner) runs per
    iteration."""
    sb = runner.graph.source_block_layout() if runner.remainder_cols else None
    return kernel_plan(runner.width, K, runner.remainder_cols, sb)


def rank_traffic_key(workload, dtype_name, runner, K) -> str:
    """traffic_key of ``runner``'s iteration: the same for rank r of a real P-rank run and for
    ``--emulate P:r`` (tests/test_bench_roofline.py pins it)."""
    kkey = rank_kernel_plan(runner, K)[1]
    return traffic_key(workload, dtype_name, kkey, runner.width, runner.graph.rows,
                       bool(getattr(runner, "overlap", False)),
                       bool(getattr(runner, "pipeline", False)))


def remainder_floor(n, rows, nnz, lpe):
    """The W = 4 lpe remainder pass's floor from counts (see REM_L2_REQ_RATE): the larger of its
    compulsory L2 fill (+ entry stream) from beyond L2 and its L2 requests at the all-hit rate."""
    slot_rows = CUS * REM_WAVES * (REM_ROWS_LPE1 // lpe)
    passes = max(1, -(-rows // slot_rows))
    fill_lines = passes * XCDS * n * 16 * lpe / 128
    entry_bytes = 4 * nnz
    fill_ms = (fill_lines / (GATHER_LINE_CEILING * 1e9) + entry_bytes / (HBM_PEAK_GBS * 1e9)) * 1e3
    req_ms = nnz / (REM_L2_REQ_RATE * 1e9) * 1e3
    return {"ms": max(fill_ms, req_ms), "fill_ms": fill_ms, "l2_request_ms": req_ms,
            "row_passes": passes, "fill_lines": fill_lines,
            "kind": "count floor (not a measured rate): max(row passes x 8 XCDs x table / 128-B "
                    f"lines at {GATHER_LINE_CEILING} G lines/s + 4 B/entry at the HBM peak, "
                    f"one L2 request per nonzero at {REM_L2_REQ_RATE:.1f} G/s ({REM_L2_REQ_SOURCE}))"}


def roofline(*, n, rows, nnz, F_local, esz, avg_iter_ms, fs, r, lpe, exchange_in_bytes=0,
             kernel="", kernel_key="", traffic=None):
    """The roofline block of one rank.

    achieved = B_iter / iteration time with B_iter = 4(rows+1) + 8 nnz + (n + 2 rows) F s: the
    rank's A_hat rows once, all n rows of its slab of Z_k once (a row-layout rank gathers every
    row), H and Z_{k+1} of its rows once.  For one GPU this is SURVEY 8(d)'s 4(N+1)+8nnz+3NFs.

    ceiling = the access-pattern floor of the iteration time, the largest of
      * the SpMM kernel's line requests beyond L2 at the fastest measured random-line rate --
        ``lines_per_nonzero`` gathered 128-B lines per nonzero (whole lines of the fs main
        columns, or all of a whole row) plus its streamed bytes (CSR, H, Z) / 128 -- plus, with
        split rows, the remainder pass's floor from counts (``remainder_floor``: its L2 fill per
        row pass and its L2 requests, not its own measured time);
      * a row layout's exchange: the bytes landing here / the xGMI links' peak;
      * B_iter at the HBM peak (the roofline itself), so ceiling.frac <= 1.
    So frac <= ceiling.frac <= 1 on a uniform random graph, up to the probe's own spread; a
    graph with gather locality (L2 hits) can beat the line bound, and then the ceiling is
    clamped to the measured time and says so."""
    from ppnp_amd.dist import _avg_lines, line_ld

    s = esz
    b_iter = 4 * (rows + 1) + 8 * nnz + (n + 2 * rows) * F_local * s
    achieved = b_iter / (avg_iter_ms * 1e-3) / 1e9 if avg_iter_ms > 0 else 0.0
    if r:
        lpn = fs * s // 128
        stream = 4 * (rows + 1) + 8 * nnz if fs else 0
        dense = 2 * rows * fs * s
    else:
        ld = line_ld(F_local, s)
        lpn = _avg_lines(F_local * s, ld * s)
        stream = 4 * (rows + 1) + 8 * nnz
        dense = 2 * rows * ld * s
    lines = nnz * lpn + (stream + dense) / 128
    width = 4 * lpe
    rem = remainder_floor(n, rows, nnz, lpe) if r else None
    rem_ms = rem["ms"] if r else 0.0
    compute_ms = lines / (GATHER_LINE_CEILING * 1e9) * 1e3 + rem_ms
    exchange_ms = exchange_in_bytes / (XGMI_IN_GBS * 1e9) * 1e3
    hbm_ms = b_iter / (HBM_PEAK_GBS * 1e9) * 1e3
    ceil_ms = max(compute_ms, exchange_ms, hbm_ms)
    note = ("a uniform random graph gathers whole cache lines per nonzero, so the "
            "compulsory-byte fraction is capped at ceiling.frac; 60 % of the compulsory-byte "
            "roofline is out of reach for it on one GPU")
    clamped = avg_iter_ms > 0 and ceil_ms > avg_iter_ms
    if clamped:
        ceil_ms = avg_iter_ms
        note = ("measured faster than the uniform-gather bound (gather locality: L2 hits), so "
                "the ceiling is the measured time")
    line_rate = lines / (avg_iter_ms * 1e-3) / 1e9 if avg_iter_ms > 0 else 0.0
    tgbs = traffic / (avg_iter_ms * 1e-3) / 1e9 if traffic and avg_iter_ms > 0 else None
    return {
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "traffic_source": "profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                          "passes of this command, kernels and kernel sources (key "
                          "roofline.traffic_key), gfx950-corrected; null when none matches",
        "traffic_GBs": tgbs,
        "traffic_frac": tgbs / HBM_PEAK_GBS if tgbs else None,
        "gather_line_rate": {
            "lines_per_iter": lines,
            "achieved_G_lines_s": line_rate,
            "ceiling_G_lines_s": GATHER_LINE_CEILING,
            "frac": line_rate / GATHER_LINE_CEILING,
            "ceiling_source": "tools/gather_probe.hip, profiles/r1_gather_probe.txt",
        },
        "kernel": kernel,
        "kernel_key": kernel_key,
        "bytes_per_launch": b_iter,
        "avg_launch_ms": avg_iter_ms,
        "ceiling": {
            "ms_per_iter": ceil_ms,
            "frac": b_iter / (ceil_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if ceil_ms > 0 else None,
            "lines_per_nonzero": lpn,
            "remainder_l2_requests_per_nonzero": lpe if r else 0,
            "compute_ms": compute_ms,
            "remainder_pass_ms": rem_ms,
            "remainder_pass_floor": rem,
            "exchange_ms": exchange_ms,
            "hbm_ms": hbm_ms,
            "exchange_in_bytes": exchange_in_bytes,
            "clamped_to_measured": clamped,
            "basis": f"max of: {lines:.4g} line requests per iteration at "
                     f"{GATHER_LINE_CEILING} G lines/s"
                     + (f" + the W{width} remainder pass's count floor for {nnz:.4g} "
                        f"nonzeros ({rem['row_passes']} row "
                        f"pass{'' if rem['row_passes'] == 1 else 'es'}; remainder_pass_floor)"
                        if r else "")
                     + f"; exchange {exchange_in_bytes / 1e6:.4g} MB in at "
                       f"{XGMI_IN_GBS:.0f} GB/s; B_iter at the HBM peak",
        },
        "note": note,
    }


# ---------------------------------------------------------------------------------------------
# timing protocol
# ---------------------------------------------------------------------------------------------


def time_steps(run, stream, steps, warmup, world, ctl):
    """W untimed warm-up steps, then exactly ``steps`` timed steps bracketed by barrier +
    synchronize on both sides; HIP events on the launch stream give the device time and the
    spread of the steps.  Max over ranks."""
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier(group=ctl)
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(steps):
        run()
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier(group=ctl)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = evs[0].elapsed_time(evs[-1])
    steps_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    if world > 1:
        t = torch.tensor([wall, dev_ms], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=ctl)
        wall, dev_ms = float(t[0]), float(t[1])
    return wall, dev_ms, steps_ms


def kernel_split(run, device, K, iteration_ms):
    """roofline.kernel_ms: the device time of every launch of ONE untimed propagation, run right
    after the timed region with the library's per-launch timer (appnp_kernel_timer_*: a HIP event
    on the launch stream after each launch; no profiler, which changed the timing state in round
    3), summarised per kind and per iteration beside the timed region's own iteration time
    (VERDICT r4 #1).  ``sum_of_kernels`` below ``iteration`` means the timed launches ran faster
    than the instrumented ones; above it, that they overlapped without the events between them."""
    from ppnp_amd.ops import kernel_times

    try:
        torch.cuda.synchronize(device)
        t = kernel_times(run, device)
    except Exception as e:  # noqa: BLE001 -- a diagnostic, not the measurement
        log(f"[bench] kernel split failed: {type(e).__name__}: {e}")
        return None
    if not t:
        # a replayed plan (--plan) records nothing: say so instead of empty stats
        return {"note": "no launches recorded (a captured hipGraph replays without the "
                        "library's per-launch events)", "iteration": iteration_ms}
    by = {}
    for kind, ms in t:
        by.setdefault(kind, []).append(ms)

    def stats(v):
        return ({"mean": sum(v) / len(v), "min": min(v), "max": max(v), "launches": len(v)}
                if v else None)

    total = sum(ms for kind, ms in t if kind != "xchg")
    return {
        "main": stats(by.get("step", []) + by.get("local", []) + by.get("remote", [])),
        "local": stats(by.get("local", [])),
        "remote": stats(by.get("remote", [])),
        "rem": stats(by.get("rem", [])),
        "copy": stats(by.get("copy", [])),
        "xchg": stats(by.get("xchg", [])),
        "sum_of_kernels": total / K if K else total,
        "iteration": iteration_ms,
        "launches": [kind for kind, _ in t],
        "ms_per_launch": [round(ms, 5) for _, ms in t],
        "source": "appnp_kernel_timer_begin/_end (include/ppnp_amd.h): one untimed propagation "
                  "after the timed region, HIP events right before and after every launch on "
                  "its stream (no wait before a launch is counted in it); main = the SpMM "
                  "kernel (local + remote halves on a row-partitioned graph), rem = the "
                  "remainder pass, copy = the split copy (once per call), xchg = the library "
                  "row loop's exchange calls (not in sum_of_kernels); sum_of_kernels and "
                  "iteration are ms per iteration",
    }


class Deadline:
    """Wall-clock deadline of one layout candidate.  If it expires, ``on_expire`` runs on the
    timer thread (it never returns: it ends the process).  ``finish`` disarms it; the lock makes
    finish and expiry mutually exclusive."""

    def __init__(self, seconds, on_expire):
        self.lock = threading.Lock()
        self.done = False
        self.on_expire = on_expire
        self.timer = threading.Timer(seconds, self._fire)
        self.timer.daemon = True

    def _fire(self):
        with self.lock:
            if self.done:
                return
            self.on_expire()

    def __enter__(self):
        self.timer.start()
        return self

    def __exit__(self, *exc):
        with self.lock:
            self.done = True
        self.timer.cancel()
        return False


def _abort_rccl():
    """Abort every process group (ncclCommAbort for RCCL ones): stalled collective kernels
    exit, so the process can end without waves left spinning on the GPU."""
    try:
        torch.distributed.distributed_c10d._abort_process_group()
    except Exception as e:  # noqa: BLE001 -- best effort on the way out
        log(f"[bench] process-group abort: {type(e).__name__}: {e}")


def process_age_s() -> float:
    """Seconds since this process started (the run budget's clock): the kernel's start time of
    the process, so the first ``import torch`` of a fresh box (1-2 minutes) counts too.  A start
    time that puts the process more than 15 minutes before this module's import (a clock the
    container does not share) is not trusted: then the import is the start, plus 2 minutes."""
    since_import = time.monotonic() - _T_IMPORT
    try:
        import psutil

        age = time.time() - psutil.Process().create_time()
    except Exception:  # noqa: BLE001 -- psutil missing
        return since_import
    return age if since_import <= age <= since_import + 900.0 else since_import + 120.0


_T_IMPORT = time.monotonic()


def run_candidates(cands, measure, ctl, timeout_s, emit, name_of, rank, world,
                   abort=_abort_rccl, exit_fn=os._exit, exchanges=lambda cand: False,
                   budget_s=0.0, age=process_age_s):
    """Measure every candidate in order and return (best result, {name: ms per step or None}).

    ``measure(cand)`` builds the candidate, times it (``time_steps``), checks parity and returns
    its result dict (``ms_per_step``, ``parity.ok``).  A candidate that raises on any rank
    (agreed over the gloo control group ``ctl``, which an RCCL error cannot poison) or fails
    parity is recorded and skipped.  Every candidate after the first runs under a deadline of
    ``timeout_s``: on expiry the RCCL communicators are aborted, rank 0 ``emit``s the best
    result so far (autotune marked "timeout") and the process ends through ``exit_fn`` -- the
    same on every rank, whose deadlines expire together.  The first candidate is normally the
    layout without a data-path exchange, which needs no deadline; one that ``exchanges`` (row
    groups forced by memory: it brings RCCL up) gets one too.

    ``budget_s`` > 0 bounds the whole run: before every candidate after the
    first, the ranks agree on the largest ``age()`` (seconds since process start) over the
    control group; with less than MIN_CANDIDATE_S of the budget left, this and every later
    candidate are recorded as "skipped: run budget" and the best line so far is returned;
    otherwise the candidate's deadline is the smaller of ``timeout_s`` and the budget left."""
    best, times = None, {}
    for i, cand in enumerate(cands):
        name = name_of(cand)
        cand_timeout = timeout_s
        if budget_s > 0 and i > 0:
            t = torch.tensor([age()], dtype=torch.float64)
            if world > 1:
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=ctl)
            left = budget_s - float(t[0])
            if left < MIN_CANDIDATE_S:
                for rest in cands[i:]:
                    times[name_of(rest)] = "skipped: run budget"
                if rank == 0:
                    log(f"[bench] run budget of {budget_s:.0f} s nearly spent ({left:.0f} s "
                        f"left): skipping {len(cands) - i} candidate(s)")
                break
            cand_timeout = min(timeout_s, left) if timeout_s > 0 else left
        if rank == 0:
            log(f"[bench] candidate {name}: building and timing")

        def expire(name=name, cand_timeout=cand_timeout):
            log(f"[bench] candidate {name} passed its {cand_timeout:.0f} s deadline on rank "
                f"{rank}: aborting the exchange, keeping the best line so far")
            t = threading.Thread(target=abort, daemon=True)
            t.start()
            t.join(30)
            times[name] = "timeout"
            if rank == 0 and best is not None:
                best["config"]["autotune_ms_per_step"] = dict(times)
                emit(best)
            exit_fn(0 if best is not None else 3)

        res, err = None, ""
        guard = (Deadline(cand_timeout, expire)
                 if cand_timeout > 0 and (i > 0 or exchanges(cand)) else None)
        if guard:
            guard.__enter__()
        try:
            try:
                res = measure(cand)
            except Exception as e:  # noqa: BLE001 -- reported and agreed on below
                err = f"{type(e).__name__}: {e}"
            failed = torch.tensor([1.0 if err else 0.0], dtype=torch.float64)
            if world > 1:
                try:
                    torch.distributed.all_reduce(failed, op=torch.distributed.ReduceOp.MAX,
                                                 group=ctl)
                except Exception as e:  # noqa: BLE001
                    # a peer is gone -- its deadline ended it while this rank had already
                    # failed or finished the candidate: end the same way, with the best line
                    log(f"[bench] candidate {name}: agreement failed on rank {rank} "
                        f"({type(e).__name__}: {e}); a peer has ended")
                    if guard:
                        guard._fire()  # unless finish() won the lock, this never returns
                    else:
                        expire()
                    raise
        finally:
            if guard:
                guard.__exit__(None, None, None)
        if float(failed) != 0.0:
            times[name] = None
            log(f"[bench] candidate {name}: FAILED on rank {rank}"
                + (f": {err}" if err else " (another rank failed)"))
            continue
        ok = res.get("parity", {}).get("ok", True)
        times[name] = res["ms_per_step"]
        if rank == 0:
            log(f"[bench] candidate {name}: {res['ms_per_step']:.3f} ms per step"
                + ("" if ok else " -- PARITY FAILURE, not eligible"))
        if ok and (best is None or res["ms_per_step"] < best["ms_per_step"]):
            best = res
    if best is None:
        raise RuntimeError(f"every candidate layout failed: {times}")
    best["config"]["autotune_ms_per_step"] = dict(times)
    return best, times


# ---------------------------------------------------------------------------------------------
# runners
# ---------------------------------------------------------------------------------------------


class SingleRunner:
    """One GPU, the whole graph: appnp_propagate (or its captured plan)."""

    def __init__(self, graph, H, K, alpha, dtype, ld, plan=False):
        import ppnp_amd

        self.graph, self.H, self.K, self.alpha = graph, H, K, alpha
        self.width = int(H.shape[1])
        n = graph.n
        self.lo, self.hi, self.f_lo, self.f_hi = 0, n, 0, self.width
        self.Z = torch.empty(n, ld, dtype=dtype, device=H.device)[:, :self.width]
        self.remainder_cols = graph.remainder_cols(self.width, dtype) if K >= 2 else 0
        if plan:
            from ppnp_amd.ops import PropagatePlan

            self._plan = PropagatePlan(graph, H, K, alpha)
            self.Z = self._plan.Z
            self.run = self._plan
        else:
            self.run = lambda: ppnp_amd.propagate_forward(graph, H, K, alpha, out=self.Z)

    @property
    def out(self):
        return self.Z


def cand_name(cand):
    layout, overlap, exchange = cand
    return (f"rows{layout.rows}xcols{layout.cols}" + ("-lines" if layout.lines else "")
            + ("-overlap" if overlap else "")
            + (f"-{exchange}" if (layout.rows > 1 and layout.cols > 1) or exchange == "native"
               else ""))


def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # one GPU per rank; on a box with fewer GPUs than ranks (multi-process rehearsal) ranks
    # share devices round-robin
    ndev = max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(dev)

    import ppnp_amd
    from ppnp_amd import synth
    from ppnp_amd import dist as pdist

    n, m, F, K, alpha, dtype = synth.CONFIGS[args.workload]
    if args.dtype:
        dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    if args.features:
        F = args.features
    dname = "bf16" if dtype == torch.bfloat16 else "f32"
    distributed = world > 1 or args.layout != "auto"
    emu = {}
    lw = world
    if args.emulate:
        P, r = (int(x) for x in args.emulate.split(":"))
        emu = dict(rank=r, world=P, comm=pdist.NullComm())
        lw = P
    esz = 2 if dtype == torch.bfloat16 else 4
    nnz_bound = 2 * m + n  # nnz(A_hat) <= 2 m + n (symmetrised edges + diagonal)
    # the device budget of a candidate: the GPU's memory less what this process holds beside
    # it for the whole run -- the input CSR of A (int32) and H
    held = 4 * (n + 1) + 4 * 2 * m + n * pdist.line_ld(F, esz) * esz
    mem = torch.cuda.get_device_properties(dev).total_memory - held
    if args.layout == "auto" and world > 1 and not args.emulate:
        cands = pdist.candidate_layouts(world, F, n, nnz_bound, esz, mem)
    else:
        layout = (pdist.choose_layout(lw, n, F, nnz_bound, esz, mem) if args.layout == "auto"
                  else pdist.Layout.parse(args.layout, lw))
        cands = [(layout, args.overlap, args.exchange)]
    # The default process group is gloo over host memory: the control plane (barriers, max
    # over ranks, the failure agreement), which an RCCL failure cannot poison.  RCCL carries
    # only the data-path exchange of layouts with row groups, on a group of its own that the
    # first such candidate brings up (pdist.ensure_data_group), inside that candidate's
    # deadline -- so an RCCL that fails to initialise, or stalls, costs that candidate, and the
    # exchange-free column layout measured first still gives the line.  The groups' own
    # watchdog (10 min) outlasts --candidate-timeout, so run_candidates ends a stall first.
    rows = any(c[0].rows > 1 for c in cands)
    data_backend = os.environ.get("PPNP_DIST_BACKEND") or ("nccl" if rows else "gloo")
    if world > 1:
        torch.distributed.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))
    ctl = None  # the default (gloo) group

    t0 = time.perf_counter()
    indptr, indices = synth.graph_for(args.workload, device=dev)
    H = synth.features(n, F, dtype=dtype, device=dev)
    ld = pdist.line_ld(F, esz)
    if ld != F:  # line-aligned rows; H/Z are [N, F] views of [N, ld] buffers
        Hbuf = torch.zeros(n, ld, dtype=dtype, device=dev)
        Hbuf[:, :F] = H
        H = Hbuf[:, :F]
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    if rank == 0:
        log(f"[bench] {args.workload}: N={n} F={F} K={K} dtype={dname}: graph (host numpy "
            f"default_rng) and H generated in {t_gen:.2f}s")

    # the CPU leg: all K iterations by default, at N > 1 too (products-synth: ~11 s at 16
    # threads, once per run), so its Z_K is the parity reference of every line
    cpu_iters = K if args.cpu_iters is None else args.cpu_iters
    adj_small = None
    if n <= 20000 and rank == 0:  # the as-shipped PPNP leg of the CPU baseline needs A
        import numpy as np
        import scipy.sparse as sp

        ip_c, ix_c = indptr.cpu().numpy(), indices.cpu().numpy()
        adj_small = sp.csr_matrix((np.ones(len(ix_c), dtype=np.float32), ix_c, ip_c),
                                  shape=(n, n))

    binfo = build_info()  # which library this process loaded, built from which sources
    extras = {}  # cpu_baseline, attached to whichever line is printed
    ORACLE_REF = "oracle fp32 torch.sparse.mm CPU loop (oracle/ppnp_oracle.py), same A_hat and H, "

    def parity_of(err, ref_max, reference):
        tol = 2e-2 * ref_max if dtype == torch.bfloat16 else 1e-5 * ref_max + 1e-6
        return {"max_abs_err": err, "tol": tol, "max_abs_ref": ref_max, "ok": err <= tol,
                "reference": reference}

    def box_line_rate():
        """roofline.box_line_rate: this GPU's random 128-B line rate right before the timed
        region (appnp_line_rate_probe on the bench's own H buffer, ~20 ms), so a line in a slow
        timing state says so itself."""
        try:
            from ppnp_amd.ops import line_rate_probe

            return line_rate_probe(H, PROBE_LINES)
        except Exception as e:  # noqa: BLE001 -- a diagnostic, not the measurement
            log(f"[bench] line-rate probe failed: {type(e).__name__}: {e}")
            return None

    def result(runner, wall, dev_ms, steps_ms, parallelism, exchange_in, box=None):
        graph = runner.graph
        F_local = runner.width
        avg_iter_ms = dev_ms / (args.steps * K)
        desc, kkey, fs, r, lpe = rank_kernel_plan(runner, K)
        tkey = rank_traffic_key(args.workload, dname, runner, K)
        sb = graph.source_block_layout() if r else None
        rl = roofline(n=n, rows=graph.rows, nnz=graph.nnz_hat, F_local=F_local, esz=esz,
                      avg_iter_ms=avg_iter_ms, fs=fs, r=r, lpe=lpe,
                      exchange_in_bytes=exchange_in, kernel=desc, kernel_key=kkey,
                      traffic=committed_traffic(tkey))
        rl["source_blocks"] = sb
        rl["traffic_key"] = tkey
        rl["kernel_ms"] = kernel_split(runner.run, dev, K, avg_iter_ms)
        rl["box_line_rate"] = box["G_lines_s"] if box else None
        rl["box_line_probe"] = (dict(box, source="appnp_line_rate_probe (ppnp_amd/csrc/"
                                     "appnp_probe.hip): random 128-B lines of the H buffer, "
                                     "right before the timed region, median of 3 launches")
                                if box else None)
        return {
            "metric": METRIC,
            "value": n * F * K * args.steps / wall,
            "unit": "node-feats/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1e3 / args.steps,
            # device time of each timed step on this rank (HIP events): spread of the run
            "step_ms": {"min": steps_ms[0], "median": steps_ms[len(steps_ms) // 2],
                        "max": steps_ms[-1]},
            "propagated_rows_per_s": n * K * args.steps / wall,  # also N*K/t
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dname,
            "data": synth.DESCRIPTIONS.get(args.workload, "synthetic") + ", H ~ N(0,1)",
            "config": {
                "workload": args.workload,
                "nodes": n,
                "nnz_a_hat": None,  # filled by the caller (whole graph)
                "F": F,
                "K": K,
                "alpha": alpha,
                "norm": "sym",
                "parallelism": parallelism,
            },
            "roofline": rl,
            "build": binfo,
            "device": device_info(dev),
        }

    stream = torch.cuda.current_stream(dev)
    if not distributed:
        t1 = time.perf_counter()
        graph = ppnp_amd.Graph.from_csr(indptr, indices, None, n, mode="sym", device=dev,
                                        features=F, dtype=dtype)
        torch.cuda.synchronize()
        t_build = time.perf_counter() - t1
        del indices
        runner = SingleRunner(graph, H, K, alpha, dtype, ld, plan=args.plan)
        log(f"[bench] nnz_hat={graph.nnz_hat} build {t_build:.3f}s")
        box = box_line_rate()
        wall, dev_ms, steps_ms = time_steps(runner.run, stream, args.steps, args.warmup, 1, None)
        res = result(runner, wall, dev_ms, steps_ms, "single", 0, box)
        res["config"]["nnz_a_hat"] = graph.nnz_hat
        if cpu_iters > 0:
            cb, Zc = cpu_baseline(graph, H, K, alpha, cpu_iters, adj_small, world)
            res["cpu_baseline"] = cb
            if cpu_iters == K:
                res["parity"] = parity_of(float((runner.out.float().cpu() - Zc).abs().max()),
                                          float(Zc.abs().max()),
                                          ORACLE_REF + "all K iterations")
        print(json.dumps(res), flush=True)
        return res

    # -- partitioned ----------------------------------------------------------------------
    # The parity reference of every candidate is the oracle's CPU loop, all K iterations, on the
    # same A_hat and H (VERDICT r3 missing #2): rank 0 runs it once, before any candidate (it
    # needs no exchange), on the device A_hat of a whole-graph build, and sends Z_K to every
    # rank over the gloo control group; each rank then checks its block of the timed Z_K
    # against it (max over ranks).  Only with the CPU leg cut short (--cpu-iters < K) is the
    # reference a single-GPU appnp_propagate of the whole graph on every rank instead.  An
    # emulated rank (no exchange: stale gathered rows) has no parity.
    nnz_total = None
    Zc = None
    if rank == 0:
        Gref = ppnp_amd.Graph.from_csr(indptr, indices, None, n, mode="sym", device=dev)
        nnz_total = Gref.nnz_hat
        if cpu_iters > 0 and not args.emulate:
            try:
                cb, Zc = cpu_baseline(Gref, H, K, alpha, cpu_iters, adj_small, world)
                extras["cpu_baseline"] = cb
            except Exception as e:  # noqa: BLE001 -- a baseline: the lines still get parity
                log(f"[bench] cpu_baseline failed: {type(e).__name__}: {e}")
                Zc = None
            if cpu_iters != K:
                Zc = None
        Gref.close()
        del Gref
        torch.cuda.empty_cache()
    # the oracle's Z_K goes to every rank's host memory: above PARITY_BCAST_MAX_BYTES (ADVICE
    # r4: it grows with n x F and only the gloo timeout bounds the broadcast) the lines fall back
    # to the single-GPU reference, and the CPU leg still gives cpu_baseline
    use_oracle = (cpu_iters == K and not args.emulate
                  and (world == 1 or n * F * 4 <= PARITY_BCAST_MAX_BYTES))
    if world > 1 and use_oracle:
        have = torch.tensor([1 if Zc is not None else 0], dtype=torch.int32)
        torch.distributed.broadcast(have, 0, group=ctl)
        use_oracle = bool(have.item())
        if use_oracle:
            Zc = (Zc.float().contiguous() if rank == 0
                  else torch.empty(n, F, dtype=torch.float32))
            torch.distributed.broadcast(Zc, 0, group=ctl)
    use_oracle = use_oracle and Zc is not None
    Zref = None
    if not use_oracle and not args.emulate:
        Gref = ppnp_amd.Graph.from_csr(indptr, indices, None, n, mode="sym", device=dev)
        Zref = ppnp_amd.propagate_forward(Gref, H, K, alpha)
        Gref.close()
        del Gref
    if use_oracle:
        ref_max = float(Zc.abs().max())
        ref_name = (ORACLE_REF + "all K iterations (rank 0, sent to every rank); each rank's "
                    "block of the timed Z_K, max over ranks")
    else:
        ref_max = float(Zref.abs().max()) if Zref is not None else 0.0
        ref_name = "single-GPU appnp_propagate of the whole graph, per rank (max over ranks)"

    pipeline = {"auto": None, "on": True, "off": False}[args.pipeline]

    def measure(cand):
        layout, overlap, exchange = cand
        if world > 1 and layout.rows > 1:
            pdist.ensure_data_group(data_backend, dev)  # collective; RCCL comes up here
        t1 = time.perf_counter()
        kw = dict(emu)
        if "comm" in kw:  # emulated rank: pipelines only where the real exchange could
            kw["comm"] = pdist.NullComm(broadcast=not pdist.relayed(layout, exchange))
        runner = pdist.PartitionedAPPNP.create(indptr, indices, n, H, K, alpha, dev,
                                               layout=layout, overlap=overlap,
                                               exchange=exchange, pipeline=pipeline, **kw)
        torch.cuda.synchronize()
        t_build = time.perf_counter() - t1
        try:
            box = box_line_rate()
            wall, dev_ms, steps_ms = time_steps(runner.run, stream, args.steps, args.warmup,
                                                world, ctl)
            par = cand_name(cand) + ("-pipelined" if getattr(runner, "pipeline", False)
                                     else "")
            if args.emulate:
                par += f"-EMULATED-rank{args.emulate}"
            R = runner.layout.rows
            # the other row shards of this rank's column group land here every iteration
            exchange_in = ((R - 1) * runner.shard * runner.width * esz
                           if R > 1 and not args.emulate else 0)
            res = result(runner, wall, dev_ms, steps_ms, par, exchange_in, box)
            res["config"]["nnz_a_hat"] = nnz_total
            res["config"]["build_s"] = t_build
            ref = Zc if use_oracle else Zref
            if ref is not None:
                blk = ref[runner.lo:runner.hi, runner.f_lo:runner.f_hi]
                got = runner.out if blk.device == runner.out.device else runner.out.cpu()
                err = float((got.double() - blk.double()).abs().max()) if blk.numel() else 0.0
                e = torch.tensor([err], dtype=torch.float64)
                if world > 1:
                    torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX,
                                                 group=ctl)
                res["parity"] = parity_of(float(e[0]), ref_max, ref_name)
                if use_oracle:
                    # the same check, under the name the N = 1 line's oracle comparison had
                    # before round 4 (every N > 1 line now carries it)
                    res["parity_cpu"] = res["parity"]
            return res
        finally:
            del runner
            torch.cuda.empty_cache()

    def emit(res):
        if "cpu_baseline" in extras:
            res["cpu_baseline"] = extras["cpu_baseline"]
        print(json.dumps(res), flush=True)

    if len(cands) == 1:
        res = measure(cands[0])
        if args.layout == "auto":
            res["config"]["autotune_ms_per_step"] = {cand_name(cands[0]): res["ms_per_step"]}
    else:
        res, _ = run_candidates(cands, measure, ctl, args.candidate_timeout, emit, cand_name,
                                rank, world, exchanges=lambda c: c[0].rows > 1,
                                budget_s=args.run_budget if world > 1 else 0.0)
    if rank == 0:
        emit(res)
    if world > 1:
        # the line is out; a teardown that stalls (a communicator some candidate left busy)
        # must not turn a finished run into a timeout
        with Deadline(60.0, lambda: os._exit(0)):
            torch.distributed.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
