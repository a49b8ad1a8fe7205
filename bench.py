#!/usr/bin/env python
"""Benchmark of the APPNP propagation hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload products-synth]

A "step" is one full propagation call -- K=10 fused SpMM+AXPBY iterations over the whole
graph (appnp_propagate, or the row-partitioned multi-GPU loop) -- on synthetic input that is
resident in HBM before the timed region.  value = nodes * F * K * steps / time (whole job).

N > 1 (launched by torch.distributed.run, one rank per GPU): the ranks form an R x C layout
(ppnp_amd/dist.py): C feature slabs need no exchange, R row groups
exchange their Z shards over RCCL every iteration.  --layout auto times the candidate layouts
of ppnp_amd.dist.candidate_layouts after warm-up (max over ranks) and keeps the fastest; the
timed region is bracketed by barrier + synchronize and the max over ranks is reported.

Extra JSON fields:
  roofline      HBM roofline of the dominant kernel (k_step_*): algorithmic bytes per launch
                B_iter = 4(N+1) + 8 nnz(A_hat) + 3 N F s   / average
                launch time, measured with HIP events on the launch stream; peak 8 TB/s.
  cpu_baseline  the oracle's torch.sparse.mm CPU loop (oracle/ppnp_oracle.py) on the same graph
                and H, a bounded number of iterations, rank 0 at N=1 only.
"""

from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "APPNP K=10 propagated node-feats/sec; achieved HBM GB/s vs peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level parameters)
# random row-gather ceiling measured on MI355X: ~54-57 G cache-line requests/s for 64-512 B
# rows from a 1 GB table (profiles/r1_gather_probe.txt)
GATHER_LINE_CEILING = 56.0


def parse():
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
    p.add_argument("--exchange", default="multipath", choices=["multipath", "group"],
                   help="R x C layouts: relayed exchange over every rank, or one all-gather "
                        "per column group")
    return p.parse_args()


def committed_traffic(workload, dtype, parallelism):
    """HBM bytes per launch of the SpMM kernel from the committed PMC profile of the same
    command (tools/summarize_profile.py writes profiles/pmc_traffic.json), or None."""
    key = f"{workload}:{'bf16' if dtype == torch.bfloat16 else 'f32'}:{parallelism}"
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            return json.load(fh).get(key)
    except (OSError, ValueError):
        return None


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


def cpu_threads() -> tuple[int, int]:
    """(threads to use, CPUs this process may run on).  BASELINE.md asks for every core; on the
    GPU box the process's share is what OMP_NUM_THREADS names (16 of a much larger machine, whose
    full count os.cpu_count() reports), so that bounds it."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or visible
    return max(1, min(visible, share)), visible


def cpu_baseline(graph, H, K, alpha, iters, adj=None):
    """Time the oracle's CPU torch.sparse.mm APPNP loop on the same operator and H (SURVEY.md
    8(d) CPU baseline (i)); return (the JSON object, Z of the CPU loop).  For N <= 20k also time
    the reference's as-shipped PPNP path, compute_ppr + dense Pi @ H (helpers.py:68-71,
    model.py:63; baseline (ii))."""
    from oracle import ppnp_oracle as O

    threads, visible = cpu_threads()
    torch.set_num_threads(threads)
    rp, col, val, _ = graph.csr()
    a_t = torch.sparse_csr_tensor(rp.cpu().long(), col.cpu().long(), val.cpu(),
                                  size=(graph.n, graph.n))
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


def tune_layouts(cands, indptr, indices, n, H, K, alpha, dev, ctl, reps=2):
    """Build each candidate layout, time ``reps`` propagations after one warm-up (barrier on
    both sides, max over ranks: every rank sees the same numbers and picks the same layout),
    keep the fastest and free the others.  A candidate that raises on any rank (agreed over the
    gloo control group ``ctl``, which an RCCL error cannot poison) is recorded as failed and
    skipped, so one broken exchange does not cost the whole scaling run."""
    from ppnp_amd import dist as pdist

    best, best_ms, times = None, None, {}
    for layout, overlap, exchange in cands:
        name = (f"rows{layout.rows}xcols{layout.cols}" + ("-overlap" if overlap else "")
                + (f"-{exchange}" if (layout.rows > 1 and layout.cols > 1)
                   or exchange == "native" else ""))
        if torch.distributed.get_rank() == 0:
            log(f"[bench] autotune: building {layout} overlap={overlap} exchange={exchange}")
        r, err, dt = None, "", 0.0
        try:
            r = pdist.PartitionedAPPNP.create(indptr, indices, n, H, K, alpha, dev,
                                              layout=layout, overlap=overlap, exchange=exchange)
            r.run()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- reported and agreed on below
            err = f"{type(e).__name__}: {e}"
        failed = torch.tensor([1.0 if err else 0.0], dtype=torch.float64)
        torch.distributed.all_reduce(failed, op=torch.distributed.ReduceOp.MAX, group=ctl)
        if float(failed) == 0.0:
            torch.distributed.barrier(group=ctl)
            t0 = time.perf_counter()
            try:
                for _ in range(reps):
                    r.run()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
            t = torch.tensor([dt, 1.0 if err else 0.0], dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=ctl)
            dt, failed = float(t[0]), t[1:]
        if float(failed) != 0.0:
            times[name] = None
            log(f"[bench] autotune {name}: FAILED on rank {torch.distributed.get_rank()}"
                + (f": {err}" if err else " (another rank failed)"))
            del r
            torch.cuda.empty_cache()
            continue
        ms = dt * 1e3 / reps
        times[name] = ms
        if torch.distributed.get_rank() == 0:
            log(f"[bench] autotune {name}: {ms:.3f} ms per propagation")
        if best_ms is None or ms < best_ms:
            best, best_ms = r, ms
        else:
            del r
        torch.cuda.empty_cache()
    if best is None:
        raise RuntimeError(f"every candidate layout failed: {times}")
    return best, times


def main():
    args = parse()
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
    seed = synth.SEEDS.get(args.workload, 0)
    distributed = world > 1 or args.layout != "auto"
    emu = {}
    lw = world
    if args.emulate:
        P, r = (int(x) for x in args.emulate.split(":"))
        emu = dict(rank=r, world=P, comm=pdist.NullComm())
        lw = P
    esz = 2 if dtype == torch.bfloat16 else 4
    mem = torch.cuda.get_device_properties(dev).total_memory
    nnz_bound = 2 * m + n  # nnz(A_hat) <= 2 m + n (symmetrised edges + diagonal)
    if args.layout == "auto" and world > 1 and not args.emulate:
        cands = pdist.candidate_layouts(world, F, n, nnz_bound, esz, mem)
    else:
        layout = (pdist.choose_layout(lw, n, F, nnz_bound, esz, mem) if args.layout == "auto"
                  else pdist.Layout.parse(args.layout, lw))
        cands = [(layout, args.overlap, args.exchange)]
    if world > 1:
        # RCCL only where a layout has a data-path exchange (row groups); pure column layouts
        # have none, so their control plane (barrier, max-over-ranks) runs over gloo
        rows = any(c[0].rows > 1 for c in cands)
        backend = os.environ.get("PPNP_DIST_BACKEND") or ("nccl" if rows else "gloo")
        if backend == "nccl":
            # a collective that stalls aborts the job after 5 minutes (watchdog) instead of
            # holding the node for the default 10
            torch.distributed.init_process_group("nccl", device_id=dev,
                                                 timeout=datetime.timedelta(minutes=5))
        else:
            torch.distributed.init_process_group(backend)
    # control plane (barriers, max over ranks, failure agreement) on gloo over host memory:
    # RCCL carries only the data-path exchange
    ctl = None
    if world > 1 and torch.distributed.get_backend() == "nccl":
        ctl = torch.distributed.new_group(backend="gloo")

    stagger = float(os.environ.get("PPNP_BENCH_STAGGER") or 0)
    if stagger and world > 1:
        # rehearsals with all ranks on ONE GPU only: concurrent generation of a products-sized
        # graph by 8 processes time-slicing one device stalls in torch.unique for minutes
        # (0.23 s alone), so rank r starts r * stagger seconds late; never set on a real node
        time.sleep(rank * stagger)
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
    if rank == 0 and world > 1:
        log(f"[bench] {args.workload}: graph and H generated in {t_gen:.2f}s")

    autotune = None
    if distributed:
        t1 = time.perf_counter()
        if len(cands) == 1:
            layout, overlap, exchange = cands[0]
            runner = pdist.PartitionedAPPNP.create(indptr, indices, n, H, K, alpha, dev,
                                                   layout=layout, overlap=overlap,
                                                   exchange=exchange, **emu)
        else:
            runner, autotune = tune_layouts(cands, indptr, indices, n, H, K, alpha, dev, ctl)
        torch.cuda.synchronize()
        t_build = time.perf_counter() - t1
        graph = runner.graph
        run = runner.run
        stream = torch.cuda.current_stream(dev)
        F_local = runner.width
        mine = graph.nnz_hat if runner.layout.coords(runner.rank)[1] == 0 else 0
        nnz_t = torch.tensor([mine], dtype=torch.int64)
        if world > 1:
            torch.distributed.all_reduce(nnz_t, group=ctl)
        nnz_total = int(nnz_t.item())
    else:
        t1 = time.perf_counter()
        graph = ppnp_amd.Graph.from_csr(indptr, indices, None, n, mode="sym", device=dev,
                                        features=F, dtype=dtype)
        torch.cuda.synchronize()
        t_build = time.perf_counter() - t1
        Z = torch.empty(n, ld, dtype=dtype, device=dev)[:, :F]

        if args.plan:
            from ppnp_amd.ops import PropagatePlan

            plan = PropagatePlan(graph, H, K, alpha)
            Z = plan.Z

            def run():
                plan()
        else:

            def run():
                ppnp_amd.propagate_forward(graph, H, K, alpha, out=Z)

        stream = torch.cuda.current_stream(dev)
        F_local = F
        nnz_total = graph.nnz_hat
    adj_small = None
    if n <= 20000 and world == 1:  # the as-shipped PPNP leg of the CPU baseline needs A
        import numpy as np
        import scipy.sparse as sp

        ip_c, ix_c = indptr.cpu().numpy(), indices.cpu().numpy()
        adj_small = sp.csr_matrix((np.ones(len(ix_c), dtype=np.float32), ix_c, ip_c),
                                  shape=(n, n))
    if distributed:
        ref_csr = (indptr, indices)  # rank-0 style verification of the partitioned result
    del indices
    if rank == 0:
        log(f"[bench] {args.workload}: N={n} nnz_hat={nnz_total} F={F} K={K} dtype={dtype} "
            f"gen {t_gen:.2f}s build {t_build:.3f}s"
            + (f" layout {runner.layout}" if distributed else ""))

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier(group=ctl)
    torch.cuda.synchronize()
    # one event per step boundary on the launch stream: the timed region's device time and the
    # spread of the individual steps (reported as step_ms)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev0, ev1 = evs[0], evs[-1]
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        run()
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier(group=ctl)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1)
    steps_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    if world > 1:
        t = torch.tensor([wall, dev_ms], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=ctl)
        wall, dev_ms = float(t[0]), float(t[1])

    # parity of the timed result: at N > 1 every rank compares its block of Z_K with a
    # single-GPU appnp_propagate of the whole graph on its own device (max over ranks), so a
    # wrong exchange fails loudly instead of printing a throughput
    dist_parity = None
    if distributed and not args.emulate:
        Zblk = runner.out
        ip_r, ix_r = ref_csr
        Gref = ppnp_amd.Graph.from_csr(ip_r, ix_r, None, n, mode="sym", device=dev)
        Zref = ppnp_amd.propagate_forward(Gref, H, K, alpha)
        blk = Zref[runner.lo:runner.hi, runner.f_lo:runner.f_hi]
        err = float((Zblk.double() - blk.double()).abs().max()) if blk.numel() else 0.0
        ref_max = float(Zref.abs().max())
        e = torch.tensor([err, ref_max], dtype=torch.float64)
        if world > 1:
            torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX, group=ctl)
        err, ref_max = float(e[0]), float(e[1])
        tol = 1e-5 * ref_max + 1e-6
        dist_parity = {"max_abs_err": err, "tol": tol, "max_abs_ref": ref_max,
                       "ok": err <= tol,
                       "reference": "single-GPU appnp_propagate of the whole graph, per rank"}
        del Gref, Zref, blk, ref_csr
        if not dist_parity["ok"]:
            log(f"[bench] PARITY FAILURE of the partitioned result: {dist_parity}")

    s = 2 if dtype == torch.bfloat16 else 4
    rows_local = graph.rows
    nnz_local = graph.nnz_hat
    # dominant kernel: one SpMM launch per iteration per rank
    b_iter = 4 * (rows_local + 1) + 8 * nnz_local + 3 * rows_local * F_local * s
    avg_launch_ms = dev_ms / (args.steps * K)
    achieved = b_iter / (avg_launch_ms * 1e-3) / 1e9
    # gather line-request rate: every nonzero gathers one row of Z_k; with
    # split rows only the fs main columns are gathered (whole lines), the rest run the
    # L2-blocked remainder pass (appnp_blocks.hip)
    # (single GPU, or a column layout, whose ranks call appnp_propagate on their slab)
    whole = not distributed or runner.layout.rows == 1
    r_cols = graph.remainder_cols(F_local, dtype) if whole and K >= 2 else 0
    fs = F_local - r_cols if r_cols else 0
    ld_l = pdist.line_ld(F_local, s)
    lines_per_row = (fs * s // 128 if r_cols else
                     1 if ld_l * s <= 128 else -(-(F_local * s) // 128))
    lines = nnz_local * lines_per_row + (8 * nnz_local + 3 * rows_local * ld_l * s) / 128
    line_rate = lines / (avg_launch_ms * 1e-3) / 1e9
    value = n * F * K * args.steps / wall
    rows_per_s = n * K * args.steps / wall  # also N*K/t
    parallelism = ((f"rows{runner.layout.rows}xcols{runner.layout.cols}"
                    + ("-overlap" if runner.overlap else "")
                    + (f"-{runner.exchange}" if (runner.layout.rows > 1 and runner.layout.cols > 1
                       and runner.exchange != "none") or runner.exchange == "native" else "")
                    + (f"-EMULATED-rank{args.emulate}" if args.emulate else ""))
                   if distributed else "single")
    traffic = committed_traffic(args.workload, dtype, parallelism)
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "node-feats/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / args.steps,
        # device time of each timed step on this rank (HIP events): spread of the run
        "step_ms": {"min": steps_ms[0], "median": steps_ms[len(steps_ms) // 2],
                    "max": steps_ms[-1]},
        "propagated_rows_per_s": rows_per_s,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
        "data": synth.DESCRIPTIONS.get(args.workload, "synthetic") + ", H ~ N(0,1)",
        "config": {
            "workload": args.workload,
            "nodes": n,
            "nnz_a_hat": nnz_total,
            "F": F,
            "K": K,
            "alpha": alpha,
            "norm": "sym",
            "parallelism": parallelism,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": "profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / "
                              "WRITE_SIZE passes of this bench command, gfx950-corrected)",
            # the PMC bytes per launch over the same launch time: how fast the kernel moves
            # the bytes the random gathers force it to move (Infinity-Cache hits included)
            "traffic_GBs": (traffic / (avg_launch_ms * 1e-3) / 1e9) if traffic else None,
            "traffic_frac": (traffic / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                            if traffic else None,
            "gather_line_rate": {
                "lines_per_launch": lines,
                "achieved_G_lines_s": line_rate,
                "ceiling_G_lines_s": GATHER_LINE_CEILING,
                "frac": line_rate / GATHER_LINE_CEILING,
                "ceiling_source": "tools/gather_probe.hip, profiles/r1_gather_probe.txt",
            },
            "kernel": ("k_step_wide (one launch per iteration)" if not r_cols else
                       ("k_rem_persist on all the slab's columns (narrow rows: one persistent "
                        "L2-blocked launch per iteration)") if not fs else
                       f"k_step_wide on columns [0, {fs}) of the slab + k_rem_persist (the "
                       f"remainder columns, one persistent L2-blocked launch) per iteration; "
                       f"times are per iteration"),
            "bytes_per_launch": b_iter,
            "avg_launch_ms": avg_launch_ms,
            # the access-pattern bound: every nonzero gathers a random row of Z,
            # i.e. `lines_per_row` 128-B line requests (3 for a split F = 100 fp32 row), plus the
            # streamed lines, at the chip's measured random-line rate; the L2-resident remainder
            # pass is left out, so this is a lower bound on the iteration time
            "ceiling": {
                "ms_per_iter": lines / (GATHER_LINE_CEILING * 1e9) * 1e3,
                "frac": b_iter / (lines / (GATHER_LINE_CEILING * 1e9)) / 1e9 / HBM_PEAK_GBS,
                "lines_per_nonzero": lines_per_row,
                "basis": f"{lines:.4g} line requests per iteration at the {GATHER_LINE_CEILING} "
                         "G lines/s random-gather rate of tools/gather_probe.hip",
            },
            "note": "a uniform random graph gathers whole cache lines per nonzero, so the "
                    "compulsory-byte fraction is capped at ceiling.frac; 60 % of the "
                    "compulsory-byte roofline is out of reach for it on one GPU",
        },
    }
    if autotune is not None:
        res["config"]["autotune_ms_per_step"] = autotune
    if dist_parity is not None:
        res["parity"] = dist_parity
    cpu_iters = K if args.cpu_iters is None else args.cpu_iters
    if world == 1 and cpu_iters > 0 and not distributed:
        res["cpu_baseline"], Zc = cpu_baseline(graph, H, K, alpha, cpu_iters, adj_small)
        if cpu_iters == K:
            # value parity of the timed GPU result against the oracle's fp32 CPU loop on the
            # same A_hat and H; fp32 bar of the tests: 1e-5 max|Z_ref| + 1e-6
            err = float((Z.float().cpu() - Zc).abs().max())
            ref_max = float(Zc.abs().max())
            tol = 1e-5 * ref_max + 1e-6
            if dtype == torch.bfloat16:
                tol = 2e-2 * ref_max  # bf16 storage bar
            res["parity"] = {"max_abs_err": err, "tol": tol, "max_abs_ref": ref_max,
                             "ok": err <= tol,
                             "reference": "oracle fp32 torch.sparse.mm CPU loop, same A_hat "
                                          "and H, all K iterations"}
        del Zc
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
