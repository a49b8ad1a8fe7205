#!/usr/bin/env python
"""Summarise rocprofv3 output (kernel stats + separate --pmc FETCH_SIZE / WRITE_SIZE passes)
into profiles/<tag>_summary.json, and copy the kernel stats CSV next to it.

    python tools/summarize_profile.py <tag> <stats_dir> <pmc_fetch_dir> <pmc_write_dir> \
        [--workload products-synth] [--bench-json gpurun_out/x.log]

HBM traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
fetch_bytes = 2 * FETCH_SIZE * 1024 (the kernel's reads are 16 B/lane), write_bytes =
WRITE_SIZE * 1024 (16 B/lane stores read exactly).  Infinity-Cache hits are included.
"""

import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not hits:
        raise FileNotFoundError(f"no *{suffix} under {d}")
    return hits[0]


def per_dispatch(path, match):
    """{counter: [value per dispatch]} for the kernels whose name contains ``match``."""
    vals = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            vals[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = collections.defaultdict(list)
    for (d, c), v in vals.items():
        out[c].append(v)
    return out, names


def per_iteration(path, counter, kernels, iterations):
    """Counter total of one APPNP iteration: the sum over the dispatches of every kernel of
    the iteration (the SpMM kernel; with split rows also the remainder passes and the per-call
    split copy; with overlap the local and the remote launch) divided by the iterations the
    profiled command ran ((warmup + steps) x K of its bench line).  Without a count, by the
    dispatches of the first kernel that ran (one per iteration)."""
    total, n_first = 0.0, 0
    for k in kernels:
        d, _ = per_dispatch(path, k)
        total += sum(d[counter])
        if not n_first:
            n_first = len(d[counter])
    n_iter = iterations or n_first
    return total / max(1, n_iter), n_iter


def main():
    p = argparse.ArgumentParser()
    p.add_argument("tag")
    p.add_argument("stats_dir")
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--kernels", default="k_step_,k_rem_persist,k_split_copy",
                   help="kernels of one iteration, the SpMM kernel (one per iteration) first")
    p.add_argument("--workload", default="products-synth")
    p.add_argument("--bench-json", default=None)
    a = p.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    bench = None
    if a.bench_json:
        for line in open(a.bench_json):
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                bench = json.loads(line)
    # iterations of the profiled command: every propagation of its warm-up and timed steps, plus
    # the one untimed propagation of roofline.kernel_ms (round 5) when the line carries it (a
    # --cpu-iters 0 run of one GPU or one emulated rank launches nothing else of these kernels)
    extra = 1 if bench and bench["roofline"].get("kernel_ms") else 0
    iters = ((bench["warmup"] + bench["steps"] + extra) * bench["config"]["K"]) if bench else 0
    stats = find(a.stats_dir, "kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    kernels = a.kernels.split(",")
    kern = [r for r in rows if any(k in r["Name"] for k in kernels)]
    first = next((k for k in kernels if any(k in r["Name"] for r in kern)), kernels[0])
    spmm_calls = iters or sum(int(r["Calls"]) for r in kern if first in r["Name"])
    iter_ns = sum(float(r["TotalDurationNs"]) for r in kern) / max(1, spmm_calls)
    f_kib, n_iter = per_iteration(find(a.fetch_dir, "counter_collection.csv"), "FETCH_SIZE",
                                  kernels, iters)
    w_kib, _ = per_iteration(find(a.write_dir, "counter_collection.csv"), "WRITE_SIZE", kernels,
                             iters)
    fetch_b = 2.0 * f_kib * 1024
    write_b = w_kib * 1024
    summ = {
        "tag": a.tag,
        "workload": a.workload,
        "kernel_stats": [
            {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
             "pct": float(r["Percentage"])} for r in kern
        ],
        # kernel time of one iteration (all its kernels), comparable to bench avg_launch_ms
        "iteration_ms": iter_ns / 1e6,
        "pmc": {
            "FETCH_SIZE_KiB_per_launch": f_kib,
            "WRITE_SIZE_KiB_per_launch": w_kib,
            "per": "iteration (SpMM launches + remainder pass + split copy / K)",
            "launches": n_iter,
            "fetch_bytes_corrected": fetch_b,
            "write_bytes": write_b,
            "traffic_bytes_per_launch": fetch_b + write_b,
            "correction": "fetch = 2 x FETCH_SIZE KiB (gfx950 half-count of wide reads); "
                          "write = WRITE_SIZE KiB",
        },
    }
    if bench:
        summ["bench"] = bench
    if "bench" in summ:
        b = summ["bench"]
        # the bench's own key: workload, dtype, layout, the iteration's kernels and a digest of
        # the kernel sources, so a profile of other or older kernels never matches a run
        key = b["roofline"].get("traffic_key") or (
            f"{b['config']['workload']}:{b['dtype']}:{b['config']['parallelism']}")
        tpath = os.path.join(prof, "pmc_traffic.json")
        table = json.load(open(tpath)) if os.path.exists(tpath) else {}
        table[key] = fetch_b + write_b
        json.dump(table, open(tpath, "w"), indent=1, sort_keys=True)
    out = os.path.join(prof, f"{a.tag}_summary.json")
    json.dump(summ, open(out, "w"), indent=1)
    print(json.dumps(summ["pmc"], indent=1))
    for k in summ["kernel_stats"]:
        print(k)


if __name__ == "__main__":
    main()
