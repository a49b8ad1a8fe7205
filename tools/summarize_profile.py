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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("tag")
    p.add_argument("stats_dir")
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--kernel", default="k_step_")
    p.add_argument("--workload", default="products-synth")
    p.add_argument("--bench-json", default=None)
    a = p.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(a.stats_dir, "kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    kern = [r for r in rows if a.kernel in r["Name"]]
    fetch, _ = per_dispatch(find(a.fetch_dir, "counter_collection.csv"), a.kernel)
    write, _ = per_dispatch(find(a.write_dir, "counter_collection.csv"), a.kernel)
    f_kib = sum(fetch["FETCH_SIZE"]) / max(1, len(fetch["FETCH_SIZE"]))
    w_kib = sum(write["WRITE_SIZE"]) / max(1, len(write["WRITE_SIZE"]))
    fetch_b = 2.0 * f_kib * 1024
    write_b = w_kib * 1024
    summ = {
        "tag": a.tag,
        "workload": a.workload,
        "kernel_stats": [
            {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
             "pct": float(r["Percentage"])} for r in kern
        ],
        "pmc": {
            "FETCH_SIZE_KiB_per_launch": f_kib,
            "WRITE_SIZE_KiB_per_launch": w_kib,
            "launches": len(fetch["FETCH_SIZE"]),
            "fetch_bytes_corrected": fetch_b,
            "write_bytes": write_b,
            "traffic_bytes_per_launch": fetch_b + write_b,
            "correction": "fetch = 2 x FETCH_SIZE KiB (gfx950 half-count of wide reads); "
                          "write = WRITE_SIZE KiB",
        },
    }
    if a.bench_json:
        for line in open(a.bench_json):
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                summ["bench"] = json.loads(line)
    if "bench" in summ:
        b = summ["bench"]
        key = f"{b['config']['workload']}:{b['dtype']}:{b['config']['parallelism']}"
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
