#!/usr/bin/env python
"""Collect the logs of tools/profile_round.sh (gpurun_out/) into profiles/<tag>_*.

    python tools/collect_round.py r1

Writes <tag>_bench_default.json, <tag>_layout_emulation.jsonl, <tag>_workloads.jsonl,
<tag>_dist_check.txt, and runs tools/summarize_profile.py for the rocprofv3 stats + PMC passes
(<tag>_kernel_stats.csv, <tag>_summary.json, profiles/pmc_traffic.json).
"""

import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def bench_lines(label):
    path = os.path.join(OUT, label + ".log")
    if not os.path.exists(path):
        return []
    return [json.loads(l) for l in open(path) if l.startswith("{") and '"metric"' in l]


def main():
    tag = sys.argv[1]
    b = bench_lines("bench_default")
    if b:
        json.dump(b[-1], open(os.path.join(PROF, f"{tag}_bench_default.json"), "w"))
    for prefix, name in (("emu_", "layout_emulation"), ("w_", "workloads")):
        rows = []
        for log in sorted(glob.glob(os.path.join(OUT, prefix + "*.log"))):
            rows += bench_lines(os.path.basename(log)[:-4])
        with open(os.path.join(PROF, f"{tag}_{name}.jsonl"), "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")
    with open(os.path.join(PROF, f"{tag}_dist_check.txt"), "w") as fh:
        for log in sorted(glob.glob(os.path.join(OUT, "dc_*.log"))):
            lines = [l for l in open(log) if l.startswith(("[dist_check]", "[dist_worker]"))]
            fh.write(f"# {os.path.basename(log)}\n" + "".join(sorted(lines)))
    if os.path.isdir(os.path.join(OUT, "pmc_fetch")):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_profile.py"), tag,
                        os.path.join(OUT, "prof_stats"), os.path.join(OUT, "pmc_fetch"),
                        os.path.join(OUT, "pmc_write"), "--bench-json",
                        os.path.join(OUT, "prof_stats.log")], check=True)


if __name__ == "__main__":
    main()
