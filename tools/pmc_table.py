#!/usr/bin/env python
"""Per-kernel mean of every counter per dispatch in rocprofv3 counter-collection CSVs.

    python tools/pmc_table.py <label>=<dir or csv> [...] [--match k_rem_persist]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def table(path, match):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(float)  # (kernel, counter, dispatch) -> value summed over dimensions
    for r in csv.DictReader(open(path)):
        if match and match not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"], r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    agg = defaultdict(list)
    for (k, c, _), v in per.items():
        agg[(k, c)].append(v)
    return {(k, c): (sum(v) / len(v), len(v)) for (k, c), v in agg.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--match")]
    match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "")
    for spec in args:
        label, path = spec.split("=", 1)
        for (k, c), (mean, n) in sorted(table(path, match).items()):
            print(f"{label:10s} {k[:70]:70s} {c:28s} {mean:16.4e} ({n} dispatches)")


if __name__ == "__main__":
    main()
