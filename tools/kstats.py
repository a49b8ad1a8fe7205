"""Print the kernels above 1 ms of total time from rocprofv3 kernel_stats.csv files.
Usage: python tools/kstats.py gpurun_out/remab/*/run_kernel_stats.csv"""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        if float(r["TotalDurationNs"]) > 1e6:
            print(f"  {r['Name'][:72]:72s} {r['Calls']:>5} {float(r['AverageNs']) / 1e6:9.4f} ms")
