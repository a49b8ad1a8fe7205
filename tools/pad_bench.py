#!/usr/bin/env python
"""Timing-state experiment: hold a device buffer of --pad-gb GiB (optionally
written once, --touch) before bench.py allocates anything, then run bench.main on the same
process with the remaining arguments.  If the iteration time depends on where in device memory
the bench's buffers land, the pad moves them.

    python tools/pad_bench.py --pad-gb 64 [--touch] -- --steps 10 --warmup 2 --cpu-iters 0
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    rest = argv[argv.index("--") + 1:] if "--" in argv else []
    ap = argparse.ArgumentParser()
    ap.add_argument("--pad-gb", type=float, default=0.0)
    ap.add_argument("--touch", action="store_true")
    a = ap.parse_args(argv[:argv.index("--")] if "--" in argv else argv)
    pad = None
    if a.pad_gb > 0:
        pad = torch.empty(int(a.pad_gb * 2**30), dtype=torch.uint8, device="cuda:0")
        if a.touch:
            pad.fill_(1)
        torch.cuda.synchronize()
        print(f"[pad] holding {a.pad_gb} GiB at 0x{pad.data_ptr():x}", file=sys.stderr, flush=True)
    import bench

    bench.main(rest)
    del pad


if __name__ == "__main__":
    main()
