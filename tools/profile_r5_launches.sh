#!/bin/bash
# Round 5: every launch's time (roofline.kernel_ms.ms_per_launch) of the headline and of the 96
# main columns alone, and the device block of the box (HBM vendor, board id, clocks).
set -u
tools/gpu_session.sh \
 "bench_l1::200::python bench.py --cpu-iters 0" \
 "bench_f96::200::python bench.py --cpu-iters 0 --features 96" \
 "bench_l2::200::python bench.py --cpu-iters 0"
