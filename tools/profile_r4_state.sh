#!/bin/bash
# Round 4: what selects the timing state?  Round 4 saw 8.22-8.27 ms per iteration
# in every fresh process, and 7.78 ms in a bench run right after the 9-minute -m gpu suite, with
# the same box line rate (55.5 G lines/s) in both.  Here: on a fresh box, bench at F = 100 / 96 /
# 4 (which kernel changes?), then with a device pad of 16 / 64 / 160 GiB held before the bench's
# own allocations (does placement matter?), then after heavy GPU work in other processes, again.
set -u
B="--steps 10 --warmup 2 --cpu-iters 0"
specs=(
 "a_f100::200::python tools/pad_bench.py -- $B"
 "a_f96::200::python tools/pad_bench.py -- $B --features 96"
 "a_f4::200::python tools/pad_bench.py -- $B --features 4"
 "a_pad16::200::python tools/pad_bench.py --pad-gb 16 --touch -- $B"
 "a_pad64::200::python tools/pad_bench.py --pad-gb 64 --touch -- $B"
 "a_pad160::200::python tools/pad_bench.py --pad-gb 160 --touch -- $B"
 "heavy::600::python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'products'"
 "b_f100::200::python tools/pad_bench.py -- $B"
 "b_f96::200::python tools/pad_bench.py -- $B --features 96"
 "b_f4::200::python tools/pad_bench.py -- $B --features 4"
 "b_pad64::200::python tools/pad_bench.py --pad-gb 64 --touch -- $B"
)
tools/gpu_session.sh "${specs[@]}"
