#!/bin/bash
# Round 5 box survey: one short bench line (with its device block and per-launch split) per
# gpurun call, so the timing state can be tied to hardware across boxes.
set -u
tools/gpu_session.sh "bench_box::200::python bench.py --cpu-iters 0 --steps 10"
