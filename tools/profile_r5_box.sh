#!/bin/bash
# Round 5 box survey: two short bench lines (fresh processes) per gpurun call, each with its
# device block and per-launch split, so the timing state can be tied to hardware across boxes.
set -u
tools/gpu_session.sh "bench_box::200::python bench.py --cpu-iters 0 --steps 10" \
  "bench_box2::200::python bench.py --cpu-iters 0 --steps 10"
