#!/bin/bash
# Single-GPU evidence for profiles/ (the subset of tools/profile_round.sh that the one-GPU
# kernels change): default bench (with the CPU baseline and parity), rocprofv3 kernel stats,
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss), and the other workloads.
# Afterwards (in the build container): python tools/collect_round.py <tag>
set -u
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
tools/gpu_session.sh \
 "bench_default::400::python bench.py" \
 "prof_stats::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- $B" \
 "pmc_fetch::300::timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B" \
 "pmc_write::300::timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B" \
 "pmc_l2::300::timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- $B" \
 "w_pubmed::200::$B --workload pubmed-synth" \
 "w_msacad::200::$B --workload ms-academic-synth" \
 "w_arxiv::200::$B --workload arxiv-synth" \
 "w_cora::200::$B --workload cora-ml" \
 "w_cora_real::200::$B --workload cora-ml-real" \
 "w_powerlaw::200::$B --workload products-powerlaw" \
 "w_local::200::$B --workload products-local" \
 "w_bf16::200::$B --dtype bf16"
