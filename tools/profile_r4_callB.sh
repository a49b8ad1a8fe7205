#!/bin/bash
# Round 4, after the per-rank PMC entries are committed: the default bench line (traffic, line-rate
# probe, build provenance), the driver's N = 2 and N = 8 products commands rehearsed on the one GPU
# (gloo exchange: every candidate measured, parity of every line against the CPU oracle), and the
# new multi-process GPU tests.  Logs under gpurun_out/.
set -u
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
 "bench_default::400::python bench.py" \
 "new_gpu_tests::900::python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_configs.py -k 'products_row_partition or two_d_layout'" \
 "n2_products::600::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 2 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1" \
 "n8_products::900::PPNP_DIST_BACKEND=gloo $R --nproc-per-node 8 --master-port 29518 bench.py --gpus 8 --steps 2 --warmup 1"
