#!/bin/bash
# Round 5, first session: the per-launch timer's GPU tests, the default bench line (now with
# roofline.kernel_ms), and configs 2 / 3 with the full CPU leg (cpu_baseline + parity).
set -u
tools/gpu_session.sh \
 "probe_tests::300::python -u -m pytest tests/test_gpu_probe.py -x -v --timeout 120 --timeout-method thread" \
 "bench_default::300::python bench.py" \
 "bench_pubmed::300::python bench.py --workload pubmed-synth" \
 "bench_msacad::300::python bench.py --workload ms-academic-synth"
