#!/bin/bash
# Round 5: the only sequence that has produced the fast timing state so far --
# the whole -m gpu suite, then the bench -- with roofline.kernel_ms in every line, so the lines
# say which launch is faster in the fast state (or whether the launches overlapped).
set -u
tools/gpu_session.sh \
 "gpu_tests::900::python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread" \
 "bench_after_suite_1::200::python bench.py --cpu-iters 0" \
 "bench_after_suite_2::200::python bench.py --cpu-iters 0" \
 "bench_after_suite_3::200::python bench.py"
