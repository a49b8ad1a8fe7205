#!/bin/bash
# Round 6, final tree: the whole -m gpu suite with every test's duration,
# smoke(), the default bench line, and the driver's bench command under rocprofv3 (kernel trace).
set -u
tools/gpu_session.sh \
 "f_suite::900::python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=0" \
 "f_smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "f_bench_default::300::python bench.py" \
 "f_driver_stats::300::rocprofv3 --kernel-trace --stats -o run --output-format csv -d gpurun_out/drv6 -- python bench.py"
