#!/bin/bash
# Round 4: the whole -m gpu suite and smoke() on the final tree.  Logs under gpurun_out/.
set -u
tools/gpu_session.sh \
 "gpu_tests::1080::python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'"
