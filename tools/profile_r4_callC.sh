#!/bin/bash
# Round 4: the flat-mapping gather probe (tools/flat_probe.hip), then the whole -m gpu suite and
# smoke() on the final tree.  Logs under gpurun_out/.
set -u
tools/gpu_session.sh \
 "flat_probe::120::tools/bin/flat_probe 940" \
 "gpu_tests::1020::python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'"
