"""bench.py with a periodic stack dump of every thread (faulthandler, every 60 s, to stderr):
locates where a multi-rank rehearsal stalls.  Usage: as bench.py, e.g.
torch.distributed.run --nproc-per-node 8 tools/bench_trace.py --gpus 8"""
import faulthandler
import os
import runpy
import sys

faulthandler.dump_traceback_later(60, repeat=True)
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
