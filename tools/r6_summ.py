#!/usr/bin/env python
"""Print one line per bench log (gpurun_out/<name>.log): per-step ms, remainder / main kernel
means, row passes, direct rows and overrides.  Usage: tools/r6_summ.py name [name ...]"""
import json
import sys

for name in sys.argv[1:]:
    path = name if name.endswith((".log", ".json")) else f"gpurun_out/{name}.log"
    try:
        line = [ln for ln in open(path) if ln.startswith("{")][-1]
    except (OSError, IndexError):
        print(f"{name}: no line")
        continue
    d = json.loads(line)
    rl = d["roofline"]
    km = rl.get("kernel_ms") or {}
    g = lambda k: (km.get(k) or {}).get("mean")  # noqa: E731
    sb = rl.get("source_blocks") or {}
    fmt = lambda x: f"{x:.4f}" if isinstance(x, float) else str(x)  # noqa: E731
    print(f"{name}: step {d['ms_per_step']:.3f} ms  main {fmt(g('main'))}  local {fmt(g('local'))}"
          f"  remote {fmt(g('remote'))}  rem {fmt(g('rem'))}  copy {fmt(g('copy'))}"
          f"  passes {sb.get('row_passes')} cols {sb.get('cols')} direct {sb.get('direct_rows')}"
          f"  frac {rl['frac']:.4f}  box {fmt(rl.get('box_line_rate'))}"
          f"  ovr {d['build'].get('overrides')}  parity {(d.get('parity') or {}).get('max_abs_err')}")
