#!/usr/bin/env python
"""One row per bench line: the iteration time of the timed region beside roofline.kernel_ms (the
per-launch split of one untimed propagation, appnp_kernel_timer_*) and the box's line rate.

    python tools/kernel_split_table.py <label>=<bench log or json> ...
"""
import json
import sys


def line_of(path):
    with open(path) as fh:
        for s in fh:
            if s.startswith("{"):
                d = json.loads(s)
                return d.get("parsed", d)
    raise SystemExit(f"no JSON line in {path}")


def main():
    print(f"{'run':24s} {'ms/iter':>8s} {'main':>7s} {'rem':>7s} {'copy/call':>9s} "
          f"{'sum/iter':>8s} {'box G lines/s':>13s}")
    for arg in sys.argv[1:]:
        label, path = arg.split("=", 1)
        d = line_of(path)
        r = d["roofline"]
        k = r.get("kernel_ms") or {}

        def m(key):
            v = k.get(key)
            return f"{v['mean']:.4f}" if v else "-"

        print(f"{label:24s} {r['avg_launch_ms']:8.4f} {m('main'):>7s} {m('rem'):>7s} "
              f"{m('copy'):>9s} {k.get('sum_of_kernels', float('nan')):8.4f} "
              f"{r.get('box_line_rate') or float('nan'):13.2f}")


if __name__ == "__main__":
    main()
