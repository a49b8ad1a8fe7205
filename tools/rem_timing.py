#!/usr/bin/env python
"""Per-wave timeline of one remainder-pass launch (k_rem_persist) on products-synth.

Diagnostic only: needs the variant library built with wave timestamps (s_memrealtime, 100 MHz)
at the start, after the block sweep and at the end of every wave, plus its chunk count
(tools/bin/rem_timing.so: tools/rem_timing.patch applied to a copy of the sources; see DESIGN.md
4.2 and profiles/r3_rem_timeline.txt):

    tools/build_rem_timing.sh
    PPNP_AMD_LIB=tools/bin/rem_timing.so python tools/rem_timing.py

Prints where the launch's time goes: the start skew of the 4096 waves (dispatch), the spread of
their sweep times (imbalance), the epilogue, and the end skew -- the question of VERDICT r2 #7
(the pass's 0.09 ms over the probe's floor).
"""

import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import ppnp_amd
    from ppnp_amd import _lib, synth

    dev = torch.device("cuda", 0)
    n, m, F, K, alpha, _ = synth.CONFIGS["products-synth"]
    ip, ix = synth.graph_for("products-synth", device=dev)
    H = synth.features(n, F, device=dev)
    G = ppnp_amd.Graph.from_csr(ip, ix, None, n, device=dev, features=F)
    lib = _lib.load()
    lib.appnp_debug_rem_times.argtypes = [C.c_void_p, C.c_int]
    slots = 256 * 16
    buf = np.zeros(slots * 4, dtype=np.uint64)
    for K_ in (2, 10):
        for _ in range(3):
            ppnp_amd.propagate_forward(G, H, K_, alpha)
        torch.cuda.synchronize()
        assert lib.appnp_debug_rem_times(buf.ctypes.data, slots) == 0
        t = buf.reshape(slots, 4).astype(np.int64)
        t0 = t[:, 0].min()
        start, sweep, end, chunks = t[:, 0] - t0, t[:, 1] - t0, t[:, 2] - t0, t[:, 3]
        us = 0.01  # 100 MHz ticks -> microseconds
        dur = (sweep - start) * us
        print(f"K={K_} (last launch: the final iteration, epilogue into Z)")
        print(f"  launch span            {end.max() * us:8.1f} us")
        print(f"  wave start skew        {start.max() * us:8.1f} us  (median {np.median(start) * us:.1f})")
        print(f"  sweep duration         min {dur.min():.1f}  median {np.median(dur):.1f}  "
              f"max {dur.max():.1f} us")
        print(f"  sweep end              min {sweep.min() * us:.1f}  median {np.median(sweep) * us:.1f}"
              f"  max {sweep.max() * us:.1f} us")
        print(f"  epilogue               median {np.median(end - sweep) * us:.1f}  "
              f"max {(end - sweep).max() * us:.1f} us")
        print(f"  chunks per wave        min {chunks.min()}  median {np.median(chunks):.0f}  "
              f"max {chunks.max()}")
        c = np.corrcoef(chunks, dur)[0, 1]
        print(f"  corr(chunks, sweep)    {c:.3f}")
        wg = np.arange(slots) // 16
        wv = np.arange(slots) % 16
        per_wg = np.array([dur[wg == w].mean() for w in range(256)])
        per_wv = np.array([np.median(dur[wv == v]) for v in range(16)])
        print(f"  per-workgroup mean sweep: min {per_wg.min():.1f} median {np.median(per_wg):.1f} "
              f"max {per_wg.max():.1f} us; within-workgroup spread (max-min) median "
              f"{np.median([np.ptp(dur[wg == w]) for w in range(256)]):.1f} us")
        print("  per wave index median sweep: " + " ".join(f"{x:.0f}" for x in per_wv))
        slow = np.argsort(dur)[-16:]
        print("  16 slowest waves (workgroup, wave, chunks, sweep us): " +
              "; ".join(f"({wg[i]},{wv[i]},{chunks[i]},{dur[i]:.0f})" for i in slow))
        np.save(f"gpurun_out/rem_timing_K{K_}.npy", t)
        # by XCD (workgroup id mod 8) and by position of the CU
        xcd = (np.arange(slots) // 16) % 8
        for x in range(8):
            sel = xcd == x
            print(f"    xcd {x}: sweep median {np.median(dur[sel]):.1f} us, end max "
                  f"{end[sel].max() * us:.1f} us")


if __name__ == "__main__":
    main()
