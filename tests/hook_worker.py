#!/usr/bin/env python
"""Child process of the fault-injection tests of tests/test_gpu_split.py.

It runs against libppnp_amd_test.so (the parent sets PPNP_AMD_LIB), the library built with the
test hooks (-DAPPNP_TESTING); the product library has none.

    python tests/hook_worker.py --case max-blocks|oom --data in.npz --out out.npz

in.npz: the CSR of A (indptr, indices, n) and H.  The graph is built with the source-blocked
copy requested while the hook makes it fail; the child checks the best-effort fallback (warning,
no copy, whole rows) and writes Z = APPNP_K(H) for the parent to compare with the oracle.
"""

import argparse
import os
import sys
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--case", required=True, choices=["max-blocks", "oom"])
    p.add_argument("--data", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--K", type=int, default=2)
    a = p.parse_args()

    import ppnp_amd
    from ppnp_amd import _lib

    if "testing=1" not in _lib.load().appnp_build_info().decode():
        raise SystemExit("needs PPNP_AMD_LIB=" + _lib.TEST_LIB_PATH)
    d = np.load(a.data, allow_pickle=False)
    n = int(d["n"])
    dev = torch.device("cuda:0")
    # max-blocks: a lower source-block limit (300k rows need 10 blocks of 2^15);
    # oom: the copy's entry array asks hipMalloc for 2^60 bytes
    hook = {"max-blocks": ("APPNP_SB_MAX_BLOCKS", "2"), "oom": ("APPNP_SB_TEST_OOM", "1")}[a.case]
    os.environ[hook[0]] = hook[1]
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        G = ppnp_amd.Graph.from_csr(d["indptr"], d["indices"], None, n, device=dev,
                                    source_blocks=True)
    del os.environ[hook[0]]
    warned = any("could not be built" in str(w.message) for w in caught)
    assert warned, [str(w.message) for w in caught]
    assert G.source_block_bytes() == 0 and G.source_block_layout() is None
    assert G.split_point(100) == 0 and G.remainder_cols(100) == 0
    H = torch.from_numpy(d["H"]).to(dev)
    Z = ppnp_amd.propagate_forward(G, H, a.K, 0.1)
    # the failed hipMalloc left no stale error: an unrelated torch kernel still runs
    x = torch.arange(1 << 20, device=dev, dtype=torch.float32).sum()
    torch.cuda.synchronize()
    assert torch.isfinite(Z).all() and float(x) > 0
    np.savez(a.out, Z=Z.cpu().numpy())
    print(f"[hook_worker] {a.case}: fallback to whole rows OK", flush=True)


if __name__ == "__main__":
    main()
