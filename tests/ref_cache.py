"""The float64 reference Z_K of a full-size workload, computed once per GPU test session.

The products-scale parity tests (tests/test_gpu_configs.py and the row-partition workers in
tests/dist_worker.py) compare against the oracle's float64 torch.sparse CPU loop
(oracle/ppnp_oracle.py appnp_propagate_torch_cpu) over the device A_hat -- 10-20 s of the box's
CPU share per call.  With PPNP_SYNTH_CACHE naming a directory (tests/conftest.py sets one for
the session) the first caller's result is kept there as a .npy and every later caller, child
ranks included, reads it back: the same bits, since the loop is row-parallel and so
deterministic.  Test infrastructure only.
"""

import os

import numpy as np


def reference(tag, build, mmap=False):
    """The reference named ``tag`` (workload, H seed, K, alpha): ``build()`` -> a float64 numpy
    array, run only when no cached copy exists.  ``mmap`` returns a read-only memory map, for
    ranks that slice out their block."""
    cache = os.environ.get("PPNP_SYNTH_CACHE")
    if not cache:
        return build()
    path = os.path.join(cache, f"ref-{tag}.npy")
    if not os.path.exists(path):
        ref = np.ascontiguousarray(build(), dtype=np.float64)
        os.makedirs(cache, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp.npy"
        np.save(tmp, ref)
        os.replace(tmp, path)  # concurrent ranks never read a partial file
        if not mmap:
            return ref
    return np.load(path, mmap_mode="r" if mmap else None, allow_pickle=False)
