"""ppnp_amd -- MI355X (gfx950) APPNP propagation path for bkj/ppnp.

The hot path: A_hat construction (helpers.py:58-66) and the APPNP
propagation loop Z <- (1-a) A_hat Z + a H that replaces the dense PPR product of
model.py:63, as hand-written HIP kernels behind the C ABI in include/ppnp_amd.h.
"""

from . import _lib
from .graph import Graph
from .model import APPNP, PPNP, CustomLinear
from .ops import (propagate, propagate_backward, propagate_forward, split_copy, step,
                  step_split)
from .sparse import SparseFeatures, sparse_linear

__all__ = [
    "APPNP",
    "PPNP",
    "CustomLinear",
    "Graph",
    "propagate",
    "propagate_forward",
    "propagate_backward",
    "step",
    "step_split",
    "split_copy",
    "SparseFeatures",
    "sparse_linear",
    "_lib",
]
