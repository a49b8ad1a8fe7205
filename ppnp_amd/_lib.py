"""ctypes binding of libppnp_amd.so (the C ABI declared in include/ppnp_amd.h).

This is the binding a maintainer of the reference would add: plain
pointers, sizes and a hipStream_t as ``void*``; no torch types cross the ABI.

There is deliberately NO fallback: if the shared library is missing or fails to load, every
entry point of ``ppnp_amd`` raises.  Build it with ``make -C ppnp_amd/csrc`` (or
``python -c "import __graft_entry__ as g; g.build()"``).
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PPNP_AMD_LIB", os.path.join(_HERE, "libppnp_amd.so"))
# the same library with the fault-injection hooks of the tests compiled in (make's test target;
# -DAPPNP_TESTING): tests run it in child processes through PPNP_AMD_LIB
TEST_LIB_PATH = os.path.join(_HERE, "libppnp_amd_test.so")
ABI_VERSION = 2  # PPNP_AMD_ABI_VERSION of include/ppnp_amd.h

APPNP_OK = 0
APPNP_EDEVICE = -5
APPNP_ENOMEM = -12
APPNP_EINVAL = -22
APPNP_ERANGE = -34
APPNP_ENOTSUP = -95

NORM = {"sym": 0, "rw": 1}
GRAPH_TRANSPOSE = 0x100
GRAPH_SOURCE_BLOCKS = 0x200
GRAPH_SB_W8 = 0x400  # remainder of up to 8 columns (include/ppnp_amd.h)
GRAPH_SB_W16 = 0x800  # up to 16

F32, BF16 = 0, 1
PART_ALL, PART_LOCAL, PART_REMOTE = 0, 1, 2
SHARDS_FIRST, SHARDS_ACC, SHARDS_LAST, SHARDS_ONLY = 0, 1, 2, 3  # appnp_shard_mode
KT_COPY, KT_STEP, KT_REM, KT_LOCAL, KT_REMOTE, KT_XCHG = 1, 2, 3, 4, 5, 6  # appnp_kernel_kind

_vp, _i64, _i32, _f32, _u64, _sz = C.c_void_p, C.c_int64, C.c_int, C.c_float, C.c_uint64, C.c_size_t

_SIGS = {
    "appnp_abi_version": (_i32, []),
    "appnp_build_info": (C.c_char_p, []),
    "appnp_strerror": (C.c_char_p, [_i32]),
    "appnp_graph_create": (_i32, [_vp, _vp, _vp, _i64, _i64, _i32, _vp, C.POINTER(_vp)]),
    "appnp_graph_create_rows": (
        _i32,
        [_vp, _vp, _vp, _i64, _i64, _i32, _i64, _i64, _i32, _vp, C.POINTER(_vp)],
    ),
    "appnp_graph_destroy": (None, [_vp]),
    "appnp_graph_info": (
        _i32,
        [_vp, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64),
         C.POINTER(_i32), C.POINTER(_i32)],
    ),
    "appnp_graph_csr": (_i32, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp)]),
    "appnp_graph_copy_csr": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "appnp_graph_dinv": (_i32, [_vp, C.POINTER(_vp)]),
    "appnp_workspace_bytes": (_sz, [_vp, _i64, _i64, _i32]),
    "appnp_propagate_split_point": (_i32, [_vp, _i64, _i32, C.POINTER(_i64)]),
    "appnp_propagate_remainder_cols": (_i32, [_vp, _i64, _i32, C.POINTER(_i64)]),
    "appnp_graph_source_blocks": (_i32, [_vp, C.POINTER(_i64)]),
    "appnp_graph_source_block_layout": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i64),
                                               C.POINTER(_i32), C.POINTER(_i32),
                                               C.POINTER(_i64)]),
    "appnp_propagate": (
        _i32,
        [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _f32, _f32, _u64, _vp, _sz, _vp],
    ),
    "appnp_propagate_bwd": (
        _i32,
        [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _f32, _f32, _u64, _vp, _sz, _vp],
    ),
    "appnp_standardize": (_i32, [_vp, _vp, _vp, _i64, _i64, _i32, _vp, C.POINTER(_vp)]),
    "appnp_csr_info": (_i32, [_vp, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64)]),
    "appnp_csr_copy": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "appnp_csr_destroy": (None, [_vp]),
    "appnp_csr_transpose": (_i32, [_vp, _vp, _vp, _i64, _i64, _i64, _vp, C.POINTER(_vp)]),
    "appnp_csr_values": (_i32, [_vp, _vp, _vp]),
    "appnp_spmm": (
        _i32,
        [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _f32, _u64, _i32, _vp],
    ),
    "appnp_plan_create": (
        _i32,
        [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _f32, _f32, _u64, _vp, _sz,
         C.POINTER(_vp)],
    ),
    "appnp_plan_launch": (_i32, [_vp, _vp]),
    "appnp_plan_destroy": (None, [_vp]),
    "appnp_dist_create": (
        _i32,
        [_vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, C.POINTER(_vp)],
    ),
    "appnp_dist_rows": (_i32, [_vp, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64)]),
    "appnp_dist_graph": (_vp, [_vp]),
    "appnp_dist_workspace_bytes": (_sz, [_vp, _i64, _i32]),
    "appnp_dist_propagate": (
        _i32,
        [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _f32, _f32, _u64, _vp, _sz, _vp],
    ),
    "appnp_dist_destroy": (None, [_vp]),
    "appnp_allgather_rccl": (_i32, [_vp, _sz, _i32, _i32, _vp, _vp]),
    "appnp_bcast_rccl": (_i32, [_vp, _sz, _i32, _i32, _vp, _vp]),
    "appnp_dist_set_broadcast": (_i32, [_vp, _vp, _vp, _vp]),
    "appnp_dist_pipeline_groups": (_i32, [_vp, _vp, _vp, _i32, C.POINTER(_i32)]),
    "appnp_line_rate_probe": (_i32, [_vp, _i64, _i64, _u64, _vp, _vp]),
    "appnp_kernel_timer_begin": (_i32, [_i32, _vp]),
    "appnp_kernel_timer_end": (_i32, [_vp, _vp, _i32, C.POINTER(_i32)]),
    "appnp_tuning_overrides": (C.c_char_p, []),
    "appnp_tuning_names": (C.c_char_p, []),
    "appnp_step": (
        _i32,
        [_vp, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _f32,
         _f32, _u64, _vp],
    ),
    "appnp_graph_shard_offsets": (_i32, [_vp, _i32, _i64, _vp]),
    "appnp_step_shards": (
        _i32,
        [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _f32,
         _f32, _u64, _vp],
    ),
    "appnp_step_split_shards": (
        _i32,
        [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _i64, _i32,
         _f32, _f32, _u64, _vp],
    ),
    "appnp_split_layout": (_i32, [_vp, _i64, C.POINTER(_i64), C.POINTER(_i64)]),
    "appnp_split_copy": (_i32, [_vp, _vp, _i64, _i64, _vp, _vp, _vp]),
    "appnp_step_split": (
        _i32,
        [_vp, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _i64, _i32, _f32,
         _f32, _u64, _vp],
    ),
}

EXPORTED = tuple(_SIGS)

# appnp_allgather_fn (include/ppnp_amd.h): in-place all-gather of equal row shards
ALLGATHER_FN = C.CFUNCTYPE(_i32, _vp, _sz, _i32, _i32, _vp, _vp)
# appnp_bcast_fn: in-place broadcast of one row shard from its owner
BCAST_FN = C.CFUNCTYPE(_i32, _vp, _sz, _i32, _i32, _vp, _vp)

_lib = None


class AppnpError(RuntimeError):
    def __init__(self, fn: str, code: int):
        self.code = code
        super().__init__(f"{fn} failed: {strerror(code)} ({code})")


def load():
    """Load (once) and return the ctypes handle; raises if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"ppnp_amd: native library not found at {LIB_PATH}; build it with "
            "`make -C ppnp_amd/csrc` (there is no CPU fallback)"
        )
    # The HIP runtime must be the one torch already loaded (same soname libamdhip64.so.7):
    # import torch first so our DT_NEEDED resolves to it.
    import torch  # noqa: F401

    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.appnp_abi_version() != ABI_VERSION:
        raise ImportError("ppnp_amd: ABI version mismatch")
    _lib = lib
    return lib


def strerror(code: int) -> str:
    try:
        return load().appnp_strerror(code).decode()
    except ImportError:
        return f"error {code}"


def check(fn: str, code: int) -> None:
    if code != APPNP_OK:
        raise AppnpError(fn, code)
