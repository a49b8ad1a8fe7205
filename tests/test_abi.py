"""CPU: the C-ABI library loads and exports every symbol include/ppnp_amd.h declares.

No compute call is made (there is no GPU here); only argument validation that returns
before touching the device.
"""

import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ppnp_amd.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(appnp_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = declared()
    for must in ("appnp_graph_create", "appnp_propagate", "appnp_propagate_bwd",
                 "appnp_step", "appnp_workspace_bytes", "appnp_graph_destroy",
                 "appnp_strerror"):
        assert must in names


def test_library_exports_all_declared_symbols():
    from ppnp_amd import _lib

    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), f"missing export {name}"
    assert set(_lib.EXPORTED) == set(declared())


def test_abi_version_and_strerror():
    from ppnp_amd import _lib

    lib = _lib.load()
    assert lib.appnp_abi_version() == _lib.ABI_VERSION == 2
    assert lib.appnp_strerror(0) == b"ok"
    assert lib.appnp_strerror(_lib.APPNP_EINVAL) == b"invalid argument"
    assert lib.appnp_strerror(_lib.APPNP_ENOTSUP) == b"not supported"


def test_build_info_names_the_sources_of_this_tree():
    """the library carries the digest of the HIP sources it was compiled from
    (Makefile -> appnp_build_info), and it equals the digest of the sources in this tree
    (ppnp_amd/csrc/srcdigest.py, what bench.py prints beside it).  A stale build fails here."""
    import bench

    info = bench.build_info()
    assert info["info"].startswith("src=") and "arch=gfx950" in info["info"]
    assert info["match"], info


def test_line_rate_probe_validates_arguments():
    """appnp_line_rate_probe returns before any launch on bad arguments (no device here)."""
    from ppnp_amd import _lib

    lib = _lib.load()
    sink = C.c_void_p(0x1000)
    assert lib.appnp_line_rate_probe(None, 1 << 20, 10, 0, sink, None) == _lib.APPNP_EINVAL
    # a table base that is not 128-B aligned, a table under one line, a negative count
    assert lib.appnp_line_rate_probe(C.c_void_p(0x1040), 1 << 20, 10, 0, sink,
                                     None) == _lib.APPNP_EINVAL
    assert lib.appnp_line_rate_probe(C.c_void_p(0x1000), 64, 10, 0, sink,
                                     None) == _lib.APPNP_EINVAL
    assert lib.appnp_line_rate_probe(C.c_void_p(0x1000), 1 << 20, -1, 0, sink,
                                     None) == _lib.APPNP_EINVAL
    assert lib.appnp_line_rate_probe(C.c_void_p(0x1000), 1 << 20, 0, 0, sink,
                                     None) == _lib.APPNP_OK  # nothing to do


def test_kernel_timer_validates_arguments():
    """appnp_kernel_timer_begin / _end: bad capacities and an end without a begin return codes
    before any device call."""
    from ppnp_amd import _lib

    lib = _lib.load()
    n = C.c_int(-1)
    assert lib.appnp_kernel_timer_begin(0, None) == _lib.APPNP_EINVAL
    assert lib.appnp_kernel_timer_begin(-3, None) == _lib.APPNP_EINVAL
    assert lib.appnp_kernel_timer_begin(1 << 21, None) == _lib.APPNP_EINVAL
    assert lib.appnp_kernel_timer_end(None, None, 0, C.byref(n)) == _lib.APPNP_EINVAL


def test_argument_validation_without_device():
    """Errors are returned as codes, never raised/aborted across the ABI."""
    from ppnp_amd import _lib

    lib = _lib.load()
    out = C.c_void_p()
    # bad mode
    assert lib.appnp_graph_create(None, None, None, 0, 0, 7, None, C.byref(out)) == _lib.APPNP_EINVAL
    # negative sizes
    assert lib.appnp_graph_create(None, None, None, -1, 0, 0, None, C.byref(out)) == _lib.APPNP_EINVAL
    # n > int32 range
    assert lib.appnp_graph_create(None, None, None, 2**31, 0, 0, None, C.byref(out)) == _lib.APPNP_ERANGE
    # null graph handle
    assert lib.appnp_propagate(None, None, 0, None, 0, 1, 0, 1, 0.1, 0.0, 0, None, 0, None) == _lib.APPNP_EINVAL
    assert lib.appnp_propagate_bwd(None, None, 0, None, 0, 1, 0, 1, 0.1, 0.0, 0, None, 0, None) == _lib.APPNP_EINVAL
    assert lib.appnp_step(None, 0, None, 0, None, 0, None, 0, None, 0, 1, 0, 0, 0.1, 0.0, 0, None) == _lib.APPNP_EINVAL
    assert lib.appnp_workspace_bytes(None, 10, 10, 0) == 0
    lib.appnp_graph_destroy(None)  # no-op
    # the row-partitioned engine: validation before any device work
    h = C.c_void_p()
    assert lib.appnp_dist_create(None, None, None, 10, 0, 0, 0, 2, 1, None, None, None,
                                 C.byref(h)) == _lib.APPNP_EINVAL  # 2 ranks, no exchange
    assert lib.appnp_dist_create(None, None, None, 10, 0, 0, 2, 2, 0, None, None, None,
                                 C.byref(h)) == _lib.APPNP_EINVAL  # rank out of range
    assert lib.appnp_dist_create(None, None, None, 10, 0, 0, 0, 1, 0, None, None, None,
                                 None) == _lib.APPNP_EINVAL
    assert lib.appnp_dist_propagate(None, None, 0, None, 0, 1, 0, 1, 0.1, 0.0, 0, None, 0,
                                    None) == _lib.APPNP_EINVAL
    assert lib.appnp_dist_rows(None, None, None, None) == _lib.APPNP_EINVAL
    assert lib.appnp_dist_graph(None) is None
    assert lib.appnp_dist_workspace_bytes(None, 10, 0) == 0
    assert lib.appnp_allgather_rccl(None, 16, 0, 1, None, None) == _lib.APPNP_EINVAL
    lib.appnp_dist_destroy(None)  # no-op


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    """The product path fails loudly when the HIP extension is absent."""
    import importlib

    from ppnp_amd import _lib

    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError):
        _lib.load()
    importlib.reload(_lib)


def test_torch_library_ops_registered_with_fake_kernels():
    """ppnp_amd::propagate / propagate_bwd are dispatcher ops with fake (meta) kernels, so
    torch.compile can trace them; shapes propagate without touching a device."""
    import torch

    import ppnp_amd  # noqa: F401  (registers the ops)

    for name in ("propagate", "propagate_bwd"):
        op = getattr(torch.ops.ppnp_amd, name)
        H = torch.empty(7, 3, device="meta")
        Z = op(H, 1, 10, 0.1, 0.0, 0)
        assert Z.shape == (7, 3) and Z.device.type == "meta" and Z.dtype == H.dtype
    with pytest.raises(RuntimeError):
        from ppnp_amd.graph import Graph

        Graph.lookup(10**9)  # not a live graph: loud, no fallback


def test_product_library_carries_no_test_or_measurement_hooks():
    """the fault injectors of the tests live in libppnp_amd_test.so only
    (-DAPPNP_TESTING), and the losing XCD-pacing experiment is gone, so the shipped library
    names none of them; the test library does name its hooks."""
    from ppnp_amd import _lib

    prod = open(_lib.LIB_PATH, "rb").read()
    for bad in (b"_TEST_", b"_PACE_", b"APPNP_SB_MAX_BLOCKS", b"ALLHIT"):
        assert bad not in prod, bad
    test = open(_lib.TEST_LIB_PATH, "rb").read()
    for hook in (b"APPNP_SB_TEST_OOM", b"APPNP_SB_MAX_BLOCKS", b"APPNP_DIST_TEST_AGREE_FAIL"):
        assert hook in test, hook


def _overrides_in_child(env_extra):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if not k.startswith("APPNP_")}
    env.update(env_extra, PYTHONPATH=ROOT)
    code = ("from ppnp_amd import _lib; lib = _lib.load(); "
            "print(lib.appnp_tuning_overrides().decode() + '|' + "
            "lib.appnp_tuning_names().decode())")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=120, check=True).stdout.strip().splitlines()[-1]
    active, names = out.split("|")
    return active, names.split(";")


def test_tuning_overrides_need_APPNP_TUNING():
    """a stray tuning variable in the environment changes nothing unless
    APPNP_TUNING=1 is set too, and then appnp_tuning_overrides names it (bench.py prints it as
    build.overrides)."""
    active, names = _overrides_in_child({"APPNP_UW": "4", "APPNP_SPLIT": "0"})
    assert active == ""
    assert {"APPNP_UW", "APPNP_SPLIT", "APPNP_VEC", "APPNP_REM_SYNC_W16"} <= set(names)
    active, _ = _overrides_in_child({"APPNP_UW": "4", "APPNP_SPLIT": "0", "APPNP_TUNING": "1"})
    assert active == "APPNP_SPLIT=0;APPNP_UW=4"
    active, _ = _overrides_in_child({"APPNP_TUNING": "1"})
    assert active == ""
