"""GPU: the in-library random-line probe behind bench.py's roofline.box_line_rate
(appnp_line_rate_probe, ppnp_amd/csrc/appnp_probe.hip) and the bench line's build provenance.

The probe only reads its table, so it must leave it untouched; it must handle tables of any
size (a whole number of lines is gathered from a 128-B aligned start inside the storage) and
report a rate in the range the gather probe measured (tools/gather_probe.hip: 53-60 G lines/s
for 64 MB-1 GB tables on an idle MI355X)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.mark.parametrize("nbytes", [128, 4096 + 44, 1 << 20, 1 << 28])
def test_probe_reads_only_and_reports_a_rate(nbytes):
    from ppnp_amd.ops import line_rate_probe

    t = torch.arange(nbytes // 4, dtype=torch.float32, device=DEV)
    before = t.clone()
    res = line_rate_probe(t, 1 << 22)
    torch.cuda.synchronize()
    assert torch.equal(t, before)
    assert res["lines"] == 1 << 22 and res["ms"] > 0 and res["G_lines_s"] > 0
    assert res["table_MB"] * 2**20 <= t.untyped_storage().nbytes()


def test_probe_rate_on_a_bench_sized_table():
    """A 1 GB table (the bench's H): the rate lands in the band the standalone probe measured,
    with room for box-to-box spread."""
    from ppnp_amd.ops import line_rate_probe

    t = torch.zeros(1 << 28, dtype=torch.float32, device=DEV)
    res = line_rate_probe(t, 1 << 30)
    assert 30.0 < res["G_lines_s"] < 120.0, res


def test_bench_build_info_matches_the_tree():
    """The library this process loaded was compiled from the sources in this tree."""
    import bench

    info = bench.build_info()
    assert info["match"], info


def _split_graph(n=200_000, m=2_000_000, F=100):
    import ppnp_amd
    from ppnp_amd import synth

    indptr, indices = synth.uniform_graph(n, m, seed=11, device=DEV)
    g = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=DEV, features=F)
    H = synth.features(n, F, device=DEV, seed=3)
    return g, H


def test_kernel_timer_splits_a_propagation_by_launch():
    """appnp_kernel_timer_* times every launch of one call.  A split F = 100
    propagation enqueues the split copy, then K x (SpMM on the main columns, remainder pass);
    whole rows enqueue K SpMM launches.  Every interval is a positive device time, and the
    timed call computes exactly what an untimed one does."""
    import ppnp_amd
    from ppnp_amd.ops import kernel_times

    g, H = _split_graph()
    K = 3
    assert g.remainder_cols(100, torch.float32) == 4
    ref = ppnp_amd.propagate_forward(g, H, K, 0.1)
    out = torch.empty_like(ref)
    t = kernel_times(lambda: ppnp_amd.propagate_forward(g, H, K, 0.1, out=out), DEV)
    torch.cuda.synchronize()
    assert [k for k, _ in t] == ["copy"] + ["step", "rem"] * K
    assert all(ms > 0 and ms == ms for _, ms in t), t
    assert torch.equal(out, ref)
    # whole rows (F = 32: one line per row, no split)
    H32 = H[:, :32].contiguous()
    t = kernel_times(lambda: ppnp_amd.propagate_forward(g, H32, K, 0.1), DEV)
    assert [k for k, _ in t] == ["step"] * K and all(ms > 0 for _, ms in t)


def test_kernel_timer_overflow_and_state():
    """More launches than the capacity: the first ones are timed and the call reports
    APPNP_ERANGE; the timer is off afterwards (a second end is EINVAL)."""
    import ctypes as C

    import ppnp_amd
    from ppnp_amd import _lib

    g, H = _split_graph(n=70_000, m=300_000, F=32)
    lib = _lib.load()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.appnp_kernel_timer_begin(2, s) == _lib.APPNP_OK
    ppnp_amd.propagate_forward(g, H, 5, 0.1)
    ms = (C.c_float * 2)()
    kinds = (C.c_int * 2)()
    n = C.c_int(0)
    assert lib.appnp_kernel_timer_end(ms, kinds, 2, C.byref(n)) == _lib.APPNP_ERANGE
    assert n.value == 2 and list(kinds) == [_lib.KT_STEP] * 2 and min(ms) > 0
    assert lib.appnp_kernel_timer_end(ms, kinds, 2, C.byref(n)) == _lib.APPNP_EINVAL
