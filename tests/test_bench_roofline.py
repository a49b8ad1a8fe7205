"""CPU: the roofline block bench.py prints is self-consistent for every kind of iteration the
runs take -- one GPU with split rows, a narrow 8-rank column slab that runs wholly in the
remainder pass, a row-layout rank with an exchange, and a graph with gather locality.

The ceiling is a lower bound on the iteration time, so ``ceiling.frac >= frac`` always (the
round-2 rehearsal line reported a ceiling from the streams alone, with 0 lines per nonzero).
No GPU: ``bench.roofline`` is plain arithmetic on the shape and the measured time."""

import pytest

import bench

N, NNZ, F = 2_449_029, 126_165_965, 100


def _check(rl, measured_ms):
    assert rl["avg_launch_ms"] == measured_ms
    assert 0 < rl["frac"] <= rl["ceiling"]["frac"] <= 1.0 + 1e-12
    assert rl["ceiling"]["ms_per_iter"] <= measured_ms
    assert rl["achieved"] == pytest.approx(rl["bytes_per_launch"] / (measured_ms * 1e-3) / 1e9)
    return rl


def test_single_gpu_split_rows():
    rl = _check(bench.roofline(n=N, rows=N, nnz=NNZ, F_local=F, esz=4, avg_iter_ms=7.79, fs=96,
                               r=4, lpe=1, rb_total=136_000_000, rb_entry_bytes=4), 7.79)
    # B_iter = 4(N+1) + 8 nnz + 3 N F s on one GPU
    assert rl["bytes_per_launch"] == 4 * (N + 1) + 8 * NNZ + 3 * N * F * 4
    assert rl["ceiling"]["lines_per_nonzero"] == 3
    assert rl["ceiling"]["remainder_l2_requests_per_nonzero"] == 1
    assert 0.06 < rl["frac"] < 0.07 and rl["ceiling"]["frac"] < 0.08
    assert not rl["ceiling"]["clamped_to_measured"]


def test_whole_rows_count_four_lines():
    rl = _check(bench.roofline(n=N, rows=N, nnz=NNZ, F_local=F, esz=4, avg_iter_ms=9.57, fs=F,
                               r=0, lpe=1), 9.57)
    assert rl["ceiling"]["lines_per_nonzero"] == 4  # a 400-B packed row spans 4 lines


def test_narrow_column_slab_in_the_remainder_pass():
    """13 of 100 columns on 8 ranks: no direct gather (0 lines per nonzero), 4 L2 requests per
    nonzero in the W16 pass, and a ceiling from its streamed entries and rows."""
    rl = _check(bench.roofline(n=N, rows=N, nnz=NNZ, F_local=13, esz=4, avg_iter_ms=2.015,
                               fs=0, r=13, lpe=4, rb_total=137_000_000, rb_entry_bytes=4), 2.015)
    assert rl["ceiling"]["lines_per_nonzero"] == 0
    assert rl["ceiling"]["remainder_l2_requests_per_nonzero"] == 4
    assert rl["bytes_per_launch"] == 4 * (N + 1) + 8 * NNZ + 3 * N * 13 * 4
    # the round-3 rehearsal line read ceiling.frac 1.57 before the L2 and HBM terms: the bound
    # is now the remainder gathers at the L2 peak plus the streams, never above the roofline
    c = rl["ceiling"]
    assert c["remainder_l2_bytes"] == NNZ * 64 and c["ms_per_iter"] >= c["hbm_ms"]


def test_row_layout_rank_with_exchange():
    rows, nnz = -(-N // 8), NNZ // 8
    ex = 7 * rows * F * 4
    rl = _check(bench.roofline(n=N, rows=rows, nnz=nnz, F_local=F, esz=4, avg_iter_ms=2.5,
                               fs=F, r=0, lpe=1, exchange_in_bytes=ex), 2.5)
    # the rank reads all n rows of Z_k (gathered), its own H rows and writes its Z rows
    assert rl["bytes_per_launch"] == 4 * (rows + 1) + 8 * nnz + (N + 2 * rows) * F * 4
    c = rl["ceiling"]
    assert c["exchange_in_bytes"] == ex and c["exchange_ms"] > c["compute_ms"]
    assert c["ms_per_iter"] == c["exchange_ms"]  # the 857 MB all-gather bounds this layout


def test_gather_locality_clamps_the_ceiling():
    """products-local runs faster than the uniform-gather bound (L2 hits): the ceiling is the
    measured time and the note says why, so ceiling.frac == frac rather than below it."""
    rl = _check(bench.roofline(n=N, rows=N, nnz=NNZ, F_local=F, esz=4, avg_iter_ms=4.0, fs=F,
                               r=0, lpe=1), 4.0)
    assert rl["ceiling"]["clamped_to_measured"]
    assert rl["ceiling"]["frac"] == pytest.approx(rl["frac"])
    assert "locality" in rl["note"]


def test_kernel_plan_names_what_runs():
    sb = {"width": 4, "entries": 10, "value_free": True, "row_passes": 1, "launches": 0}
    desc, key, fs, r, lpe = bench.kernel_plan(100, 10, 4, sb)
    assert (fs, r, lpe) == (96, 4, 1) and key == "k_step[0,96)+k_rem_persist<W4,vf>[96,100)"
    assert bench.kernel_plan(100, 10, 0, None)[1] == "k_step"
    sb16 = dict(sb, width=16, value_free=False, row_passes=4)
    desc, key, fs, r, lpe = bench.kernel_plan(13, 10, 13, sb16)
    assert (fs, r, lpe) == (0, 13, 4) and key == "k_rem_persist<W16>[0,13)"
    # K = 1 never splits
    assert bench.kernel_plan(100, 1, 4, sb)[1] == "k_step"


def test_traffic_key_tracks_kernels_and_sources():
    k1 = bench.traffic_key("products-synth", "f32", "single", "k_step")
    k2 = bench.traffic_key("products-synth", "f32", "single", "k_step[0,96)+k_rem_persist<W4>")
    assert k1 != k2 and k1.startswith("products-synth:f32:single:k_step:src=")
    assert bench.committed_traffic("no-such-key") is None


def test_cpu_leg_threads_and_sample(monkeypatch):
    """N > 1: torch.distributed.run sets OMP_NUM_THREADS=1 per rank, but rank 0 runs the CPU leg
    while the others wait, so it takes up to 16 visible CPUs; N = 1 keeps the box's share.  The
    N > 1 sample is bounded: 1 products-synth iteration, all K = 10 of arxiv-synth."""
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(64)), raising=False)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.cpu_threads(1) == (1, 64)
    assert bench.cpu_threads(8) == (16, 64)
    monkeypatch.setenv("OMP_NUM_THREADS", "32")
    assert bench.cpu_threads(8) == (32, 64)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(4)), raising=False)
    assert bench.cpu_threads(8) == (4, 4)
    for workload, iters in (("products-synth", 1), ("arxiv-synth", 10)):
        n, m, f, k = bench_config(workload)
        assert max(1, min(k, int(bench.CPU_LEG_WORK // (m * 2 * f)))) == iters


def bench_config(workload):
    from ppnp_amd import synth

    n, m, f, k = synth.CONFIGS[workload][:4]
    return n, m, f, k
