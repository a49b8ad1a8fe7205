"""CPU: bench.py's multi-GPU candidate loop (run_candidates) over a gloo process group of 2 ranks.

The measurement of a layout is replaced by a stub that returns after a layout-dependent time,
raises or fails parity on ONE rank, or never returns, so the test pins what the driver's N > 1
bench relies on:

* every rank sees the same max-over-ranks results and reports the same layout;
* a candidate that fails on any rank (agreed over the control group) or fails parity is
  recorded and skipped instead of ending the scaling run;
* a candidate that stalls (an RCCL exchange that never completes) is ended by its deadline:
  rank 0 still prints the line of the exchange-free layout measured first, and every rank
  exits with status 0 instead of waiting for the process group's watchdog.

No GPU, no HIP library.
"""

import json
import os
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _rendezvous():
    """A file:// init method, fresh per run: no TCP port to race for between picking it and
    the store binding it (torch's FileStore removes the file when the last rank is done)."""
    import tempfile
    import uuid

    d = os.path.join(tempfile.gettempdir(), "ppnp_rdv")
    os.makedirs(d, exist_ok=True)
    return "file://" + os.path.join(d, uuid.uuid4().hex)


def _worker(rank, world, init, plan, out, timeout_s, budget_s=0.0):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    import bench

    bench.MIN_CANDIDATE_S = 0.5  # the budget's floor, scaled to the stubs' seconds
    t_start = time.monotonic() - 0.1 * rank  # the ranks' clocks differ: they agree on the max

    def measure(tag):
        delay, who, what = plan[tag]
        if isinstance(who, dict):  # a per-rank action
            what = who.get(rank)
            who = rank if what else None
        if who == rank and what == "die":  # a peer whose own deadline ended it early
            time.sleep(1.0)
            os._exit(0)
        mine = who in (rank, "all")
        if mine and what == "raise":
            raise RuntimeError(f"injected exchange failure in {tag}")
        if mine and what == "hang":
            time.sleep(3600)
        time.sleep(delay)
        ok = not (mine and what == "parity")
        return {"tag": tag, "ms_per_step": delay * 1e3, "config": {},
                "parity": {"ok": ok}}

    def emit(res):
        with open(f"{out}.{rank}", "w") as fh:
            fh.write(json.dumps(res))
            fh.flush()
            os.fsync(fh.fileno())

    try:
        best, times = bench.run_candidates(list(plan), measure, None, timeout_s, emit,
                                           lambda t: t, rank, world, abort=lambda: None,
                                           budget_s=budget_s,
                                           age=lambda: time.monotonic() - t_start)
        if rank == 0:
            emit(best)
    except RuntimeError as e:
        emit({"error": str(e)})
    finally:
        dist.destroy_process_group()


def _run(plan, tmp_path, world=2, timeout_s=60.0, budget_s=0.0):
    out = str(tmp_path / "line")
    init = _rendezvous()
    try:
        mp.start_processes(_worker, args=(world, init, plan, out, timeout_s, budget_s),
                           nprocs=world, join=True, start_method="spawn")
    finally:
        # a rank that leaves without destroying its group (the deadline paths) keeps the file
        if os.path.exists(init[len("file://"):]):
            os.remove(init[len("file://"):])
    res = {}
    for r in range(world):
        if os.path.exists(f"{out}.{r}"):
            res[r] = json.load(open(f"{out}.{r}"))
    return res


def test_candidates_agree_and_skip_failures(tmp_path):
    plan = {
        "col": (0.030, None, None),      # the exchange-free layout: slow
        "row-ov": (0.001, 1, "raise"),   # fastest, but its exchange fails on rank 1
        "row": (0.005, 0, "parity"),     # fast, but its result is wrong on rank 0
        "2x1": (0.010, None, None),      # the fastest that works
    }
    res = _run(plan, tmp_path)
    assert list(res) == [0]  # only rank 0 prints
    line = res[0]
    assert line["tag"] == "2x1"
    times = line["config"]["autotune_ms_per_step"]
    assert times["row-ov"] is None  # failed on one rank: skipped on both
    assert times["col"] >= 30.0 and times["2x1"] >= 10.0
    assert times["row"] is not None  # measured, but not eligible (parity)


def test_all_failing_raises_on_every_rank(tmp_path):
    plan = {"col": (0.0, "all", "raise"), "row": (0.0, 0, "raise")}
    res = _run(plan, tmp_path)
    assert set(res) == {0, 1}
    assert all("every candidate layout failed" in r["error"] for r in res.values())


def test_stalled_exchange_still_prints_the_column_line(tmp_path):
    """An exchange candidate that never returns on one rank (the other waits for it in the
    control group's agreement): both deadlines expire, rank 0 prints the column layout's line
    with the stalled candidate marked, and both processes exit 0 (start_processes raises
    otherwise)."""
    plan = {"col": (0.02, None, None), "2x4-multipath": (0.0, 1, "hang"),
            "never": (0.0, None, None)}
    t0 = time.time()
    res = _run(plan, tmp_path, timeout_s=4.0)
    assert time.time() - t0 < 60
    assert list(res) == [0]
    line = res[0]
    assert line["tag"] == "col"
    times = line["config"]["autotune_ms_per_step"]
    assert times["2x4-multipath"] == "timeout" and times["col"] >= 20.0
    assert "never" not in times


def test_peer_gone_during_agreement_still_prints_the_line(tmp_path):
    """Rank 0 fails a candidate and waits in the control group's agreement while rank 1 (stuck
    in the exchange rank 0 never joined) is ended by its own deadline first: rank 0's agreement
    then fails, and it must end like a deadline does -- the column layout's line printed, exit
    status 0 -- instead of raising out of the loop with no line."""
    plan = {"col": (0.02, None, None), "2x4-multipath": (0.0, {0: "raise", 1: "die"}, None),
            "never": (0.0, None, None)}
    res = _run(plan, tmp_path, timeout_s=30.0)
    assert list(res) == [0]
    line = res[0]
    assert line["tag"] == "col"
    assert line["config"]["autotune_ms_per_step"]["2x4-multipath"] == "timeout"


def test_run_budget_skips_candidates_and_prints_the_column_line(tmp_path):
    """slow-but-not-stalled candidates cannot together outlast the driver's
    timeout.  With a 3 s budget the first exchange candidate (2.7 s) is measured, then less than
    MIN_CANDIDATE_S is left: the rest are skipped on both ranks, rank 0 prints the fastest line
    (the column layout's) and both processes exit 0."""
    plan = {"col": (0.02, None, None), "row": (2.7, None, None), "2x1": (0.01, None, None),
            "1x2": (0.01, None, None)}
    t0 = time.time()
    res = _run(plan, tmp_path, timeout_s=60.0, budget_s=3.0)
    assert time.time() - t0 < 60
    assert list(res) == [0]
    line = res[0]
    assert line["tag"] == "col"
    times = line["config"]["autotune_ms_per_step"]
    assert times["row"] >= 2700.0
    assert times["2x1"] == times["1x2"] == "skipped: run budget"


def test_run_budget_cuts_a_running_candidate_short(tmp_path):
    """A candidate that starts with budget left but would run past it is ended by a deadline of
    the budget left (not the much longer candidate timeout): the column line is printed, the
    candidate marked "timeout", and both processes exit 0."""
    plan = {"col": (0.02, None, None), "row": (1.0, None, None), "2x1": (30.0, None, None),
            "never": (0.0, None, None)}
    t0 = time.time()
    res = _run(plan, tmp_path, timeout_s=120.0, budget_s=3.0)
    assert time.time() - t0 < 60
    assert list(res) == [0]
    line = res[0]
    assert line["tag"] == "col"
    times = line["config"]["autotune_ms_per_step"]
    assert times["2x1"] == "timeout" and "never" not in times


if __name__ == "__main__":
    pytest.main([__file__, "-q"])


def test_process_age_distrusts_a_foreign_clock(monkeypatch):
    """The run budget's clock: the process's start time, unless it lies before this module's
    import by more than 15 minutes (a clock the container does not share)."""
    import types

    import bench

    assert 0.0 <= bench.process_age_s() < 900.0
    fake = types.SimpleNamespace(Process=lambda: types.SimpleNamespace(
        create_time=lambda: time.time() - 10 * 3600))
    monkeypatch.setitem(__import__("sys").modules, "psutil", fake)
    age = bench.process_age_s()
    assert age < 900.0
