"""CPU: bench.py's multi-GPU autotune (tune_layouts) over a gloo process group of 2 ranks.

The partitioned runner is replaced by a stub whose run() sleeps a layout-dependent time or
raises on ONE rank, so the test pins what the driver's N > 1 bench relies on: every rank
sees the same max-over-ranks times, picks the same layout, and a candidate that fails on any
rank is recorded as failed and skipped on all of them (agreed over the control group) instead
of ending the scaling run.  No GPU, no HIP library.
"""

import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _StubRunner:
    def __init__(self, tag, delay, fail):
        self.tag, self.delay, self.fail = tag, delay, fail

    def run(self):
        if self.fail == "run":
            raise RuntimeError(f"injected exchange failure in {self.tag}")
        time.sleep(self.delay)


def _worker(rank, world, port, plan, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from ppnp_amd import dist as pdist

        torch.cuda.synchronize = lambda *a, **k: None  # CPU: nothing queued on a device
        torch.cuda.empty_cache = lambda: None

        def create(indptr, indices, n, H, K, alpha, dev, layout, overlap, exchange):
            tag = f"{layout.rows}x{layout.cols}-{int(overlap)}"
            delay, fail_rank, where = plan[tag]
            fail = where if fail_rank in (rank, "all") else None
            if fail == "create":
                raise RuntimeError(f"injected build failure in {tag}")
            return _StubRunner(tag, delay, fail)

        pdist.PartitionedAPPNP.create = staticmethod(create)
        cands = [(pdist.Layout.parse(t.split("-")[0], world), t.endswith("-1"), "group")
                 for t in plan]
        try:
            best, times = bench.tune_layouts(cands, None, None, 0, None, 10, 0.1, "cpu", None,
                                             reps=2)
            q.put((rank, best.tag, times))
        except RuntimeError as e:
            q.put((rank, "error", str(e)))
    finally:
        dist.destroy_process_group()


def _run(plan, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _free_port(), plan, q), nprocs=world, join=True,
                       start_method="spawn")
    return sorted(q.get() for _ in range(world))


def test_autotune_agrees_and_skips_a_candidate_failing_on_one_rank():
    plan = {
        "1x2-0": (0.030, None, None),    # column layout: slow
        "2x1-1": (0.001, 1, "run"),      # row + overlap: fastest, but its exchange fails on rank 1
        "2x1-0": (0.010, 0, "create"),   # row: fails to build on rank 0
    }
    res = _run(plan)
    assert [r[0] for r in res] == [0, 1]
    for rank, best, times in res:
        assert best == "1x2-0", (rank, best, times)
        assert times["rows2xcols1-overlap"] is None and times["rows2xcols1"] is None
        assert times["rows1xcols2"] >= 30.0
    assert res[0][2] == res[1][2]  # the same (max-over-ranks) numbers on every rank


def test_autotune_picks_the_fastest():
    plan = {"1x2-0": (0.030, None, None), "2x1-1": (0.005, None, None)}
    res = _run(plan)
    assert all(best == "2x1-1" for _, best, _ in res)
    assert res[0][2] == res[1][2]


def test_autotune_all_failing_raises_on_every_rank():
    plan = {"1x2-0": (0.0, "all", "create"), "2x1-1": (0.0, 0, "run")}
    res = _run(plan)
    assert all(best == "error" and "every candidate layout failed" in msg
               for _, best, msg in res)


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
