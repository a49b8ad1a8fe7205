#!/usr/bin/env python
"""End-to-end check of the multi-GPU path on real HIP kernels.

    torchrun --nproc-per-node P --master-addr 127.0.0.1 tests/dist_worker.py --layout row|col|RxC
        [--overlap] [--exchange multipath|group] [--graph-n 60000] [--graph-m 400000] [--f 20]
        [--K 10]
        [--p-drop 0.0] [--workload arxiv-synth] [--oracle]

Every rank runs its share (ppnp_amd.dist.PartitionedAPPNP) and compares its block of Z_K with
the single-GPU propagation of the whole graph computed on its own device.  Backend: RCCL when
the layout has row groups, gloo otherwise; PPNP_DIST_BACKEND=gloo forces gloo (lets P ranks
share one GPU on a single-GPU box; the all-gather then stages through host memory).
Exit status 1 on mismatch.
"""

import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _require_test_library():
    """Fault injection needs libppnp_amd_test.so (the product library has no hooks): the test
    sets PPNP_AMD_LIB; fail loudly rather than run without the injected fault."""
    from ppnp_amd import _lib

    if "testing=1" not in _lib.load().appnp_build_info().decode():
        raise SystemExit("fault injection needs PPNP_AMD_LIB=" + _lib.TEST_LIB_PATH)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--layout", default="col")
    p.add_argument("--overlap", action="store_true")
    p.add_argument("--exchange", default="multipath", choices=["multipath", "group"])
    # not --n / --m: torch.distributed.run would take them as abbreviations of its own options
    p.add_argument("--graph-n", dest="n", type=int, default=60000)
    p.add_argument("--graph-m", dest="m", type=int, default=400000)
    p.add_argument("--f", type=int, default=20)
    p.add_argument("--K", type=int, default=None, help="iterations (default 10, or the "
                                                       "workload's K)")
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--p-drop", type=float, default=0.0)
    p.add_argument("--workload", default=None,
                   help="a ppnp_amd.synth.CONFIGS graph (its n, m, F, K, alpha, seed) instead of "
                        "--n/--m/--f/--K/--alpha")
    p.add_argument("--oracle", action="store_true",
                   help="compare with the float64 CPU oracle (oracle/ppnp_oracle.py) instead of "
                        "the single-GPU HIP propagation")
    p.add_argument("--oracle-torch", action="store_true",
                   help="compare with the oracle's float64 torch.sparse CPU loop over the device "
                        "A_hat of a whole-graph build (products scale: tests/test_gpu_configs.py "
                        "pins that A_hat to calc_a_hat entry by entry)")
    p.add_argument("--oracle-rank0", action="store_true",
                   help="with --oracle-torch: rank 0 alone runs the oracle and sends every rank "
                        "its block (gloo point to point), instead of every rank running it -- "
                        "8 products-scale fp64 oracles would not fit the box's CPU share")
    p.add_argument("--h-seed", type=int, default=1,
                   help="seed of H (synth.features); with --oracle-torch on a workload the "
                        "reference is shared through tests/ref_cache.py, so seed 0 reads the "
                        "session's products reference instead of recomputing it")
    p.add_argument("--pipeline", default="auto", choices=["auto", "on", "off"],
                   help="the pipelined exchange (one broadcast per row shard, the product per "
                        "group of arrived shards): auto = whenever it applies")
    p.add_argument("--expect-split", type=int, default=None,
                   help="fail unless the rank's remainder columns (split rows) equal this")
    p.add_argument("--sb-oom-rank", type=int, default=-1,
                   help="this rank's source-blocked copy fails to build (APPNP_SB_TEST_OOM): "
                        "every rank must then keep whole rows")
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)

    import ppnp_amd
    from ppnp_amd import dist as pdist
    from ppnp_amd import synth

    layout = pdist.Layout.parse(a.layout, world)
    backend = os.environ.get("PPNP_DIST_BACKEND") or ("nccl" if layout.rows > 1 else "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    rank = dist.get_rank()
    if a.workload:
        a.n, a.m, a.f, K, a.alpha, _ = synth.CONFIGS[a.workload]
        a.K = K if a.K is None else a.K
        indptr, indices = synth.graph_for(a.workload, device=dev)
    else:
        a.K = 10 if a.K is None else a.K
        indptr, indices = synth.uniform_graph(a.n, a.m, 7, device=dev)
    H = synth.features(a.n, a.f, device=dev, seed=a.h_seed)
    if rank == a.sb_oom_rank:
        _require_test_library()
        os.environ["APPNP_SB_TEST_OOM"] = "1"
    runner = pdist.PartitionedAPPNP.create(indptr, indices, a.n, H, a.K, a.alpha, dev,
                                           layout=layout, overlap=a.overlap,
                                           p_drop=a.p_drop, seed=5, exchange=a.exchange,
                                           pipeline={"auto": None, "on": True,
                                                     "off": False}[a.pipeline])
    Z = runner.run()
    torch.cuda.synchronize()
    if a.oracle_torch and a.oracle_rank0:
        if dist.get_backend() != "gloo":
            raise SystemExit("--oracle-rank0 sends the blocks over gloo")
        ref = (torch.from_numpy(_torch_oracle(a, indptr, indices, H, dev, threads=16))
               if rank == 0 else None)
        block, ref_max = _send_blocks(ref, (runner.lo, runner.hi, runner.f_lo, runner.f_hi),
                                      rank, world)
        del ref
    elif a.oracle_torch:
        ref = _torch_oracle(a, indptr, indices, H, dev, threads=8, mmap=True)
        block = torch.from_numpy(np.array(ref[runner.lo:runner.hi, runner.f_lo:runner.f_hi]))
        ref_max = float(np.abs(ref).max())
        del ref
    elif a.oracle:
        ref = _fp64_oracle(a, indptr, indices, H, rank)
        block = torch.from_numpy(np.array(ref[runner.lo:runner.hi, runner.f_lo:runner.f_hi]))
        ref_max = float(np.abs(ref).max())
        del ref
    else:
        G = ppnp_amd.Graph.from_csr(indptr, indices, None, a.n, device=dev)
        ref = ppnp_amd.propagate_forward(G, H, a.K, a.alpha, p_drop=a.p_drop, seed=5)
        block = ref[runner.lo:runner.hi, runner.f_lo:runner.f_hi]
        ref_max = ref.abs().max().item()
    got = Z if Z.device == block.device else Z.cpu()
    err = (got.double() - block.double()).abs().max().item() if block.numel() else 0.0
    tol = 1e-5 * ref_max + 1e-6
    ok = err <= tol
    if a.expect_split is not None:
        ok = ok and runner.remainder_cols == a.expect_split
    print(f"[dist_worker] rank {rank}/{world} backend={dist.get_backend()} layout={layout} "
          f"overlap={runner.overlap} exchange={runner.exchange} split_cols={runner.remainder_cols} "
          f"pipeline={runner.pipeline} "
          f"rows [{runner.lo},{runner.hi}) "
          f"cols [{runner.f_lo},"
          f"{runner.f_hi}) reference={'oracle' if a.oracle or a.oracle_torch else 'hip'} "
          f"max err {err:.3e} "
          f"tol {tol:.3e} -> {'OK' if ok else 'FAIL'}",
          flush=True)
    flag = torch.tensor([0 if ok else 1], dtype=torch.int64,
                        device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag)
    dist.destroy_process_group()
    sys.exit(1 if flag.item() else 0)


def _fp64_oracle(a, indptr, indices, H, rank):
    """The float64 oracle (oracle/ppnp_oracle.py appnp_propagate over calc_a_hat, scipy) of this
    run's graph, H, K, alpha and dropout.  With the session's cache (tests/ref_cache.py) rank 0
    computes it and the other ranks wait at a barrier and map it, so ranks do not compete for the
    box's CPU share and later runs of the same case read it back."""
    import scipy.sparse as sp

    import ref_cache
    from oracle import ppnp_oracle as O

    def build():
        adj = sp.csr_matrix((np.ones(indices.numel(), dtype=np.float32),
                             indices.cpu().numpy(), indptr.cpu().numpy()), shape=(a.n, a.n))
        return O.appnp_propagate(O.calc_a_hat(adj, "sym"), H.double().cpu().numpy(), a.K,
                                 a.alpha, p_drop=a.p_drop, seed=5)

    if not os.environ.get("PPNP_SYNTH_CACHE"):
        return build()
    graph = a.workload or f"uniform-n{a.n}-m{a.m}-s7"
    tag = f"{graph}-f{a.f}-h{a.h_seed}-K{a.K}-a{a.alpha}-p{a.p_drop}-s5"
    if rank == 0:
        ref_cache.reference(tag, build, mmap=True)
    dist.barrier()
    return ref_cache.reference(tag, build, mmap=True)


def _torch_oracle(a, indptr, indices, H, dev, threads, mmap=False):
    """The oracle's float64 torch.sparse CPU loop over the device A_hat of a whole-graph build,
    as a float64 numpy array; a workload's is shared through tests/ref_cache.py (the same tag as
    tests/test_gpu_configs.py's products_ref fixture)."""
    import ppnp_amd
    import ref_cache
    from oracle import ppnp_oracle as O

    def build():
        G = ppnp_amd.Graph.from_csr(indptr, indices, None, a.n, device=dev)
        rp, col, val, _ = G.csr()
        A = torch.sparse_csr_tensor(rp.cpu().long(), col.cpu().long(), val.cpu().double(),
                                    size=(a.n, a.n))
        G.close()
        del rp, col, val
        torch.set_num_threads(max(1, min(threads, len(os.sched_getaffinity(0)))))
        return O.appnp_propagate_torch_cpu(A, H.cpu().double(), a.K, a.alpha).numpy()

    if not a.workload:
        return build()
    return ref_cache.reference(f"{a.workload}-h{a.h_seed}-K{a.K}-a{a.alpha}", build, mmap=mmap)


def _send_blocks(ref, mine, rank, world):
    """Rank 0 holds the whole Z_K (ref) and sends every other rank its (rows, columns) block,
    point to point over gloo.  Returns (this rank's block, max |Z_K| over the whole matrix)."""
    blocks = [None] * world
    dist.all_gather_object(blocks, mine)
    if rank == 0:
        for r in range(1, world):
            lo, hi, f_lo, f_hi = blocks[r]
            dist.send(ref[lo:hi, f_lo:f_hi].contiguous(), dst=r)
        block = ref[mine[0]:mine[1], mine[2]:mine[3]].clone()
        m = torch.tensor([ref.abs().max().item()], dtype=torch.float64)
    else:
        block = torch.empty((mine[1] - mine[0], mine[3] - mine[2]), dtype=torch.float64)
        dist.recv(block, src=0)
        m = torch.zeros(1, dtype=torch.float64)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)  # the tolerance scales with the whole Z_K
    return block, m.item()


if __name__ == "__main__":
    main()
