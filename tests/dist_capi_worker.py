#!/usr/bin/env python
"""End-to-end check of the library's own row-partitioned loop (appnp_dist_*, the C engine
behind ppnp_amd.dist.NativeRowAPPNP) on real HIP kernels.

    torchrun --nproc-per-node P --master-addr 127.0.0.1 tests/dist_capi_worker.py
        [--workload pubmed-synth] [--overlap] [--p-drop 0.3] [--dtype f32|bf16]

Every rank propagates its rows through appnp_dist_propagate and compares them with the
single-GPU appnp_propagate of the whole graph on its own device.  Backend gloo (the ranks may
share one GPU; the exchange callback stages the shards through host memory), or nccl with
PPNP_DIST_BACKEND=nccl: then the exchange is appnp_allgather_rccl on torch's own
communicator, and at world size 1 the worker also calls appnp_allgather_rccl directly once,
which checks that the library resolves the process's RCCL.  PPNP_DIST_BACKEND=gloo+nccl is
bench.py's arrangement: a gloo default group for the control plane and an RCCL group for the
data path (ppnp_amd.dist.ensure_data_group), whose communicator the engine then uses.  Exit
status 1 on mismatch.
"""

import argparse
import ctypes as C
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="pubmed-synth")
    p.add_argument("--features", type=int, default=None)
    p.add_argument("--overlap", action="store_true")
    p.add_argument("--p-drop", type=float, default=0.0)
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    p.add_argument("--split", action="store_true",
                   help="build the held rows' source-blocked copy for F (split rows) and fail "
                        "unless the engine takes the split layout")
    p.add_argument("--sb-oom-rank", type=int, default=-1,
                   help="this rank's copy fails to build (APPNP_SB_TEST_OOM): the engines must "
                        "agree on whole rows everywhere")
    p.add_argument("--offset-rank", type=int, default=-1,
                   help="this rank passes H and Z 4 bytes off 16-B alignment: it must stage them "
                        "and take the same (split) path as its peers (ADVICE r4)")
    p.add_argument("--agree-fail", action="store_true",
                   help="every rank's split agreement fails after its exchange "
                        "(APPNP_DIST_TEST_AGREE_FAIL): the first call returns the error, later "
                        "calls return it again without exchanging (the poisoned handle)")
    p.add_argument("--pipeline", default="auto", choices=["auto", "on", "off"],
                   help="the engine's pipelined exchange (appnp_dist_set_broadcast)")
    a = p.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)

    import ppnp_amd
    from ppnp_amd import _lib, synth
    from ppnp_amd import dist as pdist

    backend = os.environ.get("PPNP_DIST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    if backend == "gloo+nccl":
        pdist.ensure_data_group("nccl", dev)
        assert pdist.data_backend() == "nccl" and dist.get_backend() == "gloo"
    rank, world = dist.get_rank(), dist.get_world_size()
    n, m, F, K, alpha, _ = synth.CONFIGS[a.workload]
    F = a.features or F
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    indptr, indices = synth.graph_for(a.workload, device=dev)
    H = synth.features(n, F, dtype=dtype, device=dev, seed=1)

    if rank == a.sb_oom_rank or a.agree_fail:
        # fault injection needs libppnp_amd_test.so (the product library has no hooks): the
        # test sets PPNP_AMD_LIB; fail loudly rather than run without the injected fault
        if "testing=1" not in _lib.load().appnp_build_info().decode():
            raise SystemExit("fault injection needs PPNP_AMD_LIB=" + _lib.TEST_LIB_PATH)
    if rank == a.sb_oom_rank:
        os.environ["APPNP_SB_TEST_OOM"] = "1"
    runner = pdist.NativeRowAPPNP(indptr, indices, n, dev, overlap=a.overlap,
                                  features=F if a.split else None, dtype=dtype,
                                  pipeline={"auto": None, "on": True,
                                            "off": False}[a.pipeline])
    g = pdist._DistGraphInfo(C.c_void_p(_lib.load().appnp_dist_graph(runner._h)))
    before = (g.source_block_layout() or {}).get("launches", 0)
    if a.agree_fail:
        os.environ["APPNP_DIST_TEST_AGREE_FAIL"] = "1"
        codes = []
        for _ in range(2):
            try:
                runner.run(H[runner.lo:runner.hi].contiguous(), K, alpha, seed=5)
                codes.append(0)
            except _lib.AppnpError as e:
                codes.append(e.code)
            codes.append(getattr(runner, "gloo_calls", 0))
        # [first code, exchanges after it, second code, exchanges after it]: the agreement's one
        # exchange, then nothing
        ok = codes == [_lib.APPNP_EDEVICE, 1, _lib.APPNP_EDEVICE, 1]
        runner.close()
        print(f"[dist_capi] rank {rank}/{world} poisoned handle codes/exchanges {codes} -> "
              f"{'OK' if ok else 'FAIL'}", flush=True)
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(flag)
        dist.destroy_process_group()
        sys.exit(1 if flag.item() else 0)
    H_rows = H[runner.lo:runner.hi].contiguous()
    out = None
    if rank == a.offset_rank and H_rows.numel():
        # 4 bytes past a 16-B boundary: same leading dimension, misaligned base pointers
        hbuf = torch.empty(H_rows.numel() + 1, dtype=H_rows.dtype, device=dev)
        hbuf[1:].copy_(H_rows.reshape(-1))
        H_rows = hbuf[1:].view(H_rows.shape)
        out = torch.full((H_rows.numel() + 1,), float("nan"), dtype=H_rows.dtype,
                         device=dev)[1:].view(H_rows.shape)
        assert H_rows.data_ptr() % 16 and out.data_ptr() % 16
    Z = runner.run(H_rows, K, alpha, p_drop=a.p_drop, seed=5, out=out)
    torch.cuda.synchronize()
    # the split layout ran: one remainder pass per iteration (appnp_step_split)
    split_ran = (g.source_block_layout() or {}).get("launches", 0) - before == K
    if a.split and not split_ran:
        print(f"[dist_capi] rank {rank}: split layout expected but not taken", flush=True)
    G = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=dev)
    ref = ppnp_amd.propagate_forward(G, H, K, alpha, p_drop=a.p_drop, seed=5)
    block = ref[runner.lo:runner.hi]
    err = (Z.double() - block.double()).abs().max().item() if block.numel() else 0.0
    scale = ref.abs().max().item()
    tol = (1e-5 if dtype == torch.float32 else 1e-2) * scale + 1e-6
    want_split = a.split and a.sb_oom_rank < 0
    ok = err <= tol and (split_ran == want_split or runner.hi == runner.lo)
    extra = f" split={split_ran}"
    if backend in ("nccl", "gloo+nccl") and world == 1:
        # the library's RCCL callback on torch's communicator: a one-rank in-place all-gather
        lib = _lib.load()
        pg = pdist.data_group() or dist.distributed_c10d._get_default_group()
        comm = pg._get_backend(dev)._comm_ptr()
        buf = torch.arange(1024, dtype=torch.float32, device=dev)
        before = buf.clone()
        rc = lib.appnp_allgather_rccl(C.c_void_p(buf.data_ptr()), buf.numel() * 4, 0, 1,
                                      C.c_void_p(torch.cuda.current_stream(dev).cuda_stream),
                                      C.c_void_p(comm))
        torch.cuda.synchronize()
        ok = ok and rc == 0 and torch.equal(buf, before)
        extra += f" rccl_callback rc={rc}"
        # the pipelined exchange's RCCL broadcast: a one-rank in-place broadcast
        rc = lib.appnp_bcast_rccl(C.c_void_p(buf.data_ptr()), buf.numel() * 4, 0, 1,
                                  C.c_void_p(torch.cuda.current_stream(dev).cuda_stream),
                                  C.c_void_p(comm))
        torch.cuda.synchronize()
        ok = ok and rc == 0 and torch.equal(buf, before)
        extra += f" rccl_bcast rc={rc}"
        # torch's own in-place all-gather on the data-path group (the _TorchComm call)
        full = torch.arange(64, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(full, full[:64], group=pdist.data_group())
        torch.cuda.synchronize()
        ok = ok and torch.equal(full, torch.arange(64, dtype=torch.float32, device=dev))
        ok = ok and runner.exchange == "rccl"
    if runner.pipeline:
        # one broadcast per row shard and exchanged iterate (Z_0 .. Z_{K-1}), the product per
        # group of arrived shards
        bc = getattr(runner, "gloo_bcasts", None)
        # the engine's groups are dist.shard_groups' (the Python row loop's)
        ok = ok and (bc is None or bc == K * world)
        ok = ok and runner.groups == pdist.shard_groups(world, rank)
        extra += f" pipeline=True groups={runner.groups} bcasts={bc}"
    runner.close()
    print(f"[dist_capi] rank {rank}/{world} backend={dist.get_backend()} "
          f"exchange={runner.exchange} overlap={a.overlap} dtype={a.dtype} p_drop={a.p_drop} "
          f"rows [{runner.lo},{runner.hi}) max err {err:.3e} tol {tol:.3e}{extra} -> "
          f"{'OK' if ok else 'FAIL'}", flush=True)
    flag = torch.tensor([0 if ok else 1], dtype=torch.int64,
                        device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag)
    dist.destroy_process_group()
    sys.exit(1 if flag.item() else 0)


if __name__ == "__main__":
    main()
