"""GPU parity on BASELINE.json's configs at their full sizes.

Every check runs the HIP path through the C ABI on the synthetic graph the bench uses and
compares the WHOLE Z_K with an oracle computed on the CPU from the same A and H:

* config 2, pubmed-synth (19,717 x 3, K = 10, fp32) and config 4, arxiv-synth (169,343 x 128,
  K = 10, fp32): the float64 oracle (oracle/ppnp_oracle.py appnp_propagate, the K-step series
  of helpers.py:58-71), fp32 bar max|Z - Z_ref| <= 1e-5 max|Z_ref| + 1e-6;
* config 3, ms-academic-synth (18,333 x 15, K = 20, alpha = 0.2, bf16 storage): the bf16 bar
  <= 2e-2 max|Z_ref| with >= 98 % argmax agreement;
* config 5, products-synth (2,449,029 x 100, K = 10, fp32; 126 M nonzeros): the split-row path
  (96 gathered columns + the L2-blocked remainder pass) against a float64 torch.sparse CPU
  loop over the same A_hat, all ten iterations -- forward, the adjoint, and the power-law
  graph of the same size (hub rows);
* config 4 row-partitioned over 2 and 4 ranks sharing the one GPU (gloo exchange, with and
  without the overlapped local/remote split), each rank against the float64 oracle:
  tests/dist_worker.py launched by torch.distributed.run as fresh child processes;
* config 5 row-partitioned: products-synth over 2 ranks and over the north_star's 8
  ranks (all K = 10 iterations, rank 0's float64 oracle sent to every rank).
"""

import os
import re
import socket
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import ppnp_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _workload(name):
    from ppnp_amd import synth

    n, m, F, K, alpha, dtype = synth.CONFIGS[name]
    indptr, indices = synth.graph_for(name, device=DEV)
    H = synth.features(n, F, dtype=dtype, device=DEV)
    return n, F, K, alpha, dtype, indptr, indices, H


def _adj(indptr, indices, n):
    ix = indices.cpu().numpy()
    return sp.csr_matrix((np.ones(len(ix), dtype=np.float32), ix, indptr.cpu().numpy()),
                         shape=(n, n))


@pytest.mark.parametrize("name", ["pubmed-synth", "arxiv-synth"])
def test_config_fp32_full_size_matches_oracle(name):
    import ppnp_amd

    n, F, K, alpha, dtype, indptr, indices, H = _workload(name)
    G = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=DEV, features=F, dtype=dtype)
    Z = ppnp_amd.propagate_forward(G, H, K, alpha)
    ref = O.appnp_propagate(O.calc_a_hat(_adj(indptr, indices, n), "sym"),
                            H.double().cpu().numpy(), K, alpha)
    err = np.abs(Z.double().cpu().numpy() - ref).max()
    assert err <= 1e-5 * np.abs(ref).max() + 1e-6, err
    # the captured plan (hipGraph of the K launches) gives the same bits
    from ppnp_amd.ops import PropagatePlan

    plan = PropagatePlan(G, H, K, alpha)
    try:
        assert torch.equal(plan(), Z)
    finally:
        plan.close()


def test_config3_msacad_bf16_full_size():
    import ppnp_amd

    n, F, K, alpha, dtype, indptr, indices, H = _workload("ms-academic-synth")
    assert dtype == torch.bfloat16 and K == 20
    G = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=DEV)
    Z = ppnp_amd.propagate_forward(G, H, K, alpha)
    ref = O.appnp_propagate(O.calc_a_hat(_adj(indptr, indices, n), "sym"),
                            H.float().double().cpu().numpy(), K, alpha)
    got = Z.float().double().cpu().numpy()
    assert np.abs(got - ref).max() <= 2e-2 * np.abs(ref).max()
    assert (got.argmax(1) == ref.argmax(1)).mean() >= 0.98


def _products_case(name):
    """The full-size split-path case of workload ``name``: its graph (built with the bench's
    source-blocked copy), H, and A_hat as a float64 torch.sparse CSR on the CPU."""
    import ppnp_amd

    n, F, K, alpha, dtype, indptr, indices, H = _workload(name)
    G = ppnp_amd.Graph.from_csr(indptr, indices, None, n, device=DEV, features=F, dtype=dtype)
    assert G.split_point(F) == 96  # the bench's path: 3 gathered lines + remainder pass
    rp, col, val, _ = G.csr()
    a = torch.sparse_csr_tensor(rp.cpu().long(), col.cpu().long(), val.cpu().double(),
                                size=(n, n))
    adj = _adj(indptr, indices, n)
    del rp, col, val, indices
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    return G, H, K, alpha, a, adj


def _check_full(got, ref):
    err = float((got.double() - ref).abs().max())
    tol = 1e-5 * float(ref.abs().max()) + 1e-6
    assert err <= tol, (err, tol)


@pytest.fixture(scope="module")
def products():
    G, H, K, alpha, a, adj = _products_case("products-synth")
    yield G, H, K, alpha, a, adj
    G.close()


@pytest.fixture(scope="module")
def products_ref(products):
    """The float64 torch.sparse loop of the products fixture's A_hat on its H (seed 0), all K
    iterations: computed once per session (tests/ref_cache.py) and shared by the forward, the
    adjoint, the column slab and the row-partition workers."""
    import ref_cache

    _, H, K, alpha, a, _ = products
    ref = ref_cache.reference(_ref_tag("products-synth", 0, K, alpha),
                       lambda: O.appnp_propagate_torch_cpu(a, H.cpu().double(), K, alpha).numpy())
    return torch.from_numpy(ref)


def _ref_tag(workload, h_seed, K, alpha):
    return f"{workload}-h{h_seed}-K{K}-a{alpha}"


def test_products_a_hat_matches_calc_a_hat(products):
    """The device CSR build at products scale (126 M entries of A_hat) against the oracle's
    calc_a_hat (helpers.py:58-66) on the same A: row pointers and column indices bit-exact,
    values equal to float32 of the fp64 reference, every entry (pinned so far only
    up to arxiv size)."""
    G, _, _, _, _, adj = products
    ref = O.calc_a_hat(adj, "sym")
    rp, col, val, dinv = G.csr()
    assert np.array_equal(rp.cpu().numpy().astype(np.int64), ref.indptr.astype(np.int64))
    col = col.cpu().numpy()
    assert np.array_equal(col, ref.indices.astype(np.int32))
    del col
    assert np.array_equal(val.cpu().numpy(), ref.data.astype(np.float32))
    # the fp64 degree scale the build keeps: 1/sqrt(D), D the weighted row sum of A + I
    deg = np.diff(adj.indptr).astype(np.float64) + 1.0
    rel = np.abs(dinv.cpu().numpy() * np.sqrt(deg) - 1.0).max()
    assert rel <= 2.0 ** -51, rel


def test_products_k10_matches_oracle(products, products_ref):
    """Config 5 at full size, K = 10, on the split-row path -- every one of the 244.9 M values
    against the float64 torch.sparse CPU loop of the same A_hat (helpers.py:58-66)."""
    import ppnp_amd

    G, H, K, alpha, _, _ = products
    Z = ppnp_amd.propagate_forward(G, H, K, alpha).cpu()
    _check_full(Z, products_ref)


def test_products_k10_backward_matches_oracle(products, products_ref):
    """The adjoint at full size on the split path (appnp_propagate_bwd: main-column chain plus
    the remainder pass with its adjoint epilogue).  Without dropout APPNP_K is a polynomial in
    the symmetric A_hat, so J^T dZ = APPNP_K(dZ): the float64 forward loop is its oracle, and
    with dZ = H it is the forward's reference."""
    import ppnp_amd

    G, H, K, alpha, _, _ = products
    dH = ppnp_amd.propagate_backward(G, H, K, alpha).cpu()
    _check_full(dH, products_ref)


def test_products_k10_bf16_matches_oracle(products):
    """bf16 storage with fp32 accumulation at products scale (whole 200-B rows: the split path
    is fp32-only), against the oracle's torch.sparse loop on the bf16-rounded H: the bf16 bar of
    DESIGN.md 2.  The loop runs in float32 (its ~1e-7 relative error is five orders below the
    2e-2 bar, and it takes half the float64 loop's time)."""
    import ppnp_amd

    G, H, K, alpha, a, _ = products
    Hb = H.to(torch.bfloat16)
    assert G.split_point(int(H.shape[1]), torch.bfloat16) == 0
    Z = ppnp_amd.propagate_forward(G, Hb, K, alpha).float().cpu().double()
    ref = O.appnp_propagate_torch_cpu(a.to(torch.float32), Hb.float().cpu(), K, alpha).double()
    assert float((Z - ref).abs().max()) <= 2e-2 * float(ref.abs().max())
    assert float((Z.argmax(1) == ref.argmax(1)).double().mean()) >= 0.98


def test_products_col8_slab_matches_oracle(products, products_ref):
    """The 13-column slab of F = 100 on 8 column ranks (rank 0 of the exchange-free 8-GPU layout)
    on its W16 copy (4 row passes, piece-major LDS sums), every value of Z_K, K = 10, against the
    float64 torch.sparse loop of the same A_hat (columns are independent: the first 13 columns
    of the whole reference)."""
    import ppnp_amd

    _, H, K, alpha, _, adj = products
    G = ppnp_amd.Graph.from_scipy(adj, device=DEV, features=13)
    sb = G.source_block_layout()
    assert (sb["width"], sb["row_passes"]) == (16, 4), sb
    assert G.remainder_cols(13) == 13
    H13 = H[:, :13].contiguous()
    Z = ppnp_amd.propagate_forward(G, H13, K, alpha).cpu()
    _check_full(Z, products_ref[:, :13])
    G.close()


def test_products_powerlaw_matches_oracle():
    """The Chung-Lu power-law graph with products' node and edge counts (hub rows: the heavy /
    hub lists of the main SpMM and long runs in the remainder pass) at full size.  K = 4: every
    launch shape of K = 10 (first, middle and last iteration; hub rows in each) at 40 % of the
    oracle's time -- K = 10 itself is pinned on products-synth."""
    import ppnp_amd

    G, H, _, alpha, a, _ = _products_case("products-powerlaw")
    K = 4
    try:
        Z = ppnp_amd.propagate_forward(G, H, K, alpha).cpu()
    finally:
        G.close()
    _check_full(Z, O.appnp_propagate_torch_cpu(a, H.cpu().double(), K, alpha))


def _rank_results(stdout, tag):
    """{rank: 'OK' | 'FAIL'} from the workers' result lines ``[tag] rank r/P ... -> OK``, found
    anywhere in the merged stdout of the ranks (a line of one rank can land in the middle of
    another's when both write at once)."""
    mark = re.escape(f"[{tag}]")
    pat = mark + r" rank (\d+)/\d+ (?:(?!" + mark + r").)*?-> (OK|FAIL)"
    return {int(m.group(1)): m.group(2) for m in re.finditer(pat, stdout)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("ranks,extra", [(2, []), (2, ["--overlap"]), (4, []),
                                         (4, ["--overlap", "--pipeline", "off"]),
                                         (4, ["--overlap"]), (3, ["--overlap", "--p-drop", "0.2"])])
def test_arxiv_row_partition_matches_oracle(ranks, extra):
    """Config 4 row-partitioned: each rank's block of Z_K (real HIP kernels, gloo exchange
    staged through host memory since the ranks share one GPU) against the float64 oracle.
    From 3 ranks on, overlap pipelines the exchange (one broadcast per row shard, the product
    per group of arrived shards: appnp_step_shards) unless switched off."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT,
               OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dist_worker.py"),
           "--layout", "row", "--workload", "arxiv-synth", "--oracle", *extra]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_worker")
    assert res == {r: "OK" for r in range(ranks)}, proc.stdout[-4000:]
    piped = ranks >= 3 and "--overlap" in extra and "off" not in extra
    assert proc.stdout.count("pipeline=True") == (ranks if piped else 0), proc.stdout[-4000:]


@pytest.mark.parametrize("ranks", [2, 4])
def test_line_cut_column_slabs_match_oracle(ranks):
    """Column slabs cut at whole lines (dist.line_slab_cols; the autotune candidate that wins
    on 2 ranks): F = 100 as 64 | 36 (the 36-column slab on the split path: 32 + a 4-column
    remainder pass) and 32 | 32 | 32 | 4 (a narrow slab wholly in the pass), real HIP kernels on
    a 200k-node graph, each rank's block against the float64 oracle."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dist_worker.py"),
           "--layout", "col-lines", "--f", "100", "--graph-n", "200000", "--graph-m", "1000000",
           "--K", "4", "--oracle"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_worker")
    assert res == {r: "OK" for r in range(ranks)}, proc.stdout[-4000:]
    lines = [l for l in proc.stdout.splitlines() if l.startswith("[dist_worker]")]
    assert any("split_cols=4" in l for l in lines), lines  # the last slab took the pass


def test_stream_done_orders_consumer_after_side_stream():
    """The hand-off of the relayed exchange (dist.MultipathComm on 'nccl'): work queued on a
    side stream, then _StreamDone.wait() on the caller's stream -- a consumer queued after the
    wait sees the side stream's writes even when that work is still running at enqueue time."""
    from ppnp_amd.dist import _StreamDone

    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    x = torch.zeros(1 << 20, device=DEV)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        torch.cuda._sleep(20_000_000)  # keep the side stream busy past the enqueue below
        x.fill_(1.0)
        ev = torch.cuda.Event()
        ev.record(side)
    _StreamDone(ev).wait()
    y = x * 2.0  # on the main stream
    assert bool((y == 2.0).all())
    _StreamDone(None).wait()  # a synchronous exchange hands over no event


def test_bench_two_ranks_autotune_and_parity():
    """The driver's N = 2 bench shape, rehearsed on the one GPU: bench.py under
    torch.distributed.run (fresh child processes, gloo exchange since both ranks share the
    device) times every candidate layout, keeps the fastest and checks its Z_K against a
    single-GPU propagation of the whole graph (the line's parity field)."""
    import json

    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "arxiv-synth",
           "--steps", "2", "--warmup", "1"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = json.loads([l for l in proc.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["value"] > 0
    assert res["parity"]["ok"], res["parity"]
    tried = res["config"]["autotune_ms_per_step"]
    assert len(tried) >= 2 and all(v is not None for v in tried.values()), tried


def test_bench_eight_ranks_every_candidate():
    """The driver's N = 8 command on the one GPU (eight ranks time-sliced, gloo exchange) on
    arxiv-synth: every candidate of candidate_layouts(8) -- column, 2x4 and 4x2 with both
    exchanges, the row partition from Python and from the library's loop -- is measured, the
    printed line is one of them with parity, the CPU baseline and a coherent roofline
    (frac <= ceiling.frac <= 1)."""
    import json

    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "8", "--workload", "arxiv-synth",
           "--steps", "2", "--warmup", "1"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = json.loads([l for l in proc.stdout.splitlines() if l.startswith("{")][-1])
    tried = res["config"]["autotune_ms_per_step"]
    assert len(tried) == 7 and all(isinstance(v, float) for v in tried.values()), tried
    assert res["config"]["parallelism"] in tried and res["parity"]["ok"]
    assert res["cpu_baseline"]["value"] > 0 and res["parity_cpu"]["ok"]
    rl = res["roofline"]
    assert 0 < rl["frac"] <= rl["ceiling"]["frac"] <= 1.0


def test_bench_rccl_refused_still_prints_the_column_line():
    """The driver's N = 2 command exactly as the driver runs it (no backend override), on the
    one GPU: RCCL refuses two ranks on one device, so the data-path group cannot come up.  Since
    that group is created inside the exchange candidates (dist.ensure_data_group), they fail,
    are agreed failed over the gloo control plane and recorded as null, and the exchange-free
    column layout's line is printed with exit status 0 (before round 3's second session,
    init_process_group('nccl') at start-up ended the run with no line)."""
    import json

    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.pop("PPNP_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "arxiv-synth",
           "--steps", "2", "--warmup", "1", "--candidate-timeout", "120"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = json.loads([l for l in proc.stdout.splitlines() if l.startswith("{")][-1])
    tried = res["config"]["autotune_ms_per_step"]
    assert res["config"]["parallelism"] == "rows1xcols2" and res["parity"]["ok"]
    assert isinstance(tried["rows1xcols2"], float)
    assert all(v is None for k, v in tried.items() if k != "rows1xcols2"), tried


@pytest.mark.parametrize("ranks,extra", [
    (2, ["--overlap"]), (2, []), (3, ["--overlap", "--p-drop", "0.3"]),
    (3, ["--overlap", "--pipeline", "off"]),
    (2, ["--dtype", "bf16"]), (4, ["--workload", "arxiv-synth", "--overlap"])])
def test_native_row_engine_matches_single_gpu(ranks, extra):
    """The library's own row-partitioned loop (appnp_dist_create / appnp_dist_propagate: the
    C engine of SURVEY.md 8(b)) over 2-4 ranks sharing the GPU, with the exchange supplied
    as a host-staged gloo callback, against the single-GPU appnp_propagate.  From 3 ranks on,
    overlap pipelines the exchange through a broadcast callback (appnp_dist_set_broadcast)
    unless switched off."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dist_capi_worker.py"),
           *extra]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_capi")
    assert res == {r: "OK" for r in range(ranks)}, proc.stdout[-4000:]
    piped = ranks >= 3 and "--overlap" in extra and "off" not in extra
    assert proc.stdout.count("pipeline=True") == (ranks if piped else 0), proc.stdout[-4000:]


@pytest.mark.parametrize("backend", ["nccl", "gloo+nccl"])
def test_native_row_engine_rccl_callback_one_rank(backend):
    """appnp_allgather_rccl resolves the RCCL PyTorch loaded and runs on its communicator
    (one rank: RCCL refuses two ranks on one device), and the engine's one-rank run agrees
    with appnp_propagate.  'gloo+nccl' is bench.py's arrangement: gloo default group, RCCL
    data-path group brought up by ppnp_amd.dist.ensure_data_group; the engine, the library's
    callback and torch's in-place all-gather all run on that group's communicator."""
    env = dict(os.environ, PPNP_DIST_BACKEND=backend, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_capi_worker.py")]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    lines = [l for l in proc.stdout.splitlines() if l.startswith("[dist_capi]")]
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert len(lines) == 1 and "rccl_callback rc=0" in lines[0] and lines[0].endswith("OK"), lines


@pytest.mark.parametrize("f", [20, 50])
def test_pipelined_narrow_and_two_line_rows_match_oracle(f):
    """The pipelined shard steps on rows narrower than a wavefront's slab: F = 20 runs G-lane
    rows (the narrow kernel, each row's shard range between two offset arrays), F = 50 two-line
    rows on a wavefront each.  3 ranks sharing the GPU (gloo), overlap on (so pipelined),
    dropout; each rank's block against the float64 oracle."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_worker.py"), "--layout", "row", "--graph-n",
           "200000", "--graph-m", "1000000", "--f", str(f), "--K", "3", "--oracle", "--overlap",
           "--p-drop", "0.2"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert _rank_results(proc.stdout, "dist_worker") == {r: "OK" for r in range(3)}, \
        proc.stdout[-4000:]
    assert proc.stdout.count("pipeline=True") == 3, proc.stdout[-4000:]


@pytest.mark.parametrize("ranks,extra", [(2, []), (2, ["--overlap"]),
                                         (3, ["--overlap", "--p-drop", "0.3"])])
def test_row_partition_split_rows_matches_oracle(ranks, extra):
    """the north_star's row partition at F = 100 on a graph above 2^16 nodes
    takes the split layout on every rank (appnp_step_split: 3 gathered lines of the 96 main
    columns, the L2-blocked pass for the last 4, both parts exchanged), with and without the
    overlapped local/remote split and with dropout; each rank's block against the float64
    oracle."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dist_worker.py"),
           "--layout", "row", "--graph-n", "200000", "--graph-m", "1000000", "--f", "100",
           "--K", "4",
           "--oracle", "--expect-split", "4", *extra]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_worker")
    assert res == {r: "OK" for r in range(ranks)}, proc.stdout[-4000:]


@pytest.mark.parametrize("extra", [["--overlap"], []])
def test_products_row_partition_matches_oracle(extra):
    """the north_star's row partition on config 5's own workload -- products-synth
    (2,449,029 x 100, 126 M nonzeros) over 2 ranks sharing the GPU (gloo exchange), K = 10, every
    rank on the split rows of its held rows (3 gathered lines + the L2-blocked remainder pass,
    both parts exchanged), with and without the overlapped local/remote split.  Each rank's
    block of Z_K against the float64 torch.sparse loop over the device A_hat, which
    test_products_a_hat_matches_calc_a_hat pins to calc_a_hat (helpers.py:58-66) -- the
    session's products reference on H of seed 0 (tests/ref_cache.py)."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="8")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_worker.py"), "--layout", "row", "--workload",
           "products-synth", "--h-seed", "0", "--oracle-torch", "--expect-split", "4", *extra]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_worker")
    assert res == {0: "OK", 1: "OK"}, proc.stdout[-4000:]


def test_products_eight_rank_row_partition_k10_matches_oracle():
    """the north_star's own shape -- products-synth row-partitioned over 8
    ranks (time-sliced on the one GPU, gloo exchange staged through host memory), all K = 10
    iterations, overlapped local/remote split, every rank on the split rows of its held rows.
    Rank 0 runs the float64 torch.sparse oracle once and sends each rank its block; every block
    of Z_K must match it to 1e-5 of max |Z_K|."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_worker.py"), "--layout", "row", "--workload",
           "products-synth", "--h-seed", "0", "--oracle-torch", "--oracle-rank0",
           "--expect-split", "4", "--overlap"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_worker")
    assert res == {r: "OK" for r in range(8)}, proc.stdout[-4000:]
    lines = [l for l in proc.stdout.splitlines() if l.startswith("[dist_worker]")]
    assert all("rows=8, cols=1" in l and "overlap=True" in l for l in lines), lines


@pytest.mark.parametrize("f,exchange,split", [(72, "multipath", 4), (72, "group", 4),
                                              (73, "multipath", 0)])
def test_two_d_layout_split_rows_match_oracle(f, exchange, split):
    """a 2 x 2 layout on 4 ranks sharing the GPU, on the split layout of its held rows.
    F = 72 is 36 | 36 columns (32 + 4 on both column groups): the two parts of every iterate go
    through the relayed exchange (MultipathComm) or the column-group all-gather.  F = 73 is
    37 | 36 (a W8 copy beside a W4 copy): the ranks agree to keep whole rows instead of
    exchanging parts of different widths.  Each rank's block against the float64 oracle."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_worker.py"), "--layout", "2x2", "--f", str(f),
           "--graph-n", "200000", "--graph-m", "1000000", "--K", "3", "--oracle", "--overlap",
           "--exchange", exchange, "--expect-split", str(split)]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_worker")
    assert res == {r: "OK" for r in range(4)}, proc.stdout[-4000:]


def test_split_decision_is_collective():
    """The regrouped copy is best-effort: when it cannot be built on ONE rank (rank 1 here,
    APPNP_SB_TEST_OOM), every rank keeps whole rows -- both the Python row loop (an all-reduce at
    create) and the library's engine (one small exchange at the first propagation) -- instead
    of exchanging two parts on some ranks and one on others.  Results still match.  The fault
    is injected through the test library (libppnp_amd_test.so): the product one has no hooks."""
    from ppnp_amd import _lib

    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2",
               PPNP_AMD_LIB=_lib.TEST_LIB_PATH)
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
            "--master-addr=127.0.0.1"]
    py = base + [f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dist_worker.py"),
                 "--layout", "row", "--graph-n", "200000", "--graph-m", "1000000", "--f", "100",
                 "--K", "3", "--expect-split", "0", "--sb-oom-rank", "1", "--overlap"]
    proc = subprocess.run(py, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert _rank_results(proc.stdout, "dist_worker") == {0: "OK", 1: "OK"}, proc.stdout[-4000:]
    nat = base + [f"--master-port={_free_port()}",
                  os.path.join(ROOT, "tests", "dist_capi_worker.py"), "--workload", "arxiv-synth",
                  "--features", "100", "--split", "--sb-oom-rank", "1", "--overlap"]
    proc = subprocess.run(nat, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert _rank_results(proc.stdout, "dist_capi") == {0: "OK", 1: "OK"}, proc.stdout[-4000:]
    assert proc.stdout.count("split=False") == 2, proc.stdout[-4000:]


@pytest.mark.parametrize("extra", [[], ["--overlap"]])
def test_native_row_engine_misaligned_rank_stays_split(extra):
    """one rank passes H and Z 4 bytes off 16-B alignment.  It stages them through
    the workspace and takes the split layout like its peer (round 4 returned APPNP_EINVAL there
    while the peer waited in the split loop's exchange), and both match appnp_propagate."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_capi_worker.py"), "--workload", "arxiv-synth",
           "--features", "100", "--split", "--offset-rank", "1", *extra]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert _rank_results(proc.stdout, "dist_capi") == {0: "OK", 1: "OK"}, proc.stdout[-4000:]
    assert proc.stdout.count("split=True") == 2, proc.stdout[-4000:]


def test_native_row_engine_poisoned_after_failed_agreement():
    """a split agreement that fails after its exchange poisons the handle.  Both
    ranks inject the failure (APPNP_DIST_TEST_AGREE_FAIL), so neither waits on the other: the
    first call returns APPNP_EDEVICE after the agreement's one exchange, and the second returns
    the stored code without exchanging again.  (Test library: the product one has no hooks.)"""
    from ppnp_amd import _lib

    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2",
               PPNP_AMD_LIB=_lib.TEST_LIB_PATH)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_capi_worker.py"), "--workload", "arxiv-synth",
           "--features", "100", "--split", "--agree-fail"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert _rank_results(proc.stdout, "dist_capi") == {0: "OK", 1: "OK"}, proc.stdout[-4000:]


@pytest.mark.parametrize("ranks,extra", [(2, []), (2, ["--overlap", "--p-drop", "0.3"]),
                                         (3, ["--overlap"])])
def test_native_row_engine_split_rows(ranks, extra):
    """The library's own row loop (appnp_dist_propagate) on the split layout: arxiv-synth's
    graph at F = 100, every rank's held rows with their own source-blocked copy, both parts
    exchanged through the callback, against the single-GPU appnp_propagate."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dist_capi_worker.py"),
           "--workload", "arxiv-synth", "--features", "100", "--split", *extra]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_capi")
    assert res == {r: "OK" for r in range(ranks)}, proc.stdout[-4000:]
    assert proc.stdout.count("split=True") == ranks, proc.stdout[-4000:]


def test_native_row_engine_products_eight_ranks():
    """The library's own row loop (appnp_dist_propagate, the bench's rows8xcols1-overlap-native
    candidate) at the north_star's shape: products-synth over 8 ranks sharing the GPU, all
    K = 10 iterations, overlapped, every rank on the split layout of its held rows (3 gathered
    lines + the remainder pass, both parts exchanged through the callback), against the
    single-GPU appnp_propagate, which test_products_k10_matches_oracle pins to the float64
    oracle."""
    env = dict(os.environ, PPNP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_capi_worker.py"), "--workload", "products-synth",
           "--split", "--overlap"]
    proc = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    res = _rank_results(proc.stdout, "dist_capi")
    assert res == {r: "OK" for r in range(8)}, proc.stdout[-4000:]
    assert proc.stdout.count("split=True") == 8, proc.stdout[-4000:]
