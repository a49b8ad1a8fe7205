"""Latency-regime probe: does one launch over A_hat^2 cost about what one launch over A_hat
costs?  If so, Z_{k+2} = (1-a)^2 A_hat^2 Z_k + H' halves the dependent launches of a K-step
propagation (no dropout).  Both operators go through the raw-CSR SpMM (appnp_spmm), K
dependent launches captured in one CUDA graph and replayed; per-launch time reported.
Usage: python tools/square_probe.py [workload ...]"""
import sys
import os

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ppnp_amd import synth  # noqa: E402
from ppnp_amd.sparse import spmm  # noqa: E402


def a_hat(n, indptr, indices):
    a = sp.csr_matrix((np.ones(len(indices)), indices, indptr), shape=(n, n)) + sp.eye(n)
    d = np.asarray(a.sum(1)).ravel()
    di = sp.diags(1.0 / np.sqrt(d))
    return (di @ a @ di).tocsr()


def timed(csr, F, reps=50, launches=10):
    dev = "cuda"
    ip = torch.from_numpy(csr.indptr.astype(np.int32)).to(dev)
    ix = torch.from_numpy(csr.indices.astype(np.int32)).to(dev)
    v = torch.from_numpy(csr.data.astype(np.float32)).to(dev)
    n = csr.shape[0]
    bufs = [torch.randn(n, F, device=dev), torch.empty(n, F, device=dev)]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for k in range(launches):  # warm
            spmm(ip, ix, v, n, n, bufs[k % 2], out=bufs[(k + 1) % 2])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for k in range(launches):
            spmm(ip, ix, v, n, n, bufs[k % 2], out=bufs[(k + 1) % 2])
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * launches)


for w in sys.argv[1:] or ["pubmed-synth", "ms-academic-synth"]:
    n, m, F = synth.CONFIGS[w][:3]
    ip, ix = synth.graph_for(w, device="cpu")
    A = a_hat(n, ip.numpy(), ix.numpy())
    A2 = (A @ A).tocsr()
    A2.sort_indices()
    t1, t2 = timed(A, F), timed(A2, F)
    rl2 = np.diff(A2.indptr)
    print(f"{w}: n={n} F={F} nnz(A_hat)={A.nnz} nnz(A_hat^2)={A2.nnz} (max row {rl2.max()}): "
          f"A_hat {t1:.2f} us/launch, A_hat^2 {t2:.2f} us/launch, "
          f"two steps {2 * t1:.2f} -> {t2:.2f} us", flush=True)
