#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own code.

Runs only in the build container (it needs /root/reference); its outputs -- small .npz
files of inputs and expected outputs -- are committed and travel to the GPU box, the
reference does not.  Regenerate with:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Reference functions exercised (file:line under /root/reference):
  SparseGraph.standardize          ppnp/data/sparsegraph.py:191-222
  helpers.calc_A_hat               helpers.py:58-66
  helpers.compute_ppr              helpers.py:68-71
  model.PPNP.forward               model.py:61-67
The reference datasets are read with np.load(allow_pickle=False) and only their numeric
arrays are used (the object-array keys are never unpickled).
"""

import os
import sys

import numpy as np
import scipy.sparse as sp

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import torch  # noqa: E402

import helpers  # noqa: E402  (reference)
import model  # noqa: E402  (reference)
from ppnp.data.sparsegraph import SparseGraph  # noqa: E402  (reference)
from ppnp.preprocessing import gen_splits, normalize_attributes  # noqa: E402  (reference)


def load_raw(name):
    d = np.load(os.path.join(REF, "ppnp", "data", name + ".npz"), allow_pickle=False)
    adj = sp.csr_matrix(
        (d["adj_matrix.data"], d["adj_matrix.indices"], d["adj_matrix.indptr"]),
        shape=tuple(d["adj_matrix.shape"]),
    )
    attr = sp.csr_matrix(
        (d["attr_matrix.data"], d["attr_matrix.indices"], d["attr_matrix.indptr"]),
        shape=tuple(d["attr_matrix.shape"]),
    )
    return adj, attr, np.asarray(d["labels"]).astype(np.int64)


def csr_sorted(m):
    m = sp.csr_matrix(m)
    m.sort_indices()
    return m


def iterate(a_hat, H, K, alpha):
    """APPNP K-step iteration on the reference's own operator, fp64."""
    Z = H.astype(np.float64)
    H64 = H.astype(np.float64)
    for _ in range(K):
        Z = (1 - alpha) * (a_hat @ Z) + alpha * H64
    return Z


def dataset(name, with_attr):
    adj_raw, attr, labels = load_raw(name)
    g = SparseGraph(adj_matrix=adj_raw.copy(), attr_matrix=attr, labels=labels)
    g.standardize(select_lcc=True)
    adj = csr_sorted(g.adj_matrix)
    n = adj.shape[0]
    C = int(g.labels.max()) + 1
    out = {
        "adj_raw_indptr": adj_raw.indptr.astype(np.int32),
        "adj_raw_indices": adj_raw.indices.astype(np.int32),
        "adj_raw_data": adj_raw.data.astype(np.float32),
        "adj_raw_n": np.int64(adj_raw.shape[0]),
        "adj_indptr": adj.indptr.astype(np.int32),
        "adj_indices": adj.indices.astype(np.int32),
        "adj_data": adj.data.astype(np.float32),
        "n": np.int64(n),
        "n_classes": np.int64(C),
    }
    for mode in ("sym", "rw"):
        ah = csr_sorted(helpers.calc_A_hat(adj, mode))
        out[f"ahat_{mode}_indptr"] = ah.indptr.astype(np.int32)
        out[f"ahat_{mode}_indices"] = ah.indices.astype(np.int32)
        out[f"ahat_{mode}_data"] = ah.data.astype(np.float64)
    gen = torch.Generator().manual_seed(0)
    H = torch.randn(n, C, generator=gen).numpy().astype(np.float32)
    out["H"] = H
    a_sym = helpers.calc_A_hat(adj, "sym")
    a_rw = helpers.calc_A_hat(adj, "rw")
    out["Z_sym_K10_a0.1"] = iterate(a_sym, H, 10, 0.1)
    out["Z_sym_K20_a0.2"] = iterate(a_sym, H, 20, 0.2)
    out["Z_rw_K10_a0.1"] = iterate(a_rw, H, 10, 0.1)
    ppr = helpers.compute_ppr(adj, alpha=0.1)
    out["pprH_a0.1"] = ppr @ H.astype(np.float64)
    ppr_rw = helpers.compute_ppr(adj, alpha=0.1, mode="rw")
    out["pprH_rw_a0.1"] = ppr_rw @ H.astype(np.float64)

    # model.PPNP forward (eval mode, fixed weights, small dense X)
    torch.manual_seed(1)
    F_in = 32
    X = torch.rand(n, F_in, generator=torch.Generator().manual_seed(2))
    net = model.PPNP(n_features=F_in, n_classes=C, ppr=torch.FloatTensor(ppr))
    net.eval()
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(3))[:140]
    with torch.no_grad():
        logits = net(X, idx)
        sub = net.ppr[idx[:16]][:, :]
        logits_ppr_mode = net(X, idx=None, ppr=sub)
    out["ppnp_X"] = X.numpy()
    out["ppnp_W1"] = net.encoder[1].weight.detach().numpy()  # (F_in, hidden)
    out["ppnp_W2"] = net.encoder[4].weight.detach().numpy()  # (C, hidden)
    out["ppnp_idx"] = idx.numpy().astype(np.int64)
    out["ppnp_logits"] = logits.numpy()
    out["ppnp_logits_ppr_mode"] = logits_ppr_mode.numpy()

    # preprocessing.py:9-64 -- splits for two seeds (main.py:84-98 call pattern), L1 norm
    for tag, sd in (("a", 2413340114), ("b", 123456789)):
        args = {"ntrain_per_class": 20, "nstopping": 500, "nknown": 1500, "seed": sd}
        tr, st, va = gen_splits(g.labels, args, test=False)
        _, _, te = gen_splits(g.labels, args, test=True)
        out[f"split_{tag}_seed"] = np.int64(sd)
        out[f"split_{tag}_train"] = np.asarray(tr, dtype=np.int64)
        out[f"split_{tag}_stop"] = np.asarray(st, dtype=np.int64)
        out[f"split_{tag}_valid"] = np.asarray(va, dtype=np.int64)
        out[f"split_{tag}_test"] = np.asarray(te, dtype=np.int64)
    xn = normalize_attributes(g.attr_matrix)
    out["attr_l1_rowsum"] = np.asarray(abs(xn).sum(axis=1)).ravel().astype(np.float64)
    if with_attr:
        at = csr_sorted(g.attr_matrix)
        out["attr_indptr"] = at.indptr.astype(np.int32)
        out["attr_indices"] = at.indices.astype(np.int32)
        out["attr_data"] = at.data.astype(np.float32)
        out["attr_shape"] = np.asarray(at.shape, dtype=np.int64)
        out["labels"] = np.asarray(g.labels, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, n, adj.nnz, {k: v.shape for k, v in out.items() if hasattr(v, "shape")})


def kats():
    """Closed-form known-answer graphs."""
    out = {}
    graphs = {
        "complete5": sp.csr_matrix(np.ones((5, 5)) - np.eye(5), dtype=np.float32),
        "complete2": sp.csr_matrix(np.ones((2, 2)) - np.eye(2), dtype=np.float32),
        "path3": sp.csr_matrix(
            np.array([[0, 1, 0], [1, 0, 1], [0, 1, 0]], dtype=np.float32)
        ),
        "isolated3": sp.csr_matrix(
            np.array([[0, 1, 0], [1, 0, 0], [0, 0, 0]], dtype=np.float32)
        ),
        "weighted4": sp.csr_matrix(
            np.array(
                [[0, 2, 0, 0.5], [2, 0, 1, 0], [0, 1, 0, 3], [0.5, 0, 3, 0]],
                dtype=np.float32,
            )
        ),
        "selfloop3": sp.csr_matrix(
            np.array([[1, 1, 0], [1, 0, 1], [0, 1, 2]], dtype=np.float32)
        ),
    }
    for gname, a in graphs.items():
        a = csr_sorted(a)
        out[f"{gname}_indptr"] = a.indptr.astype(np.int32)
        out[f"{gname}_indices"] = a.indices.astype(np.int32)
        out[f"{gname}_data"] = a.data.astype(np.float32)
        for mode in ("sym", "rw"):
            ah = csr_sorted(helpers.calc_A_hat(a, mode))
            out[f"{gname}_ahat_{mode}_dense"] = ah.toarray()
            out[f"{gname}_ppr_{mode}_a0.1"] = helpers.compute_ppr(a, 0.1, mode=mode)
    np.savez_compressed(os.path.join(OUT, "kat.npz"), **out)
    print("kat", sorted(out))


if __name__ == "__main__":
    kats()
    dataset("cora_ml", with_attr=True)
    dataset("citeseer", with_attr=True)
