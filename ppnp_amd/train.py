"""main.py-equivalent training harness for APPNP on the HIP propagation path.

Reproduces the call pattern of /root/reference/main.py:63-175:

* seeds (helpers.py:13-17)
* L1 attribute normalisation (preprocessing.py:54-64)
* known/unknown + train/stopping/validation splits with a fresh uint32 seed per run
  (preprocessing.py:9-52, main.py:33-35, 84-98)
* Adam(lr 0.01) on cross-entropy + reg_lambda/2 * ||W1||^2 (main.py:109-127)
* three forwards per epoch (main.py:121, 138, 145)
* SimpleEarlyStopping with patience 100 (helpers.py:19-55)

The model is ``ppnp_amd.APPNP`` (the dense ``ppnp_amd.PPNP`` with ``--model ppnp``), so the
propagation of every forward and backward runs on the fused HIP kernels.  The splitting,
seeding and early stopping are host bookkeeping, restated so that the harness runs without
the reference; tests/test_train.py pins them to the reference's own outputs.

    python -m ppnp_amd.train --dataset cora_ml --n-runs 5      # data: tests/golden/*.npz
"""

from __future__ import annotations

import argparse
import copy
import json
import os
import random
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# -- helpers.py:13-17 ---------------------------------------------------------------------
def set_seeds(seed):
    random.seed(seed + 1)
    np.random.seed(seed + 2)
    torch.manual_seed(seed + 3)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed + 4)


def gen_seeds():
    """main.py:33-35."""
    max_uint32 = np.iinfo(np.uint32).max
    return np.random.randint(max_uint32 + 1, size=1, dtype=np.uint32)


# -- preprocessing.py:9-64 ----------------------------------------------------------------
def exclude_idx(idx, idx_exclude_list):
    idx_exclude = np.concatenate(idx_exclude_list)
    return np.asarray(idx)[~np.isin(idx, idx_exclude)]


def known_unknown_split(idx, nknown=1500, seed=4143496719):
    rnd_state = np.random.RandomState(seed)
    known_idx = rnd_state.choice(idx, nknown, replace=False)
    return known_idx, exclude_idx(idx, [known_idx])


def train_stopping_split(idx, labels, ntrain_per_class=20, nstopping=500, seed=2413340114):
    rnd_state = np.random.RandomState(seed)
    train_idx_split = []
    for i in range(max(labels) + 1):
        train_idx_split.append(rnd_state.choice(idx[labels == i], ntrain_per_class,
                                                replace=False))
    train_idx = np.concatenate(train_idx_split)
    stopping_idx = rnd_state.choice(exclude_idx(idx, [train_idx]), nstopping, replace=False)
    return train_idx, stopping_idx


def gen_splits(labels, idx_split_args, test=False):
    all_idx = np.arange(len(labels))
    known_idx, unknown_idx = known_unknown_split(all_idx, idx_split_args["nknown"])
    stopping_split_args = copy.copy(idx_split_args)
    del stopping_split_args["nknown"]
    train_idx, stopping_idx = train_stopping_split(known_idx, labels[known_idx],
                                                   **stopping_split_args)
    if test:
        val_idx = unknown_idx
    else:
        val_idx = exclude_idx(known_idx, [train_idx, stopping_idx])
    return train_idx, stopping_idx, val_idx


def normalize_attributes(attr_matrix):
    epsilon = 1e-12
    if sp.issparse(attr_matrix):
        attr_norms = np.asarray(abs(attr_matrix).sum(axis=1)).ravel()
        attr_invnorms = 1 / np.maximum(attr_norms, epsilon)
        return sp.csr_matrix(attr_matrix.multiply(attr_invnorms[:, np.newaxis]))
    attr_norms = np.linalg.norm(attr_matrix, ord=1, axis=1)
    attr_invnorms = 1 / np.maximum(attr_norms, epsilon)
    return attr_matrix * attr_invnorms[:, np.newaxis]


# -- helpers.py:19-55 ---------------------------------------------------------------------
class SimpleEarlyStopping:
    def __init__(self, model, patience=100, store_weights=False):
        self.model = model
        self.patience = patience
        self.max_patience = patience
        self.store_weights = store_weights
        self.record = (None,)  # reference quirk: `self.record = None,` (helpers.py:26)
        self.best_acc = -np.inf
        self.best_nloss = -np.inf
        self.best_epoch = -1
        self.best_epoch_score = (-np.inf, -np.inf)

    def should_stop(self, acc, loss, epoch, record=None):
        nloss = -1 * loss
        if (acc < self.best_acc) and (nloss < self.best_nloss):
            self.patience -= 1
            return self.patience == 0
        self.patience = self.max_patience
        self.best_acc = max(acc, self.best_acc)
        self.best_nloss = max(nloss, self.best_nloss)
        if (acc, nloss) > self.best_epoch_score:
            self.best_epoch = epoch
            self.best_epoch_score = (acc, nloss)
            if self.store_weights:
                self.best_state = {k: v.cpu() for k, v in self.model.state_dict().items()}
            if record:
                self.record = record
        return False


# -- data -----------------------------------------------------------------------------------
def load_dataset(name):
    """Standardized LCC adjacency, attributes and labels from tests/golden/<name>.npz (the
    reference's own SparseGraph.standardize output, see tests/golden/make_golden.py)."""
    path = os.path.join(ROOT, "tests", "golden", name + ".npz")
    d = np.load(path, allow_pickle=False)
    n = int(d["n"])
    adj = sp.csr_matrix((d["adj_data"], d["adj_indices"], d["adj_indptr"]), shape=(n, n))
    attr = sp.csr_matrix((d["attr_data"], d["attr_indices"], d["attr_indptr"]),
                         shape=tuple(d["attr_shape"]))
    return adj, attr, np.asarray(d["labels"])


# -- main.py:71-165 -------------------------------------------------------------------------
def run_once(adj, attr, labels, args, device):
    from .model import APPNP, PPNP

    idx_split_args = {"ntrain_per_class": args.ntrain_per_class, "nstopping": args.nstopping,
                      "nknown": args.nknown, "seed": gen_seeds()}
    X = normalize_attributes(attr)
    if args.sparse_x:  # keep X sparse on the GPU (main.py:91 densifies it)
        from .sparse import SparseFeatures

        X = SparseFeatures.from_scipy(X, device=device)
    else:
        X = torch.FloatTensor(np.asarray(X.todense())).to(device)
    y = torch.LongTensor(labels)
    idx_train, idx_stop, idx_valid = gen_splits(labels, idx_split_args, test=args.test)
    idx_train, idx_stop, idx_valid = map(torch.LongTensor, (idx_train, idx_stop, idx_valid))
    y_train, y_stop, y_valid = y[idx_train], y[idx_stop], y[idx_valid]
    idx_train, idx_stop, idx_valid = (t.to(device) for t in (idx_train, idx_stop, idx_valid))
    y_train, y_stop, y_valid = (t.to(device) for t in (y_train, y_stop, y_valid))

    torch.manual_seed(int(gen_seeds()[0]))
    n_classes = int(y.max()) + 1
    if args.model == "ppnp":
        ppr = torch.FloatTensor(_dense_ppr(adj, args.alpha))
        model = PPNP(n_features=X.shape[1], n_classes=n_classes, ppr=ppr).to(device)
    else:
        model = APPNP(n_features=X.shape[1], n_classes=n_classes, adj=adj, alpha=args.alpha,
                      K=args.K, edge_drop=args.edge_drop).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    early_stopping = SimpleEarlyStopping(model)
    t = time.time()
    for epoch in range(args.max_epochs):
        model.train()
        logits = model(X, idx_train)
        train_loss = F.cross_entropy(logits, y_train)
        train_loss = train_loss + args.reg_lambda / 2 * model.get_norm()
        opt.zero_grad()
        train_loss.backward()
        opt.step()
        train_acc = (logits.argmax(dim=-1) == y_train).float().mean()

        model.eval()
        with torch.no_grad():
            logits = model(X, idx_stop)
            stop_loss = F.cross_entropy(logits, y_stop)
            stop_loss = stop_loss + args.reg_lambda / 2 * model.get_norm()
            stop_acc = (logits.argmax(dim=-1) == y_stop).float().mean()
            valid_acc = (model(X, idx_valid).argmax(dim=-1) == y_valid).float().mean()
        record = {"epoch": int(epoch), "elapsed": float(time.time() - t),
                  "train_acc": float(train_acc), "stop_acc": float(stop_acc),
                  "valid_acc": float(valid_acc)}
        if args.verbose:
            print(json.dumps(record), file=sys.stderr)
        if early_stopping.should_stop(acc=float(stop_acc), loss=float(stop_loss), epoch=epoch,
                                      record=record):
            break
    return early_stopping.record


def _dense_ppr(adj, alpha):
    """Dense alpha (I - (1-alpha) A_hat)^-1 for --model ppnp (helpers.py:68-71), with A_hat
    from the device build (bit-identical to calc_A_hat in fp32)."""
    from .graph import Graph

    G = Graph.from_scipy(adj, device="cuda")
    rp, col, val, _ = G.csr()
    n = adj.shape[0]
    A = torch.sparse_csr_tensor(rp.long(), col.long(), val.double(), size=(n, n)).to_dense()
    inner = torch.eye(n, dtype=torch.float64, device=A.device) - (1 - alpha) * A
    return (alpha * torch.linalg.inv(inner)).float().cpu()


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--dataset", default="cora_ml")
    p.add_argument("--n-runs", type=int, default=5)
    p.add_argument("--seed", type=int, default=123)
    p.add_argument("--ntrain-per-class", type=int, default=20)
    p.add_argument("--nstopping", type=int, default=500)
    p.add_argument("--nknown", type=int, default=1500)
    p.add_argument("--max-epochs", type=int, default=10_000)
    p.add_argument("--reg-lambda", type=float, default=5e-3)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--K", type=int, default=10)
    p.add_argument("--edge-drop", type=float, default=0.0)
    p.add_argument("--model", default="appnp", choices=["appnp", "ppnp"])
    p.add_argument("--sparse-x", action="store_true",
                   help="keep the attribute matrix as a CSR on the GPU (sparse encoder input)")
    p.add_argument("--test", action="store_true")
    p.add_argument("--verbose", action="store_true")
    args = p.parse_args(argv)
    if "ms_academic" in args.dataset:  # main.py:56-59
        args.alpha = 0.2
        args.nknown = 5000
    return args


def main(argv=None):
    args = parse_args(argv)
    set_seeds(args.seed)
    device = torch.device("cuda")
    adj, attr, labels = load_dataset(args.dataset)
    records = []
    for _ in range(args.n_runs):
        rec = run_once(adj, attr, labels, args, device)
        print(rec, flush=True)
        records.append(rec)
    acc = np.array([r["valid_acc"] for r in records])
    summary = {"dataset": args.dataset, "model": args.model, "K": args.K, "runs": len(acc),
               "valid_acc_mean": float(acc.mean()), "valid_acc_std": float(acc.std(ddof=1))
               if len(acc) > 1 else 0.0,
               "epochs_mean": float(np.mean([r["epoch"] for r in records])),
               "elapsed_mean": float(np.mean([r["elapsed"] for r in records]))}
    print(json.dumps(summary), flush=True)
    return summary


if __name__ == "__main__":
    main()
