#!/usr/bin/env python
"""Per-epoch time of the main.py training loop (main.py:114-159: train forward + backward +
Adam step, two eval forwards, three host syncs) for APPNP on the HIP path against the dense
PPNP, on the reference's datasets.

    python tools/epoch_time.py [--dataset cora_ml] [--epochs 300]
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def epochs(model, X, y, idx_train, idx_stop, idx_valid, n):
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    for rep in range(2):  # the first pass warms up
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            model.train()
            logits = model(X, idx_train)
            loss = F.cross_entropy(logits, y[idx_train]) + 2.5e-3 * model.get_norm()
            opt.zero_grad()
            loss.backward()
            opt.step()
            float((logits.argmax(-1) == y[idx_train]).float().mean())
            model.eval()
            with torch.no_grad():
                stop = model(X, idx_stop)
                float(F.cross_entropy(stop, y[idx_stop]))
                float((model(X, idx_valid).argmax(-1) == y[idx_valid]).float().mean())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / n
    return dt * 1e3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--dataset", default="cora_ml")
    p.add_argument("--epochs", type=int, default=300)
    a = p.parse_args()
    from ppnp_amd import train as T
    from ppnp_amd.model import APPNP, PPNP

    adj, attr, labels = T.load_dataset(a.dataset)
    dev = torch.device("cuda")
    X = torch.FloatTensor(np.asarray(T.normalize_attributes(attr).todense())).to(dev)
    y = torch.LongTensor(labels).to(dev)
    n = X.shape[0]
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(0)).to(dev)
    idx = (perm[:140], perm[140:640], perm[640:1500])
    C = int(labels.max()) + 1
    res = {"dataset": a.dataset, "epochs": a.epochs}
    res["ppnp_ms_per_epoch"] = epochs(PPNP(X.shape[1], C, T._dense_ppr(adj, 0.1)).to(dev), X, y,
                                      *idx, a.epochs)
    res["appnp_K10_ms_per_epoch"] = epochs(APPNP(X.shape[1], C, adj).to(dev), X, y, *idx,
                                           a.epochs)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
