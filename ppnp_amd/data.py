"""Graph ingest: the reference's npz flat-dict format, standardized on the GPU.

Reference:
  SparseGraph.from_flat_dict   ppnp/data/sparsegraph.py:246-297  (keys "<name>.data/.indices/
                               .indptr/.shape", legacy "_" separator and "adj"/"attr" names)
  SparseGraph.standardize      ppnp/data/sparsegraph.py:191-222  (unweighted, undirected, no
                               self loops, largest connected component)
  create_subgraph              ppnp/data/sparsegraph.py:300-352  (attributes / labels follow
                               the kept nodes)

The npz is parsed on the host with ``np.load(allow_pickle=False)`` (numeric arrays only; the
reference's object-array keys such as node_names are skipped, nothing is unpickled); the
adjacency is copied to the GPU once and ``appnp_standardize`` does the rest there.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib


def _vp(t):
    return C.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else None


def standardize_device(indptr, indices, data, n, select_lcc=True, device="cuda"):
    """Device SparseGraph.standardize.  Returns (indptr int32, indices int32, node_map int64)
    as tensors on ``device``; node_map[i] is the input id of output node i."""
    device = torch.device(device)
    ip = torch.as_tensor(np.asarray(indptr) if not torch.is_tensor(indptr) else indptr)
    ix = torch.as_tensor(np.asarray(indices) if not torch.is_tensor(indices) else indices)
    ip = ip.to(device=device, dtype=torch.int32).contiguous()
    ix = ix.to(device=device, dtype=torch.int32).contiguous()
    dv = None
    if data is not None:
        d = torch.as_tensor(np.asarray(data) if not torch.is_tensor(data) else data)
        dv = d.to(device=device, dtype=torch.float32).contiguous()
    lib = _lib.load()
    h = C.c_void_p()
    stream = C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    with torch.cuda.device(device):
        rc = lib.appnp_standardize(_vp(ip), _vp(ix), _vp(dv), int(n), int(ix.numel()),
                                   1 if select_lcc else 0, stream, C.byref(h))
    _lib.check("appnp_standardize", rc)
    try:
        n_out, nnz, n_in = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check("appnp_csr_info",
                   lib.appnp_csr_info(h, C.byref(n_out), C.byref(nnz), C.byref(n_in)))
        o_ip = torch.empty(n_out.value + 1, dtype=torch.int32, device=device)
        o_ix = torch.empty(nnz.value, dtype=torch.int32, device=device)
        o_map = torch.empty(n_out.value, dtype=torch.int64, device=device)
        with torch.cuda.device(device):
            rc = lib.appnp_csr_copy(h, _vp(o_ip), _vp(o_ix), _vp(o_map), stream)
        _lib.check("appnp_csr_copy", rc)
        torch.cuda.current_stream(device).synchronize()
    finally:
        lib.appnp_csr_destroy(h)
    return o_ip, o_ix, o_map


def read_flat_dict(path):
    """Numeric arrays of a reference .npz, with sparse matrices reassembled exactly as
    SparseGraph.from_flat_dict does (sparsegraph.py:246-297)."""
    z = np.load(path, allow_pickle=False)
    raw = {}
    for k in z.files:
        try:
            raw[k] = z[k]
        except ValueError:  # object arrays need pickle: skipped, never unpickled
            continue
    out = {}
    used = set()
    for key in list(raw):
        if key.endswith(".data") or key.endswith("_data"):
            sep = key[-5]
            name = key[:-5]
            parts = [f"{name}{sep}{s}" for s in ("indices", "indptr", "shape")]
            if not all(p in raw for p in parts):
                continue
            mname = name + "_matrix" if name in ("adj", "attr") else name
            out[mname] = sp.csr_matrix((raw[key], raw[parts[0]], raw[parts[1]]),
                                       shape=tuple(raw[parts[2]]))
            used.update([key, *parts])
    for key, val in raw.items():
        if key not in used:
            out[key] = val
    return out


def load_npz(path, device="cuda", standardize=True, select_lcc=True):
    """Load a reference dataset (.npz) and standardize its graph on the GPU.

    Returns a dict: ``adj`` (host scipy CSR fp32 of the standardized graph), ``indptr`` /
    ``indices`` (the same CSR on ``device``), ``attr`` (host CSR) and ``labels`` restricted to
    the kept nodes, and ``node_map`` (kept input node ids)."""
    d = read_flat_dict(path)
    adj = sp.csr_matrix(d["adj_matrix"], dtype=np.float32)
    adj.sort_indices()
    n = adj.shape[0]
    if standardize:
        ip, ix, nm = standardize_device(adj.indptr, adj.indices, adj.data, n,
                                        select_lcc=select_lcc, device=device)
    else:
        ip = torch.from_numpy(adj.indptr.astype(np.int32)).to(device)
        ix = torch.from_numpy(adj.indices.astype(np.int32)).to(device)
        nm = torch.arange(n, device=device)
    keep = nm.cpu().numpy()
    m = len(keep)
    std = sp.csr_matrix((np.ones(ix.numel(), dtype=np.float32), ix.cpu().numpy(),
                         ip.cpu().numpy()), shape=(m, m))
    res = {"adj": std, "indptr": ip, "indices": ix, "node_map": nm}
    if "attr_matrix" in d:
        res["attr"] = sp.csr_matrix(d["attr_matrix"], dtype=np.float32)[keep]
    if "labels" in d:
        res["labels"] = np.asarray(d["labels"])[keep]
    return res
