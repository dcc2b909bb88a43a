"""Graph file format — replaces dgl.save_graphs / dgl.load_graphs
as used by reference main_train.py:398 and src/utils_inference.py:6-12.

The DGL .bin format cannot be read offline (DGL is not installable), so the
build defines its own single-file container, designed to be memory-mapped
and streamed straight into HBM:

    b"GNNRECG1" | u64 header_len | JSON header | pad to 64 B | blobs (64-B aligned)

The header lists, per graph, node counts, every canonical edge type with its
COO (src, dst in eid order), its cached dst-major CSR (indptr int64, indices
int32, eids int64 — so loading skips the device sort), node data and edge
data; and a table of blobs {dtype, shape, offset}.  Arrays are little-endian.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .graph import HeteroGraph

MAGIC = b"GNNRECG1"
ALIGN = 64


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().numpy()


class _Writer:
    def __init__(self):
        self.blobs: List[np.ndarray] = []

    def add(self, t) -> int:
        self.blobs.append(np.ascontiguousarray(_np(t) if torch.is_tensor(t) else t))
        return len(self.blobs) - 1


def save_graphs(filename: str, g_list, labels: Optional[Dict[str, torch.Tensor]] = None):
    """Write HeteroGraphs (and optional graph labels) to `filename`."""
    if isinstance(g_list, HeteroGraph):
        g_list = [g_list]
    w = _Writer()
    graphs = []
    for g in g_list:
        rels = []
        for ce in g.canonical_etypes:
            s, d = g.all_edges(etype=ce)
            indptr, indices, eids = g.in_csr(ce)
            rels.append({"etype": list(ce), "src": w.add(s), "dst": w.add(d),
                         "csr": {"indptr": w.add(indptr), "indices": w.add(indices),
                                 "eids": w.add(eids)},
                         "edata": {k: w.add(v) for k, v in g._edata[ce].items()}})
        graphs.append({"num_nodes": {nt: g.num_nodes(nt) for nt in g.ntypes},
                       "relations": rels,
                       "ndata": {nt: {k: w.add(v) for k, v in g._ndata[nt].items()}
                                 for nt in g.ntypes}})
    lab = {k: w.add(v) for k, v in (labels or {}).items()}
    table, off = [], 0
    for a in w.blobs:
        off = (off + ALIGN - 1) // ALIGN * ALIGN
        table.append({"dtype": a.dtype.str, "shape": list(a.shape), "offset": off,
                      "nbytes": int(a.nbytes)})
        off += a.nbytes
    header = json.dumps({"version": 1, "graphs": graphs, "labels": lab, "blobs": table}).encode()
    base = (len(MAGIC) + 8 + len(header) + ALIGN - 1) // ALIGN * ALIGN
    with open(filename, "wb") as f:
        f.write(MAGIC)
        f.write(np.uint64(len(header)).tobytes())
        f.write(header)
        for a, t in zip(w.blobs, table):
            f.seek(base + t["offset"])
            f.write(a.tobytes())
        f.truncate(base + off)


def load_graphs(filename: str, idx_list: Optional[List[int]] = None,
                device=None) -> Tuple[List[HeteroGraph], Dict[str, torch.Tensor]]:
    """Read graphs written by save_graphs -> (graph list, labels), DGL's return shape."""
    with open(filename, "rb") as f:
        if f.read(len(MAGIC)) != MAGIC:
            raise ValueError(f"{filename}: not a gnnrec graph file")
        hlen = int(np.frombuffer(f.read(8), dtype=np.uint64)[0])
        header = json.loads(f.read(hlen).decode())
    base = (len(MAGIC) + 8 + hlen + ALIGN - 1) // ALIGN * ALIGN
    mm = np.memmap(filename, dtype=np.uint8, mode="c")
    table = header["blobs"]

    def blob(i) -> torch.Tensor:
        t = table[i]
        a = mm[base + t["offset"]: base + t["offset"] + t["nbytes"]].view(np.dtype(t["dtype"]))
        x = torch.from_numpy(a.reshape(t["shape"]))
        return x.to(device) if device is not None else x.clone()

    sel = range(len(header["graphs"])) if idx_list is None else idx_list
    out = []
    for gi in sel:
        gh = header["graphs"][gi]
        rels = {tuple(r["etype"]): (blob(r["src"]), blob(r["dst"])) for r in gh["relations"]}
        g = HeteroGraph(rels, gh["num_nodes"], device=device)
        for r in gh["relations"]:
            ce = tuple(r["etype"])
            c = r["csr"]
            g._csr[ce] = (blob(c["indptr"]), blob(c["indices"]), blob(c["eids"]))
            for k, b in r["edata"].items():
                g._edata[ce][k] = blob(b)
        for nt, fields in gh["ndata"].items():
            for k, b in fields.items():
                g._ndata[nt][k] = blob(b)
        out.append(g)
    labels = {k: blob(b) for k, b in header["labels"].items()}
    return out, labels


def read_graph(graph_path: str, device=None) -> HeteroGraph:
    """reference src/utils_inference.py:6-12 (`read_graph`): first graph of the file."""
    graphs, _ = load_graphs(graph_path, [0], device=device)
    return graphs[0]


def file_size(filename: str) -> int:
    return os.path.getsize(filename)
