"""In-memory stand-in for the parts of DGL 0.5.2 that reference src/model.py touches.

TEST INFRASTRUCTURE (golden-vector generation only).  DGL is the reference's
pinned dependency (requirements.txt:2: dgl==0.5.2) and is not installed here,
so `tools`-side generation imports the reference's model.py with this module
registered as `dgl`, `dgl.function`, `dgl.nn`, `dgl.nn.pytorch`.  What it
restates from DGL 0.5.2 (unpinned by any reference test — see DESIGN.md):

  * builtin message/reduce functions fn.copy_src / fn.u_mul_e / fn.u_dot_v and
    fn.mean / fn.max: zero-in-degree destinations receive 0, mean divides the
    sum by the in-degree;
  * user-defined reduce functions (ConvLayer._lstm_reducer): degree bucketing —
    destinations with the same in-degree D are reduced together on a mailbox
    [n, D, ...] whose messages are in edge-id order; zero-in-degree
    destinations are not reduced and receive 0 (the zero frame initialiser);
  * HeteroGraphConv(mods, aggregate): per canonical etype, skip relations with
    no edges or whose src/dst type has no input; stack the outputs of the
    active relations per dst type and reduce with sum / mean / max
    (DGL nn/pytorch/hetero.py); modules kept in an nn.ModuleDict keyed by the
    relation name, so state_dict keys are layers.{i}.mods.{rel}.*;
  * graph.local_scope(), nodes[nt].data, srcdata/dstdata/edata, all_edges,
    apply_edges; multi-etype edata[...] returns {canonical_etype: tensor}.

Only full (non-block) heterographs are modelled: the golden vectors are the
reference run on one "batch" containing every node, which is what the build's
layer-wise full-graph pass computes.
"""
from __future__ import annotations

import contextlib
import sys
import types
from typing import Dict, Tuple

import torch
import torch.nn as nn


# ----------------------------------------------------------- builtins -------
class _Msg:
    def __init__(self, kind, a, b, out):
        self.kind, self.a, self.b, self.out = kind, a, b, out


class _Red:
    def __init__(self, kind, msg, out):
        self.kind, self.msg, self.out = kind, msg, out


def copy_src(src, out):
    return _Msg("copy_u", src, None, out)


def u_mul_e(lhs, rhs, out):
    return _Msg("u_mul_e", lhs, rhs, out)


def u_dot_v(lhs, rhs, out):
    return _Msg("u_dot_v", lhs, rhs, out)


def mean(msg, out):
    return _Red("mean", msg, out)


def max_(msg, out):
    return _Red("max", msg, out)


def sum_(msg, out):
    return _Red("sum", msg, out)


# ------------------------------------------------------------- graphs -------
class _DataView(dict):
    pass


class RelGraph:
    """Single-relation view: what ConvLayer.forward receives from HeteroGraphConv."""

    def __init__(self, parent: "HeteroGraph", cetype):
        self.parent = parent
        self.cetype = cetype
        self.canonical_etypes = [cetype]
        self.srcdata = {}
        self.dstdata = {}
        self.edata = dict(parent._edata[cetype])

    def number_of_edges(self):
        return self.parent.num_edges(self.cetype)

    def update_all(self, msg: _Msg, red: _Red):
        s, _, d = self.cetype
        src, dst = self.parent._edges[self.cetype]
        h = self.srcdata[msg.a]
        m = h[src]
        if msg.kind == "u_mul_e":
            m = m * self.edata[msg.b]
        elif msg.kind != "copy_u":
            raise NotImplementedError(msg.kind)
        n_dst = self.parent.num_nodes(d)
        out = torch.zeros((n_dst,) + tuple(m.shape[1:]), dtype=m.dtype)
        if callable(red) and not isinstance(red, _Red):
            deg = torch.bincount(dst, minlength=n_dst)
            order = torch.argsort(dst, stable=True)  # per destination: edge-id order
            start = torch.zeros(n_dst + 1, dtype=torch.int64)
            torch.cumsum(deg, 0, out=start[1:])
            key = None
            for D in sorted(set(deg.tolist()) - {0}):
                nodes = torch.nonzero(deg == D).flatten()
                eids = order[start[nodes].view(-1, 1) + torch.arange(D).view(1, -1)]
                mailbox = types.SimpleNamespace(mailbox={"m": m[eids]})
                res = red(mailbox)
                key = next(iter(res))
                out = out.to(res[key].dtype)
                out[nodes] = res[key]
            if key is not None:
                self.dstdata[key] = out
            else:
                self.dstdata["neigh"] = out
            return
        if red.kind in ("sum", "mean"):
            out.index_add_(0, dst, m)
            if red.kind == "mean":
                deg = torch.bincount(dst, minlength=n_dst).clamp(min=1).to(m.dtype)
                out = out / deg.view(-1, *([1] * (m.dim() - 1)))
        elif red.kind == "max":
            out = torch.full_like(out, -float("inf"))
            out = out.scatter_reduce(0, dst.view(-1, *([1] * (m.dim() - 1))).expand_as(m), m,
                                     reduce="amax", include_self=True)
            deg = torch.bincount(dst, minlength=n_dst)
            out[deg == 0] = 0
        else:
            raise NotImplementedError(red.kind)
        self.dstdata[red.out] = out


class _NodeSpace:
    def __init__(self, g):
        self.g = g

    def __getitem__(self, nt):
        return types.SimpleNamespace(data=self.g._ndata[nt])


class _EdataMulti:
    def __init__(self, g):
        self.g = g

    def __getitem__(self, key):
        res = {ce: d[key] for ce, d in self.g._edata.items() if key in d}
        if len(self.g.canonical_etypes) == 1:
            return next(iter(res.values()))
        return res


class HeteroGraph:
    """COO heterograph: edges {canonical_etype: (src int64, dst int64)}."""

    def __init__(self, edges: Dict[Tuple[str, str, str], Tuple[torch.Tensor, torch.Tensor]],
                 num_nodes: Dict[str, int]):
        self._edges = {ce: (torch.as_tensor(s, dtype=torch.int64),
                            torch.as_tensor(d, dtype=torch.int64)) for ce, (s, d) in edges.items()}
        self._num_nodes = dict(num_nodes)
        self.canonical_etypes = list(edges.keys())
        self.ntypes = sorted(num_nodes.keys())
        self._ndata = {nt: {} for nt in self.ntypes}
        self._edata = {ce: {} for ce in self.canonical_etypes}
        self.nodes = _NodeSpace(self)
        self.is_block = False

    def num_nodes(self, nt):
        return self._num_nodes[nt]

    def num_edges(self, ce):
        return int(self._edges[ce][0].numel())

    def all_edges(self, etype):
        return self._edges[etype]

    def __getitem__(self, cetype):
        return RelGraph(self, cetype)

    @property
    def edata(self):
        return _EdataMulti(self)

    @contextlib.contextmanager
    def local_scope(self):
        saved_n = {nt: dict(d) for nt, d in self._ndata.items()}
        saved_e = {ce: dict(d) for ce, d in self._edata.items()}
        try:
            yield
        finally:
            self._ndata = saved_n
            self._edata = saved_e

    def apply_edges(self, func: _Msg, etype):
        assert func.kind == "u_dot_v"
        s, _, d = etype
        src, dst = self._edges[etype]
        hs = self._ndata[s][func.a]
        hd = self._ndata[d][func.b]
        self._edata[etype][func.out] = (hs[src] * hd[dst]).sum(-1, keepdim=True)


# ------------------------------------------------------ HeteroGraphConv -----
class HeteroGraphConv(nn.Module):
    def __init__(self, mods, aggregate="sum"):
        super().__init__()
        self.mods = nn.ModuleDict(mods)
        self.aggregate = aggregate

    def forward(self, g, inputs):
        if isinstance(inputs, tuple):
            src_inputs, dst_inputs = inputs
        else:
            src_inputs = dst_inputs = inputs
        outputs = {nt: [] for nt in g.ntypes}
        for stype, etype, dtype in g.canonical_etypes:
            rel_graph = g[(stype, etype, dtype)]
            if rel_graph.number_of_edges() == 0:
                continue
            if stype not in src_inputs or dtype not in dst_inputs:
                continue
            outputs[dtype].append(self.mods[etype](rel_graph,
                                                   (src_inputs[stype], dst_inputs[dtype])))
        rsts = {}
        for nt, alist in outputs.items():
            if not alist:
                continue
            stacked = torch.stack(alist, dim=0)
            if self.aggregate == "sum":
                rsts[nt] = stacked.sum(0)
            elif self.aggregate == "mean":
                rsts[nt] = stacked.mean(0)
            elif self.aggregate == "max":
                rsts[nt] = stacked.max(0)[0]
            else:
                raise KeyError(self.aggregate)
        return rsts


def install():
    """Register the shim as `dgl`, `dgl.function`, `dgl.nn`, `dgl.nn.pytorch`."""
    dgl = types.ModuleType("dgl")
    fnm = types.ModuleType("dgl.function")
    fnm.copy_src, fnm.u_mul_e, fnm.u_dot_v = copy_src, u_mul_e, u_dot_v
    fnm.mean, fnm.max, fnm.sum = mean, max_, sum_
    nnm = types.ModuleType("dgl.nn")
    nnpt = types.ModuleType("dgl.nn.pytorch")
    nnpt.HeteroGraphConv = HeteroGraphConv
    nnm.pytorch = nnpt
    dgl.function = fnm
    dgl.nn = nnm
    dgl.DGLHeteroGraph = HeteroGraph
    sys.modules.update({"dgl": dgl, "dgl.function": fnm, "dgl.nn": nnm, "dgl.nn.pytorch": nnpt})
    return dgl
