"""Readers for the golden fixtures written by tests/golden/make_golden.py."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return json.load(f)["cases"]


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def cetype(key):
    return tuple(key.split("__"))


def graph_parts(arrs, prefix="g"):
    """-> (num_nodes {nt: n}, edges {ce: (src, dst)}, occurrence {ce: int64})"""
    num_nodes, src, dst, occ = {}, {}, {}, {}
    for k, v in arrs.items():
        parts = k.split("/")
        if parts[0] != prefix:
            continue
        if parts[1] == "num_nodes":
            num_nodes[parts[2]] = int(v)
        elif parts[1] == "src":
            src[cetype(parts[2])] = v
        elif parts[1] == "dst":
            dst[cetype(parts[2])] = v
        elif parts[1] == "occurrence":
            occ[cetype(parts[2])] = v
    order = [k for k in arrs if k.startswith(prefix + "/src/")]
    edges = {cetype(k.split("/")[2]): (src[cetype(k.split("/")[2])], dst[cetype(k.split("/")[2])])
             for k in order}
    return num_nodes, edges, occ


def state_dict(arrs):
    return {k[2:]: v for k, v in arrs.items() if k.startswith("w/")}


def by_etype(arrs, prefix):
    return {cetype(k[len(prefix) + 1:]): v for k, v in arrs.items() if k.startswith(prefix + "/")}
