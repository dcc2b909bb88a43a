"""Row f3: graph file round trip (CPU; the format is device-independent)."""
import numpy as np
import torch

from gnnrec.graph import HeteroGraph
from gnnrec.io import load_graphs, read_graph, save_graphs


def _graph():
    rng = np.random.default_rng(0)
    u = torch.from_numpy(rng.integers(0, 50, 300))
    i = torch.from_numpy(rng.integers(0, 20, 300))
    g = HeteroGraph({("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u),
                     ("sport", "includes", "sport"): (torch.zeros(0, dtype=torch.int64),
                                                      torch.zeros(0, dtype=torch.int64))},
                    {"user": 50, "item": 20, "sport": 3})
    g.nodes["user"].data["features"] = torch.randn(50, 5)
    g.nodes["item"].data["features"] = torch.randn(20, 6)
    occ = torch.from_numpy(rng.integers(1, 9, 300))
    g.edges["buys"].data["occurrence"] = occ
    g.edges["bought-by"].data["occurrence"] = occ
    return g


def test_round_trip(tmp_path):
    g = _graph()
    f = str(tmp_path / "g.bin")
    save_graphs(f, [g, g], {"label": torch.tensor([1, 2])})
    gl, labels = load_graphs(f)
    assert len(gl) == 2 and torch.equal(labels["label"], torch.tensor([1, 2]))
    h = gl[1]
    assert h.canonical_etypes == g.canonical_etypes and h.ntypes == g.ntypes
    for nt in g.ntypes:
        assert h.num_nodes(nt) == g.num_nodes(nt)
        for k, v in g._ndata[nt].items():
            assert torch.equal(h.nodes[nt].data[k], v)
    for ce in g.canonical_etypes:
        for a, b in zip(h.all_edges(etype=ce), g.all_edges(etype=ce)):
            assert torch.equal(a, b)
        for a, b in zip(h._csr[ce], g.in_csr(ce)):  # cached CSR loaded, not rebuilt
            assert torch.equal(a, b) and a.dtype == b.dtype
        for k, v in g._edata[ce].items():
            assert torch.equal(h.edges[ce].data[k], v)
    assert read_graph(f).num_edges() == g.num_edges()


def test_create_graph_infers_node_counts_like_dgl_heterograph():
    """Reference src/builder.py:377-383: create_graph(graph_schema) = dgl.heterograph(
    graph_schema), node counts inferred per type as max id + 1 over every relation the
    type appears in (0 for a type with no edges); given counts are kept and checked."""
    import pytest

    from gnnrec import create_graph
    u = np.array([0, 5, 2]), np.array([1, 1, 7])
    schema = {("user", "buys", "item"): u, ("item", "bought-by", "user"): (u[1], u[0]),
              ("user", "clicks", "item"): (np.array([9]), np.array([0])),
              ("sport", "includes", "sport"): (np.zeros(0, np.int64), np.zeros(0, np.int64))}
    g = create_graph(schema)
    assert (g.num_nodes("user"), g.num_nodes("item"), g.num_nodes("sport")) == (10, 8, 0)
    assert g.canonical_etypes == list(schema)
    assert g.num_edges("buys") == 3 and g.num_edges(("user", "clicks", "item")) == 1
    g2 = create_graph(schema, num_nodes_dict={"user": 12})
    assert g2.num_nodes("user") == 12 and g2.num_nodes("item") == 8
    with pytest.raises(ValueError):
        create_graph(schema, num_nodes_dict={"user": 5})
    with pytest.raises(ValueError):
        create_graph({("user", "buys"): u})
