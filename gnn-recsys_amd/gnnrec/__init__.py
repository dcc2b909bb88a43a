"""gnnrec — MI355X-native message-passing path for the hieucnm/GNN-RecSys user–item GNN.

The hot path (neighbour gather + mean/max aggregation, fused fp32-MFMA
projection, edge-score heads, block sampler, sharded full-graph embedding
pass) is hand-written HIP for gfx950 in ../csrc, exposed through the C ABI in
include/gnnrec.h and wrapped here as drop-in replacements for the reference's
src/model.py modules and DGL loaders.  See DESIGN.md.
"""
from . import _lib
from .graph import Block, HeteroGraph, PairGraph, RelGraph, NID, EID, create_graph  # noqa: F401
from .nn import (ConvLayer, ConvModel, CosinePrediction, HeteroGraphConv,  # noqa: F401
                 NodeEmbedding, PredictingLayer, PredictingModule, max_margin_loss)

__all__ = ["ConvLayer", "ConvModel", "CosinePrediction", "HeteroGraphConv", "NodeEmbedding",
           "PredictingLayer", "PredictingModule", "max_margin_loss", "HeteroGraph", "Block",
           "PairGraph", "RelGraph", "NID", "EID", "create_graph"]

__version__ = "0.1.0"


def library_path() -> str:
    return _lib.LIB_PATH
