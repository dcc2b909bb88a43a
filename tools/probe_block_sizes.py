"""First-block source rows of the C2 training batch at K negatives (the GNNREC_TRAIN_FOLD=auto
threshold's input): python tools/probe_block_sizes.py [K ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench_minibatch import BUYS, c2_graph  # noqa: E402
from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = c2_graph(64, dev)
    for K in [int(k) for k in sys.argv[1:]] or [10, 2500]:
        el = EdgeDataLoader(g, {BUYS: torch.arange(50_000_000)}, MultiLayerNeighborSampler([10, 10]),
                            exclude="reverse_types", reverse_etypes={"buys": "bought-by",
                                                                      "bought-by": "buys"},
                            negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                            shuffle=True)
        it = iter(el)
        for _ in range(3):
            _, _, _, blocks = next(it)
            print({"K": K, "block0_src_rows": {nt: blocks[0].number_of_src_nodes(nt) for nt in blocks[0].ntypes},
                   "block0_dst_rows": {nt: blocks[0].number_of_dst_nodes(nt) for nt in blocks[0].ntypes}},
                  flush=True)


if __name__ == "__main__":
    main()
