"""bench.py's launch contract (CPU): `--gpus N` is honoured whether or not a launcher started
the process, and a line can never claim a GPU count other than the ranks that ran."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


@pytest.mark.parametrize("argv,env,want", [
    ([], {}, (1, None)),                                  # plain run: one GPU
    (["--gpus", "1"], {}, (1, None)),
    (["--gpus", "8"], {}, (None, 8)),                     # no launcher: spawn 8 ranks
    (["--gpus", "4"], {"WORLD_SIZE": "4"}, (4, None)),    # torchrun with a matching count
    ([], {"WORLD_SIZE": "2"}, (2, None)),                 # launcher without --gpus
])
def test_resolve_world(argv, env, want):
    bench = _bench()
    assert bench.resolve_world(bench.parse(argv), env) == want


@pytest.mark.parametrize("argv,env", [(["--gpus", "2"], {"WORLD_SIZE": "1"}),
                                      (["--gpus", "8"], {"WORLD_SIZE": "4"}),
                                      (["--gpus", "0"], {})])
def test_resolve_world_refuses_a_mismatch(argv, env):
    bench = _bench()
    with pytest.raises(SystemExit):
        bench.resolve_world(bench.parse(argv), env)


def test_mismatched_launch_exits_nonzero_before_any_gpu_work():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line


def test_spawn_refuses_more_ranks_than_gpus_for_rccl():
    """This container has no GPU: an RCCL launch of 2 ranks must fail before starting them."""
    bench = _bench()
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs here")
    old = os.environ.pop("GNNREC_DIST_BACKEND", None)
    try:
        assert bench.spawn_ranks(2, ["--gpus", "2"]) == 2
    finally:
        if old is not None:
            os.environ["GNNREC_DIST_BACKEND"] = old
