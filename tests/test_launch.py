"""bench.py --gpus N's rank launcher (cuda_zstd/launch.py) on CPU:
the torchrun child launch, the rank environment every rank sees, the gloo size all-gather
through it, and bench.py's refusal of more GPUs than are visible."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import zh_testlib as T
from cuda_zstd import launch, shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNK = 4096


def test_rank_env_parsing():
    assert not launch.rank_env_present({})
    assert launch.rank_env({}) == (0, 0, 1)
    env = {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}
    assert launch.rank_env_present(env)
    assert launch.rank_env(env) == (3, 3, 4)


def test_launch_command_shape():
    cmd = launch.launch_command(8, "/x/bench.py", ["--gpus", "8", "--steps", "5"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "8", "--steps", "5"]
    with pytest.raises(ValueError):
        launch.launch_command(0, "x.py", [], 1)


@pytest.mark.parametrize("world,n_total", [(2, 9), (3, 7)])
def test_spawn_ranks_gloo_gather(tmp_path, libzstd, world, n_total):
    """spawn_ranks starts `world` torchrun children from a parent with no rank environment (as
    bench.py --gpus N does); each rank sees its RANK / LOCAL_RANK / WORLD_SIZE and the loopback
    rendezvous, and the padded size all-gather gives every rank the same global offsets."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = launch.spawn_ranks(world, os.path.join(ROOT, "tests", "launch_worker.py"), [str(tmp_path), str(n_total)], env=env, timeout=300)
    assert rc == 0
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    whole = T.gen(T.KINDS["mix"], n_total, 0x5EED0003, CHUNK, first=0)
    want = [len(T.oracle_frame(whole[k * CHUNK:(k + 1) * CHUNK].tobytes())) for k in range(n_total)]
    for r, rec in enumerate(recs):
        assert (rec["rank"], rec["local_rank"], rec["world"]) == (r, r, world)
        assert list(rec["range"]) == list(shard.shard_range(r, world, n_total))
        assert rec["master"][0] == "127.0.0.1" and rec["master"][1]
        assert rec["ipc_legacy"] == "0"
        assert rec["all_sizes"] == want
        assert rec["offsets"] == list(np.concatenate([[0], np.cumsum(want)[:-1]]).astype(int))


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus 64 (more than any node here holds) must stop in the parent with a clear
    message and a non-zero code, before any rank starts."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) are visible" in r.stderr
