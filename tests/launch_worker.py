"""Rank body for tests/test_launch.py: started N times by cuda_zstd.launch.spawn_ranks (the
same torchrun child launch bench.py --gpus N uses), it reads its rank from the launcher's
environment, opens a gloo group, runs the C4 size all-gather (ShardPlan.gather_offsets) over
oracle frames of its shard_range slice, and writes what it saw to <outdir>/rank<r>.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import zh_testlib as T  # noqa: E402
from cuda_zstd import launch, shard  # noqa: E402

CHUNK = 4096


def main():
    outdir, n_total = sys.argv[1], int(sys.argv[2])
    rank, local, world = launch.rank_env()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = shard.ShardPlan(world, n_total)
    lo, hi = plan.range(rank)
    data = T.gen(T.KINDS["mix"], hi - lo, 0x5EED0003, CHUNK, first=lo)
    sizes = torch.tensor([len(T.oracle_frame(data[i * CHUNK:(i + 1) * CHUNK].tobytes())) for i in range(hi - lo)], dtype=torch.int64)
    all_sizes, offs = plan.gather_offsets(sizes)
    rec = {"rank": rank, "local_rank": local, "world": world, "range": [lo, hi],
           "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")],
           "ipc_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"),
           "all_sizes": all_sizes.tolist(), "offsets": offs.tolist()}
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
