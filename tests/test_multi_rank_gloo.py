"""Multi-rank batch path on CPU (gloo, world_size 2 and 3): sharding + the size all-gather
that bench.py runs over RCCL, for weak slices and for the strong-scaling
split of one batch (shard_range: unequal and empty slices).  Per-chunk frames come from the CPU
oracle (test infrastructure), so this checks the host logic only: every rank's slice,
the global offsets, and that the frames laid out at those offsets decode back to the
whole batch with libzstd."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import zh_testlib as T
from cuda_zstd import shard

N_PER_RANK = 6
CHUNK = 4096
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, n_total=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.weak_range(rank, N_PER_RANK) if n_total is None else shard.shard_range(rank, world, n_total)
    data = T.gen(T.KINDS["mix"], hi - lo, 0x5EED0003, CHUNK, first=lo)
    frames = [T.oracle_frame(data[i * CHUNK:(i + 1) * CHUNK].tobytes()) for i in range(hi - lo)]
    sizes = torch.tensor([len(f) for f in frames], dtype=torch.int64)
    all_sizes, offs = shard.gather_offsets(sizes, world, n_total=n_total)
    total = int(all_sizes.sum())
    # each rank writes its frames at the global offsets of a shared output image
    img = np.zeros(total, np.uint8)
    for i, f in enumerate(frames):
        o = int(offs[lo + i])
        img[o:o + len(f)] = np.frombuffer(f, np.uint8)
    t = torch.from_numpy(img)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)  # disjoint ranges: the sum is the union
    if rank == 0:
        np.save(os.path.join(outdir, "img.npy"), t.numpy())
        np.save(os.path.join(outdir, "sizes.npy"), all_sizes.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges():
    assert shard.shard_range(0, 8, 16384) == (0, 2048)
    assert shard.shard_range(7, 8, 16384) == (14336, 16384)
    assert shard.shard_range(3, 4, 10) == (9, 10)
    assert sum(b - a for a, b in (shard.shard_range(r, 3, 10) for r in range(3))) == 10
    assert shard.weak_range(2, 16384) == (32768, 49152)
    assert [shard.shard_range(r, 4, 5) for r in range(4)] == [(0, 2), (2, 4), (4, 5), (5, 5)]  # an empty slice


def _check_image(tmp_path, n):
    img = np.load(tmp_path / "img.npy")
    sizes = np.load(tmp_path / "sizes.npy")
    assert len(sizes) == n and img.size == sizes.sum()
    whole = T.gen(T.KINDS["mix"], n, 0x5EED0003, CHUNK, first=0)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    for k in range(n):
        frame = img[offs[k]:offs[k] + sizes[k]].tobytes()
        assert T.zstd_decompress(frame, CHUNK) == whole[k * CHUNK:(k + 1) * CHUNK].tobytes()


def test_two_rank_gather_offsets(tmp_path, libzstd):
    mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    _check_image(tmp_path, WORLD * N_PER_RANK)


@pytest.mark.parametrize("world,n_total", [(3, 10), (4, 5)])
def test_strong_split_gather_offsets(tmp_path, libzstd, world, n_total):
    """One batch over `world` ranks by shard_range (C4): slices of 4/4/2 and 2/2/1/0 chunks;
    the padded all-gather must still give every chunk its global offset."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_total), nprocs=world, join=True)
    _check_image(tmp_path, n_total)
