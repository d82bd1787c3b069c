"""C4's sharded batch path on the GPU: ranks (gloo process group, all on
cuda:0 -- the box has one GPU) each compress their shard_range slice of ONE batch through
the stream-ordered C entry nvcomp_zstd_batched_compress_async_v5, exchange the per-chunk
sizes with ShardPlan.gather_offsets (the all-gather bench.py runs over RCCL) and write their
frames at the global offsets of one image.  The image must hold every chunk's frame, equal
to the oracle's, and decode chunk by chunk with libzstd to the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import zh_testlib as T

pytestmark = pytest.mark.gpu
CHUNK = 65536


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, n_total):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cuda_zstd
    from cuda_zstd import shard

    plan = shard.ShardPlan(world, n_total)
    lo, hi = plan.range(rank)
    n = hi - lo
    host = T.gen(T.DG_MIX, n, 0x5EED0003, CHUNK, first=lo) if n else np.zeros(0, np.uint8)
    dev = torch.device("cuda", 0)
    sizes = torch.zeros(n, dtype=torch.int64)
    frames = []
    if n:
        bc = cuda_zstd.BatchedCompressor(3, CHUNK)
        slot = (bc.max_out(CHUNK) + 255) // 256 * 256
        d_in = torch.from_numpy(host).to(dev)
        d_out = torch.empty(n * slot, dtype=torch.uint8, device=dev)
        ar = torch.arange(n, dtype=torch.int64, device=dev)
        out_sizes = torch.zeros(n, dtype=torch.int64, device=dev)
        status = torch.full((n,), -1, dtype=torch.int32, device=dev)
        temp = torch.empty(bc.temp_size(n, CHUNK), dtype=torch.uint8, device=dev)
        bc.compress_async(d_in.data_ptr() + ar * CHUNK, torch.full((n,), CHUNK, dtype=torch.int64, device=dev), CHUNK,
                          d_out.data_ptr() + ar * slot, out_sizes, status, temp)
        torch.cuda.synchronize(dev)
        assert int((status != 0).sum()) == 0
        sizes = out_sizes.cpu()
        ob = d_out.cpu().numpy()
        frames = [ob[i * slot:i * slot + int(sizes[i])] for i in range(n)]
    all_sizes, offs = plan.gather_offsets(sizes)
    img = np.zeros(int(all_sizes.sum()), np.uint8)
    for i, f in enumerate(frames):
        o = int(offs[lo + i])
        img[o:o + len(f)] = f
    t = torch.from_numpy(img)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)  # disjoint ranges: the sum is the union
    if rank == 0:
        np.save(os.path.join(outdir, "img.npy"), t.numpy())
        np.save(os.path.join(outdir, "sizes.npy"), all_sizes.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 24), (3, 10), (8, 67)])  # (8: the driver's scaling node, ragged 9 x 7 + 4)
def test_sharded_batch_on_gpu(tmp_path, libzstd, world, n_total):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_total), nprocs=world, join=True)
    img = np.load(tmp_path / "img.npy")
    sizes = np.load(tmp_path / "sizes.npy")
    assert len(sizes) == n_total and img.size == sizes.sum()
    whole = T.gen(T.DG_MIX, n_total, 0x5EED0003, CHUNK, first=0)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    for k in range(n_total):
        frame = img[offs[k]:offs[k] + sizes[k]].tobytes()
        chunk = whole[k * CHUNK:(k + 1) * CHUNK]
        assert frame == T.oracle_frame(chunk), k
        assert T.zstd_decompress(frame, CHUNK) == chunk.tobytes(), k
