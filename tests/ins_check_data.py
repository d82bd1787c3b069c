"""Shared workload of the ZH_INS_CHECK guard test (tests/test_gpu_k1.py): 256 chunks of the C3
mix plus 16 chunks of every corpus kind, 64 KiB each, through Manager.compress_batch."""
import numpy as np

import zh_testlib as T

LEVELS = (1, 2, 3)


def chunks():
    out = [T.gen(T.DG_MIX, 256, 0x5EED0003, 65536)]
    for k, kind in enumerate(sorted(T.KINDS)):
        out.append(T.gen(T.KINDS[kind], 16, 0x1C00 + k, 65536))
    buf = np.concatenate(out)
    return [buf[i * 65536:(i + 1) * 65536] for i in range(len(buf) // 65536)]


def compress(level):
    import torch

    import cuda_zstd

    dev = [torch.from_numpy(c).cuda() for c in chunks()]
    outs = cuda_zstd.Manager(level).compress_batch(dev)
    torch.cuda.synchronize()
    return [o.cpu().numpy().tobytes() for o in outs]
