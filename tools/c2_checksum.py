"""C2 with a content checksum: one 64 MiB frame (iid 16-symbol bytes) through the
stream-ordered batch entry with enable_checksum, timed with HIP events (median of 5), next to
the same frame without the checksum.  The XXH64 of one frame is a serial chain of 2M rounds
per accumulator (zh_checksum_kernel).  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cuda_zstd  # noqa: E402
import zh_testlib as T  # noqa: E402

N = 64 << 20


def run(checksum):
    data = np.random.default_rng(5).integers(0, 16, N, dtype=np.uint8)
    dev = torch.from_numpy(data).cuda()
    bc = cuda_zstd.BatchedCompressor(3, N, checksum=checksum)
    cap = bc.max_out(N)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    args = (torch.tensor([dev.data_ptr()], dtype=torch.int64, device="cuda"), torch.tensor([N], dtype=torch.int64, device="cuda"), N,
            torch.tensor([out.data_ptr()], dtype=torch.int64, device="cuda"), torch.zeros(1, dtype=torch.int64, device="cuda"),
            torch.zeros(1, dtype=torch.int32, device="cuda"))
    temp = torch.empty(bc.temp_size(1, N), dtype=torch.uint8, device="cuda")
    bc.compress_async(*args, temp)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        bc.compress_async(*args, temp)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    size = int(args[4].item())
    frame = out[:size].cpu().numpy().tobytes()
    ok = T.zstd_decompress(frame, N) == data.tobytes()
    return sorted(ts)[2], size, ok


if __name__ == "__main__":
    t0, s0, ok0 = run(False)
    t1, s1, ok1 = run(True)
    print(json.dumps({"workload": "C2 64 MiB iid 16-symbol buffer, one frame, stream-ordered batch entry",
                      "ms_no_checksum": round(t0, 3), "ms_checksum": round(t1, 3), "GBps_no_checksum": round(N / t0 / 1e6, 2),
                      "GBps_checksum": round(N / t1 / 1e6, 2), "frame_bytes": [s0, s1], "libzstd_roundtrip": ok0 and ok1}))
