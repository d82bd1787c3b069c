"""C5: 4,096 x 16 KiB JSON-like records (tools/datagen.c kind json, seed
0x5EED0005), level 9, with a 64 KiB dictionary trained on every fourth record by libzstd's
ZDICT_trainFromBuffer and by this library's COVER trainer.  GPU:
the stream-ordered batched entry with the dictionary set on the handle (device-resident
records, HIP events, median of 5 after a warm-up).  CPU reference: libzstd
ZSTD_compress_usingCDict(level 9) with the same dictionary, one thread.  libzstd decodes every
GPU frame with the dictionary.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
import cuda_zstd  # noqa: E402
import zh_testlib as T  # noqa: E402

REC, N, SEED, DICT = 16384, 4096, 0x5EED0005, 65536
LEVEL = int(os.environ.get("C5_LEVEL", "9"))
vp = ctypes.c_void_p


def libzstd_cdict(recs, d, level):
    z = T.zstd()
    z.ZSTD_createCCtx.restype = vp
    z.ZSTD_freeCCtx.argtypes = [vp]
    z.ZSTD_createCDict.restype = vp
    z.ZSTD_createCDict.argtypes = [vp, ctypes.c_size_t, ctypes.c_int]
    z.ZSTD_freeCDict.argtypes = [vp]
    z.ZSTD_compress_usingCDict.restype = ctypes.c_size_t
    z.ZSTD_compress_usingCDict.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp]
    db = np.frombuffer(d or b"\0", np.uint8).copy()
    cd = z.ZSTD_createCDict(db.ctypes.data, len(d) if d else 0, level)
    cctx = z.ZSTD_createCCtx()
    out = np.zeros(2 * REC, np.uint8)
    total, t0 = 0, time.perf_counter()
    for r in recs:
        s = z.ZSTD_compress_usingCDict(cctx, out.ctypes.data, out.size, r.ctypes.data, r.size, cd)
        assert not z.ZSTD_isError(s)
        total += s
    el = time.perf_counter() - t0
    z.ZSTD_freeCCtx(cctx)
    z.ZSTD_freeCDict(cd)
    return total, el


def gpu_run(dev, d):
    """Stream-ordered batched compression of the device-resident records
    (nvcomp_zstd_batched_compress_async_v5 with the dictionary set on the handle): median of 5
    timed with HIP events after a warm-up.  Returns the frames (host bytes) and seconds."""
    bc = cuda_zstd.BatchedCompressor(LEVEL, REC)
    if d:
        bc.set_dictionary(cuda_zstd.Dictionary.load(d))
    slot = (bc.max_out(REC) + 255) // 256 * 256
    out = torch.empty(N * slot, dtype=torch.uint8, device="cuda")
    ar = torch.arange(N, dtype=torch.int64, device="cuda")
    in_ptrs, out_ptrs = dev.data_ptr() + ar * REC, out.data_ptr() + ar * slot
    sizes = torch.full((N,), REC, dtype=torch.int64, device="cuda")
    osz = torch.zeros(N, dtype=torch.int64, device="cuda")
    st = torch.zeros(N, dtype=torch.int32, device="cuda")
    temp = torch.empty(bc.temp_size_for([REC] * N), dtype=torch.uint8, device="cuda")
    run = lambda: bc.compress_async(in_ptrs, sizes, REC, out_ptrs, osz, st, temp)
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    assert int((st != 0).sum()) == 0
    ob, sz = out.cpu().numpy(), osz.cpu().numpy()
    frames = [ob[i * slot:i * slot + int(sz[i])].tobytes() for i in range(N)]
    return frames, sorted(ts)[2]


def main():
    host = T.gen(T.DG_JSON, N, SEED, REC)
    recs = [host[i * REC:(i + 1) * REC] for i in range(N)]
    train = recs[::4]
    dicts = {"none": None, "zdict": T.zdict_train(train, DICT), "cover": cuda_zstd.Dictionary.train(train, DICT).content()}
    dev = torch.from_numpy(host).cuda()
    total = N * REC
    res = {"workload": "C5: 4096 x 16 KiB JSON-like records, level 9, 64 KiB dictionary (trained on every 4th record)",
           "dict_bytes": {k: len(v) for k, v in dicts.items() if v}, "ratio": {}, "gpu_GBps": {}, "libzstd_l9_1thread_MBps": {}}
    verified = True
    gpu_only = os.environ.get("C5_GPU_ONLY") == "1"  # (GPU legs only; no longer needed under the profiler)
    for name, d in dicts.items():
        frames, t = gpu_run(dev, d)
        res["ratio"][f"gpu_{name}"] = round(total / sum(len(f) for f in frames), 4)
        res["gpu_GBps"][name] = round(total / t / 1e9, 3)
        if gpu_only:
            continue
        for r, f in zip(recs, frames):
            if T.zstd_decompress(f, REC, dictionary=d) != r.tobytes():
                verified = False
                break
        lz, el = libzstd_cdict(recs, d, LEVEL)
        res["ratio"][f"libzstd_l9_{name}"] = round(total / lz, 4)
        res["libzstd_l9_1thread_MBps"][name] = round(total / el / 1e6, 1)
    res["libzstd_verified"] = verified and not gpu_only
    res["libzstd_images"] = T.libzstd_images()  # (under rocprofv3: the profiler's own libzstd too)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
