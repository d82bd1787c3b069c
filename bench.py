"""Benchmark: BASELINE.json metric "compress GB/s + ratio, 1 GB @ level 3, 64 KB chunks;
libzstd round-trip OK" on MI355X.

Workload (config C3): every rank compresses 16384 x 64 KiB chunks
(1 GiB, Silesia-like synthetic mix, seed 0x5EED0003) that are already resident in
HBM, through the stream-ordered C-ABI entry nvcomp_zstd_batched_compress_async_v5
(K1 zh_lz_kernel -> K2 zh_entropy_kernel -> zh_fse_chain_kernel -> zh_seq_pack_kernel).
Multi-GPU (C4): one process per GPU,
chunks sharded by rank with no data-path collective (weak scaling); the only
collective is the RCCL all-gather of per-chunk compressed sizes that gives every
rank the global output offsets, inside the timed step.

Prints one JSON line (driver contract).  Roofline = the dominant kernel's
algorithmic bytes (input + compressed output) per launch / its
average HIP-event duration on the launch stream.  cpu_baseline = libzstd level 3
(the reference's own CPU route for <1 MiB items, src/cuda_zstd_manager.cu:1604-1668)
over a bounded sample of the same chunks on the host cores.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

CHUNK = 64 * 1024
CHUNKS_PER_GPU = 16384
HBM_PEAK_GBS = 8000.0
METRIC = "compress GB/s + ratio, 1 GB @ level 3, 64 KB chunks; libzstd round-trip OK"
SEEDS = {"mix": 0x5EED0003, "random": 0x5EED0004}


def gen_chunks(kind, n, first):
    import zh_testlib as T

    return T.gen(T.KINDS[kind], n, SEEDS[kind], CHUNK, first=first)


def cpu_baseline(data, threads, seconds=1.5):
    """libzstd ZSTD_compress(level 3) over the rank-0 chunks, one CCtx per call,
    `threads` host threads, bounded wall time."""
    import concurrent.futures as cf

    import zh_testlib as T

    z = T.zstd()
    if z is None:
        return None
    n = len(data) // CHUNK
    cap = 80000

    def work(lo, hi, out):
        tot = 0
        vp = ctypes.c_void_p
        for i in range(lo, hi):
            tot += z.ZSTD_compress(out.ctypes.data_as(vp), ctypes.c_size_t(cap), ctypes.c_void_p(data.ctypes.data + i * CHUNK), ctypes.c_size_t(CHUNK), 3)
        return tot

    bufs = [np.zeros(cap, np.uint8) for _ in range(threads)]
    per = 64  # chunks per task
    done_bytes, comp_bytes, t0 = 0, 0, time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        nxt = 0
        while time.perf_counter() - t0 < seconds:
            futs = []
            for t in range(threads):
                lo = nxt % n
                hi = min(lo + per, n)
                futs.append(ex.submit(work, lo, hi, bufs[t]))
                done_bytes += (hi - lo) * CHUNK
                nxt = hi
            comp_bytes += sum(f.result() for f in futs)
    el = time.perf_counter() - t0
    return {"value": round(done_bytes / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "reference",
            "sample": f"libzstd {z.ZSTD_versionNumber()} ZSTD_compress level 3 (the reference's CPU route) on {done_bytes >> 20} MiB "
                      f"of the same 64 KiB chunks, {threads} threads, {el:.2f} s wall; ratio {done_bytes / max(comp_bytes, 1):.3f}"}


def libzstd_roundtrip(frames, sizes, slot, host):
    """Every rank-0 frame through stock libzstd (ZSTD_decompress), 16 host threads;
    True iff all decode to their chunk.  None without libzstd."""
    import concurrent.futures as cf

    import zh_testlib as T

    z = T.zstd()
    if z is None:
        return None
    n = len(sizes)

    def work(lo, hi):
        dst = np.zeros(CHUNK, np.uint8)
        vp = ctypes.c_void_p
        for i in range(lo, hi):
            r = z.ZSTD_decompress(dst.ctypes.data_as(vp), ctypes.c_size_t(CHUNK), ctypes.c_void_p(frames.ctypes.data + i * slot), ctypes.c_size_t(int(sizes[i])))
            if r != CHUNK or not np.array_equal(dst, host[i * CHUNK:(i + 1) * CHUNK]):
                return False
        return True

    step = (n + 15) // 16
    with cf.ThreadPoolExecutor(16) as ex:
        return all(ex.map(lambda k: work(k, min(n, k + step)), range(0, n, step)))


def cpu_decompress_baseline(frames, sizes, slot, threads, seconds=1.5):
    """libzstd ZSTD_decompress (the reference's CPU decode route) over the rank-0 frames,
    `threads` host threads, bounded wall time."""
    import concurrent.futures as cf

    import zh_testlib as T

    z = T.zstd()
    if z is None:
        return None
    n = len(sizes)

    def work(lo, hi, dst):
        vp = ctypes.c_void_p
        tot = 0
        for i in range(lo, hi):
            tot += z.ZSTD_decompress(dst.ctypes.data_as(vp), ctypes.c_size_t(CHUNK), ctypes.c_void_p(frames.ctypes.data + i * slot),
                                     ctypes.c_size_t(int(sizes[i])))
        return tot

    bufs = [np.zeros(CHUNK, np.uint8) for _ in range(threads)]
    per = 64
    done, t0 = 0, time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        nxt = 0
        while time.perf_counter() - t0 < seconds:
            futs = []
            for t in range(threads):
                lo = nxt % n
                hi = min(lo + per, n)
                futs.append(ex.submit(work, lo, hi, bufs[t]))
                nxt = hi
            done += sum(f.result() for f in futs)
    el = time.perf_counter() - t0
    return {"value": round(done / el / 1e9, 3), "unit": "GB/s (decompressed bytes)", "cores": threads, "kind": "reference",
            "sample": f"libzstd {z.ZSTD_versionNumber()} ZSTD_decompress of {done >> 20} MiB of the same frames, {threads} threads, {el:.2f} s wall"}


def decompress_leg(d_in, d_out, out_ptrs, out_sizes, n, dev, steps, world):
    """GPU decompression of the frames just produced, device-resident:
    zh_decode_kernel through nvcomp_zstd_batched_decompress_async_v5, timed with events on
    the launch stream after one warm-up; output compared with the input on the device."""
    import cuda_zstd

    bd = cuda_zstd.BatchedDecompressor()
    back = torch.empty(n * CHUNK, dtype=torch.uint8, device=dev)
    ar = torch.arange(n, dtype=torch.int64, device=dev)
    back_ptrs = back.data_ptr() + ar * CHUNK
    dsizes = torch.zeros(n, dtype=torch.int64, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    temp = torch.empty(bd.temp_size(n, CHUNK), dtype=torch.uint8, device=dev)
    run = lambda: bd.decompress_async(out_ptrs, out_sizes, None, CHUNK, back_ptrs, dsizes, status, temp)
    run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        run()
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    ok = bool((status == 0).all().item()) and bool((dsizes == CHUNK).all().item()) and torch.equal(back, d_in)
    t = torch.tensor([ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = t.item()
    comp = float(out_sizes.sum().item())
    del back, temp
    return {"value": round(world * n * CHUNK / (ms / 1e3) / 1e9, 3), "unit": "GB/s (decompressed bytes)", "kernel": "zh_decode_kernel",
            "ms_per_step": round(ms, 3), "steps": steps, "roundtrip_equal": ok,
            "hbm_GBps_algorithmic": round((n * CHUNK + comp) / (ms / 1e3) / 1e9, 2)}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/*_rocprof_summary.json, written by tools/prof_summary.py: 2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of the microarchitecture guide)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_rocprof_summary.json")))
    if not files:
        return None, None
    k = json.load(open(files[-1])).get("kernels", {}).get(kernel, {})
    b = k.get("hbm_bytes")
    return (int(b) if b else None), os.path.relpath(files[-1], ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dataset", default="mix", choices=sorted(SEEDS))
    ap.add_argument("--chunks", type=int, default=CHUNKS_PER_GPU, help="chunks per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the libzstd decode of every rank-0 frame after timing")
    ap.add_argument("--no-decompress", action="store_true", help="skip the GPU decompression leg")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import cuda_zstd

    n = args.chunks
    from cuda_zstd import shard

    host = gen_chunks(args.dataset, n, first=shard.weak_range(rank, n)[0])
    d_in = torch.from_numpy(host).to(dev)
    bc = cuda_zstd.BatchedCompressor(3, CHUNK)
    slot = (bc.max_out(CHUNK) + 255) // 256 * 256
    d_out = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    ar = torch.arange(n, dtype=torch.int64, device=dev)
    in_ptrs = d_in.data_ptr() + ar * CHUNK
    out_ptrs = d_out.data_ptr() + ar * slot
    in_sizes = torch.full((n,), CHUNK, dtype=torch.int64, device=dev)
    out_sizes = torch.zeros(n, dtype=torch.int64, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)
    temp = torch.empty(bc.temp_size(n, CHUNK), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    from cuda_zstd import shard

    def step():
        bc.compress_async(in_ptrs, in_sizes, CHUNK, out_ptrs, out_sizes, status, temp, stream)
        # RCCL all-gather of the per-chunk sizes -> global frame offsets (the only exchange)
        return shard.gather_offsets(out_sizes, world)[1]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    cuda_zstd.profile_enable(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    cuda_zstd.profile_enable(False)
    launches, kms = cuda_zstd.profile_collect()

    assert int((status != 0).sum().item()) == 0, "compression failed on some chunks"
    comp = int(out_sizes.sum().item())
    stats = torch.tensor([el, float(comp), kms[0] / max(launches, 1), kms[1] / max(launches, 1)], dtype=torch.float64, device=dev)
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = stats.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        el, comp_all = mx[0].item(), tot[1].item()
        k1, k2 = mx[2].item(), mx[3].item()
    else:
        comp_all, k1, k2 = float(comp), stats[2].item(), stats[3].item()

    verified = None
    if not args.no_verify and rank == 0:
        verified = libzstd_roundtrip(d_out.cpu().numpy(), out_sizes.cpu().numpy(), slot, host)

    dec = None
    if not args.no_decompress:
        dec = decompress_leg(d_in, d_out, out_ptrs, out_sizes, n, dev, min(args.steps, 5), world)

    if rank == 0:
        total_in = float(world * n * CHUNK)
        gbs = total_in * args.steps / el / 1e9
        # dominant kernel roofline: algorithmic bytes per launch = sum over its chunks of (input + compressed)
        per_launch_bytes = n * CHUNK + comp_all / world
        dom, dom_ms = ("zh_lz_kernel", k1) if k1 >= k2 else ("entropy_stage", k2)
        achieved = per_launch_bytes / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(dom) if args.dataset == "mix" and n == CHUNKS_PER_GPU else (None, None)
        line = {
            "metric": METRIC, "value": round(gbs, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": f"synthetic {args.dataset} corpus (tools/datagen.c, seed {SEEDS[args.dataset]:#x}), device-resident",
            "config": {"workload": f"C3: {n} x 64 KiB chunks ({n * CHUNK / 2**30:.2f} GiB) per GPU, level 3, independent frames",
                       "chunk_bytes": CHUNK, "chunks_per_gpu": n, "level": 3, "ratio": round(total_in / comp_all, 4),
                       "kernel_ms": {"zh_lz_kernel": round(k1, 3), "entropy_stage": round(k2, 3)},
                       "parallelism": f"dp{world} (chunk shards, RCCL all-gather of sizes)", "libzstd_verified": verified},
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "algorithmic_bytes_per_launch": int(per_launch_bytes), "traffic_source": traffic_src},
        }
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        if dec is not None:
            if not args.no_cpu_baseline:
                dec["cpu_baseline"] = cpu_decompress_baseline(d_out.cpu().numpy(), out_sizes.cpu().numpy(), slot, threads)
            line["decompress"] = dec
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(host, threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
