"""Benchmark: BASELINE.json metric "compress GB/s + ratio, 1 GB @ level 3, 64 KB chunks;
libzstd round-trip OK" on MI355X.

Workload (config C3): 16384 x 64 KiB chunks (1 GiB, Silesia-like
synthetic mix, seed 0x5EED0003) already resident in HBM, compressed through the
stream-ordered C-ABI entry nvcomp_zstd_batched_compress_async_v5 (K1 zh_lz_kernel ->
K2 zh_entropy_kernel -> zh_fse_chain_kernel -> zh_seq_pack_kernel).

Multi-GPU (C4): one process per GPU; the SAME 16384-chunk batch is split
into contiguous ranges of ceil(B/G) chunks (shard.ShardPlan) -- strong scaling -- with no
data-path collective.  The only exchange is the RCCL all-gather of the per-chunk
compressed sizes that gives every rank the global frame offsets; it is inside the timed
step, and the step time is the max over ranks.  --weak keeps 16384 chunks per rank.
An optional payload gather (every rank's frames into one contiguous image on rank 0,
RCCL all-gather of the padded frame slots) is timed separately (--payload-gather).

Prints one JSON line (driver contract).  roofline = the dominant kernel's algorithmic
bytes (input + compressed output) per launch / its average HIP-event
duration on the launch stream, plus the measured issue-rate fraction of that kernel from
the committed rocprofv3 SQ summary (profiles/*_sq_summary.json); `limiter` compares the
two fractions.  cpu_baseline = libzstd level 3 (the reference's own CPU route,
src/cuda_zstd_manager.cu:1604-1668) through tools/libcpubench.so: one ZSTD_CCtx per
POSIX thread, ZSTD_compressCCtx over the same chunks, a 1, 2, 4, ... thread curve up to
the box's host share (--cpu-threads all: every thread of the affinity).  vs_baseline is null:
BASELINE.md publishes no number for this metric.  cpu_baseline.gpu_speedup gives GPU GB/s over
the measured thread count, one thread and all cores (the north star's ">= 10x all-core" ratio,
also the line's `vs_cpu_all_core`): all-core is measured when the process may use every core,
otherwise the larger of the measured rate and the 1-thread rate x physical cores x the measured
parallel efficiency (the conservative denominator).
Extra legs at N=1 (not `value`): C3 on uniform random bytes, C3 at levels 1 and 2, C2 (one 64 MiB frame through
ZstdManager::compress) and C5 (level 9 with a COVER dictionary on 4,096 x 16 KiB JSON records),
each with its roofline and libzstd beside it, and GPU decompression of the C3 frames.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

CHUNK = 64 * 1024
CHUNKS = 16384
HBM_PEAK_GBS = 8000.0
N_SIMD = 1024          # 256 CUs x 4 SIMDs
VALU_CYCLES_1W = 4     # one wave alone issues a wave64 VALU every 4 cycles (MI355X_MICROARCH.md)
VALU_CYCLES_PIPE = 2   # the SIMD-32 pipe takes a wave64 VALU in 2 cycles when several waves issue
METRIC = "compress GB/s + ratio, 1 GB @ level 3, 64 KB chunks; libzstd round-trip OK"
SEEDS = {"mix": 0x5EED0003, "random": 0x5EED0004}
C2_BYTES, C2_SEED = 64 << 20, 0x5EED0002


def gen_chunks(kind, n, first):
    import zh_testlib as T

    return T.gen(T.KINDS[kind], n, SEEDS[kind], CHUNK, first=first)


# ----------------------------------------------------------------------------- host CPU
def host_info():
    model, phys = None, set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if not line.strip():
                if "physical id" in cur and "core id" in cur:
                    phys.add((cur["physical id"], cur["core id"]))
                cur = {}
                continue
            k, _, v = line.partition(":")
            cur[k.strip()] = v.strip()
            if k.strip() == "model name" and model is None:
                model = v.strip()
    except OSError:
        pass
    return {"cpu_model": model, "physical_cores": len(phys) or None, "hw_threads": os.cpu_count(),
            "affinity_threads": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": cgroup_quota()}


def cgroup_quota():
    """CPUs the process's cgroup may use (cpu.max quota / period), None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def host_share():
    """Threads this process may keep busy: the affinity, capped by the cgroup quota and by the
    pool's per-GPU host share (OMP_NUM_THREADS, 16 on the GPU pool: the harness asks worker
    pools to stay within it)."""
    aff = len(os.sched_getaffinity(0))
    q = cgroup_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    t = aff
    if q:
        t = min(t, max(1, int(q)))
    if omp:
        t = min(t, omp)
    return max(1, t)


def _cpubench():
    so = os.path.join(ROOT, "tools", "libcpubench.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    L.cpub_run.restype = ctypes.c_int
    L.cpub_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_size_t)]
    L.cpub_run_pinned.restype = ctypes.c_int
    L.cpub_run_pinned.argtypes = L.cpub_run.argtypes + [ctypes.POINTER(ctypes.c_int)]
    L.cpub_zstd_version.restype = ctypes.c_uint
    return L


def cpu_run(mode, data, nchunks, threads, passes=5, sizes=None, slot=0, chunk=CHUNK, level=3, cpus=None):
    """Median wall time of `passes` sweeps over nchunks chunks (after one warm-up sweep); cpus:
    pin thread t to CPU cpus[t]."""
    L = _cpubench()
    if L is None:
        return None
    secs = (ctypes.c_double * (passes + 1))()
    outb = ctypes.c_size_t()
    sz = sizes.ctypes.data if sizes is not None else None
    pin = (ctypes.c_int * threads)(*cpus) if cpus else None
    rc = L.cpub_run_pinned(mode, data.ctypes.data, sz, nchunks, chunk, slot, level, threads, passes + 1, secs, ctypes.byref(outb), pin)
    if rc:
        return None
    t = statistics.median(list(secs)[1:])
    return {"seconds": t, "out_bytes": outb.value, "version": L.cpub_zstd_version()}


def smt_yield(host, mode=0, sizes=None, slot=0, ref_g1=None):
    """libzstd throughput (mode 0: level-3 compression of the chunks in `host`; mode 1:
    decompression of the frames in `host`, `sizes` bytes at `slot` strides) of one core's two
    hardware threads over one thread alone, both pinned (the hardware threads the affinity holds
    beyond the physical cores are worth this much each, not a whole core).  The box shares its
    host: a core whose pinned thread runs below 0.8 x `ref_g1` (the unpinned 1-thread rate) is
    busy with someone else's work, so up to 4 cores spread over the affinity are tried and the
    median yield of the uncontended ones is reported (round 6: a contended cpu 0 ran at a third
    of the unpinned rate and reported a yield above 4).  None when no sibling pair was usable."""
    aff = sorted(os.sched_getaffinity(0))
    pairs, seen = [], set()
    # candidate cores spread over the affinity list, cpu 0 last (it takes the host's interrupts)
    order = [aff[(len(aff) * j) // 8] for j in (1, 3, 5, 7, 2, 6)] + aff
    for a in order:
        if a in seen:
            continue
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{a}/topology/thread_siblings_list").read().strip()
        except OSError:
            return None
        ids = set()
        for part in sib.split(","):
            lo, _, hi = part.partition("-")
            ids.update(range(int(lo), int(hi or lo) + 1))
        seen.update(ids)
        b = next((x for x in sorted(ids) if x != a and x in aff), None)
        if b is not None and a != 0:
            pairs.append((a, b))
        if len(pairs) == 4:
            break
    avail = len(sizes) if sizes is not None else len(host) // CHUNK
    n = min(avail, 512)
    n2 = 2 * n if avail >= 2 * n else n
    tried = []
    for a, b in pairs:
        r1 = cpu_run(mode, host, n, 1, passes=3, cpus=[a], sizes=sizes, slot=slot)
        r2 = cpu_run(mode, host, n2, 2, passes=3, cpus=[a, b], sizes=sizes, slot=slot)
        if not r1 or not r2:
            continue
        g1 = n * CHUNK / r1["seconds"]
        g2 = n2 * CHUNK / r2["seconds"]
        ok = ref_g1 is None or g1 >= 0.8 * ref_g1 * 1e9
        tried.append({"cpus": [a, b], "one_thread_GBps": round(g1 / 1e9, 4), "two_siblings_GBps": round(g2 / 1e9, 4),
                      "yield": round(g2 / g1, 3), "uncontended": ok})
        if sum(t["uncontended"] for t in tried) >= 2:
            break
    good = sorted(t["yield"] for t in tried if t["uncontended"])
    if not good:
        return None
    return {"value": good[len(good) // 2], "pairs": tried,
            "rule": "median over pinned sibling pairs whose 1-thread rate is >= 0.8 x the unpinned 1-thread rate"}


def cpu_baseline(host, threads, gpu_gbs):
    """libzstd level 3 over the same chunks, median of 5 sweeps after a warm-up each:
    1 thread on a 1024-chunk (64 MiB) sample, then 2, 4, 8, ... threads on 1024 chunks per
    thread, up to `threads` threads on the whole rank-0 batch (the reported value).  The
    all-core figure extrapolates the 1-thread rate to every physical core at the parallel
    efficiency measured at `threads`; with --cpu-threads all it is measured instead."""
    n = len(host) // CHUNK
    curve, t = [], 1
    while True:
        nt = n if t >= threads else min(n, 1024 * t)
        r = cpu_run(0, host, nt, t)
        if r is None:
            return None
        curve.append({"threads": t, "chunks": nt, "GBps": round(nt * CHUNK / r["seconds"] / 1e9, 4), "_r": r})
        if t >= threads:
            break
        t = min(2 * t, threads)
    one, many = curve[0], curve[-1]
    g1, gm = one["GBps"], many["GBps"]
    info = host_info()
    cores = info["physical_cores"] or threads
    eff = gm / (threads * g1)
    all_core = g1 * cores * min(1.0, eff)
    r = many.pop("_r")
    for c in curve:
        c.pop("_r", None)
    measured_all = threads >= (info["physical_cores"] or info["affinity_threads"] or threads)
    # every hardware thread: the physical-core figure times the measured SMT yield of a core's two
    # threads (the affinity holds 2 threads per core); the denominator of
    # gpu_speedup.vs_all_core
    hw = info["affinity_threads"] or threads
    smt = smt_yield(host, ref_g1=g1) if (hw > cores and not measured_all) else None
    smt_f = min(smt["value"], 2.0) if smt else (hw / cores if hw > cores else 1.0)
    base_all = gm if measured_all else max(gm, all_core)
    all_hw = base_all * (smt_f if hw > cores and not measured_all else 1.0)
    return {"value": round(gm, 3), "unit": "GB/s", "cores": threads, "kind": "reference",
            "sample": f"libzstd {r['version']} ZSTD_compressCCtx level 3 (one CCtx per POSIX thread, tools/cpubench.c) over the same 64 KiB "
                      f"chunks: {threads} threads x {n} chunks ({n * CHUNK >> 20} MiB), median of 5 sweeps; ratio {n * CHUNK / r['out_bytes']:.4f}",
            "ratio": round(n * CHUNK / r["out_bytes"], 4),
            "single_thread": {"value": g1, "unit": "GB/s", "sample": f"{curve[0]['chunks']} chunks, median of 5 sweeps"},
            "thread_curve": curve,
            "host": info,
            "all_core": {"value": round(all_hw, 2), "unit": "GB/s", "measured": measured_all,
                         "physical_cores_value": round(base_all, 2), "hw_threads": hw, "smt_yield": smt,
                         "how": ("measured: one thread per physical core or more" if measured_all else
                                 f"1-thread rate x {cores} physical cores x the parallel efficiency {eff:.3f} measured at {threads} threads "
                                 f"= {base_all:.2f} GB/s, x {smt_f:.3f} for the second hardware thread of each core "
                                 f"({'measured: two pinned sibling threads over one' if smt else 'not measurable here: counted as a whole core'}; "
                                 f"affinity {info['affinity_threads']} threads, cgroup quota {info['cgroup_cpu_quota']}, pool share "
                                 f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}; bench.py --cpu-threads all measures it on a whole machine)")},
            "gpu_speedup": {"vs_measured_threads": round(gpu_gbs / gm, 2), "vs_single_thread": round(gpu_gbs / g1, 1),
                            "vs_all_core": round(gpu_gbs / all_hw, 2), "vs_all_physical_cores": round(gpu_gbs / base_all, 2),
                            "north_star_10x_all_core": gpu_gbs >= 10 * all_hw}}


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


# ----------------------------------------------------------------------------- GPU legs
class Batch:
    """Device-resident chunk slots + the stream-ordered batched compressor."""

    def __init__(self, host, dev, level=3):
        import cuda_zstd

        self.n = n = len(host) // CHUNK
        self.dev = dev
        self.host = host
        self.d_in = torch.from_numpy(host).to(dev)
        self.bc = cuda_zstd.BatchedCompressor(level, CHUNK)
        self.slot = (self.bc.max_out(CHUNK) + 255) // 256 * 256
        self.d_out = torch.empty(max(n, 1) * self.slot, dtype=torch.uint8, device=dev)
        ar = torch.arange(n, dtype=torch.int64, device=dev)
        self.in_ptrs = self.d_in.data_ptr() + ar * CHUNK
        self.out_ptrs = self.d_out.data_ptr() + ar * self.slot
        self.in_sizes = torch.full((n,), CHUNK, dtype=torch.int64, device=dev)
        self.out_sizes = torch.zeros(n, dtype=torch.int64, device=dev)
        self.status = torch.zeros(n, dtype=torch.int32, device=dev)
        self.temp = torch.empty(max(self.bc.temp_size(max(n, 1), CHUNK), 256), dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.current_stream(dev)

    def compress(self):
        if self.n:
            self.bc.compress_async(self.in_ptrs, self.in_sizes, CHUNK, self.out_ptrs, self.out_sizes, self.status, self.temp, self.stream)


def leg_roofline(per_launch_bytes, kms, launches, lz_name="zh_lz_kernel"):
    """Roofline of a leg's dominant kernel (K1 or the entropy stage), as the main line's: algorithmic
    bytes per launch (input + compressed output) over its average HIP-event duration on the launch
    stream (cuda_zstd.profile_*); no PMC traffic is taken for the legs."""
    k1, k2 = kms[0] / max(launches, 1), kms[1] / max(launches, 1)
    dom, ms = (lz_name, k1) if k1 >= k2 else ("entropy_stage", k2)
    ach = per_launch_bytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    return {"kernel": dom, "bound": "hbm" if ach / HBM_PEAK_GBS > 0.5 else "issue", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None, "algorithmic_bytes_per_launch": int(per_launch_bytes),
            "kernel_ms": {lz_name: round(k1, 3), "entropy_stage": round(k2, 3)}}


def timed_events(fn, steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def random_leg(dev, steps, threads):
    """C3 on uniform random bytes (seed 0x5EED0004): every block dies at K1's incompressibility
    probe and goes out raw.  Roofline of its dominant kernel and libzstd on the same chunks."""
    import cuda_zstd

    host = gen_chunks("random", CHUNKS, 0)
    b = Batch(host, dev)
    b.compress()
    torch.cuda.synchronize()
    cuda_zstd.profile_enable(True)
    ms = timed_events(b.compress, steps)
    cuda_zstd.profile_enable(False)
    launches, kms = cuda_zstd.profile_collect()
    ok = int((b.status != 0).sum().item()) == 0
    comp = int(b.out_sizes.sum().item())
    gbs = CHUNKS * CHUNK / (ms / 1e3) / 1e9
    res = {"value": round(gbs, 3), "unit": "GB/s", "ms_per_step": round(ms, 3), "ratio": round(CHUNKS * CHUNK / comp, 4),
           "status_ok": ok, "workload": "C3-random: 16384 x 64 KiB uniform random chunks, level 3",
           "roofline": leg_roofline(CHUNKS * CHUNK + comp, kms, launches)}
    verified = libzstd_roundtrip(b.d_out.cpu().numpy(), b.out_sizes.cpu().numpy(), b.slot, host)
    res["libzstd_verified"] = verified
    del b
    torch.cuda.empty_cache()
    if threads:
        res["cpu_baseline"] = cpu_baseline(host, threads, gbs)
    return res


def level_leg(host, dev, level, steps, threads):
    """C3 (the main line's 16,384 mix chunks) at another level: level 1 is
    K1's short-table greedy parse (ZH_K1_MODE 2), level 2 the short-table lazy-1 (mode 1).  GB/s,
    ratio, libzstd decode of every frame, and libzstd at the same level on one thread over the
    first 1,024 chunks (64 MiB) beside it."""
    import cuda_zstd

    b = Batch(host, dev, level)
    b.compress()
    torch.cuda.synchronize()
    cuda_zstd.profile_enable(True)
    ms = timed_events(b.compress, steps)
    cuda_zstd.profile_enable(False)
    launches, kms = cuda_zstd.profile_collect()
    ok = int((b.status != 0).sum().item()) == 0
    comp = int(b.out_sizes.sum().item())
    gbs = b.n * CHUNK / (ms / 1e3) / 1e9
    n1k = min(b.n, 1024)
    comp1k = int(b.out_sizes[:n1k].sum().item())
    res = {"value": round(gbs, 3), "unit": "GB/s", "ms_per_step": round(ms, 3), "ratio": round(b.n * CHUNK / comp, 4), "status_ok": ok,
           # (on the chunks libzstd's line below compresses: the like-for-like ratio)
           "ratio_first_1024": round(n1k * CHUNK / comp1k, 4) if comp1k else None,
           "workload": f"C3 mix: {b.n} x 64 KiB chunks, level {level}", "roofline": leg_roofline(b.n * CHUNK + comp, kms, launches)}
    res["libzstd_verified"] = libzstd_roundtrip(b.d_out.cpu().numpy(), b.out_sizes.cpu().numpy(), b.slot, host)
    del b
    torch.cuda.empty_cache()
    if threads:
        n = min(len(host) // CHUNK, 1024)
        r = cpu_run(0, host, n, 1, passes=3, level=level)
        if r:
            res["cpu_baseline"] = {"value": round(n * CHUNK / r["seconds"] / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "reference",
                                   "sample": f"libzstd {r['version']} ZSTD_compressCCtx level {level}, one thread, the first {n} chunks, "
                                             "median of 3 after a warm-up", "ratio": round(n * CHUNK / r["out_bytes"], 4)}
    return res


def c2_leg(dev, steps, threads):
    """C2: one 64 MiB buffer (iid over a seeded 16-symbol alphabet) -> one frame through
    ZstdManager::compress (cuda_zstd_compress); libzstd decodes the frame; libzstd level-3
    ratio of the same buffer beside ours, and libzstd's time for the same single 64 MiB frame
    (ZSTD_compressCCtx, one thread: one frame is one thread's work in libzstd without its
    multi-threaded frame mode)."""
    import cuda_zstd
    import zh_testlib as T

    host = T.gen(T.DG_SYM16, 1, C2_SEED, C2_BYTES)
    d = torch.from_numpy(host).to(dev)
    m = cuda_zstd.Manager(3)
    f = m.compress(d)
    torch.cuda.synchronize()
    cuda_zstd.profile_enable(True)
    ms = timed_events(lambda: m.compress(d), steps)
    cuda_zstd.profile_enable(False)
    launches, kms = cuda_zstd.profile_collect()
    frame = f.cpu().numpy().tobytes()
    res = {"value": round(C2_BYTES / (ms / 1e3) / 1e9, 3), "unit": "GB/s", "ms_per_call": round(ms, 3), "ratio": round(C2_BYTES / len(frame), 4),
           "workload": "C2: 64 MiB iid 16-symbol buffer, one frame (2048 x 32 KiB blocks, each matched against the 32 KiB before it), ZstdManager::compress incl. its host sync",
           "roofline": leg_roofline(C2_BYTES + len(frame), kms, launches)}
    if threads:
        r = cpu_run(0, host, 1, 1, passes=3, chunk=C2_BYTES)
        if r:
            res["cpu_baseline"] = {"value": round(C2_BYTES / r["seconds"] / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "reference",
                                   "sample": f"libzstd {r['version']} ZSTD_compressCCtx level 3 of the same 64 MiB buffer as one frame, "
                                             "median of 3 after a warm-up", "ratio": round(C2_BYTES / r["out_bytes"], 4)}
    z = T.zstd()
    if z is not None:
        res["libzstd_verified"] = T.zstd_decompress(frame, C2_BYTES) == host.tobytes()
        res["libzstd_l3_ratio"] = round(C2_BYTES / len(T.zstd_compress(host.tobytes(), 3)), 4)
    m.close()
    return res


def c5_leg(dev, threads):
    """C5 (BASELINE.json configs[4]): 4,096 x 16 KiB JSON-like records at level 9 (the deep chain
    matcher, LAZY2 parse) through the stream-ordered batch path, without a dictionary and with a
    64 KiB COVER dictionary trained on every fourth record (tools/c5_dict.py's workload and
    timing: device-resident records, HIP events, median of 5 after a warm-up).  CPU baseline:
    libzstd ZSTD_compress_usingCDict level 9 with the same dictionary, one thread, every record.
    libzstd decodes every GPU frame with the dictionary."""
    import cuda_zstd
    import zh_testlib as T

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c5_dict as C

    host = T.gen(T.DG_JSON, C.N, C.SEED, C.REC)
    recs = [host[i * C.REC:(i + 1) * C.REC] for i in range(C.N)]
    cover = cuda_zstd.Dictionary.train(recs[::4], C.DICT).content()
    d_recs = torch.from_numpy(host).to(dev)
    total = C.N * C.REC
    runs = {}
    for name, d in (("none", None), ("cover", cover)):
        cuda_zstd.profile_enable(True)
        frames, t = C.gpu_run(d_recs, d)
        cuda_zstd.profile_enable(False)
        launches, kms = cuda_zstd.profile_collect()
        comp = sum(len(f) for f in frames)
        ok = all(T.zstd_decompress(f, C.REC, dictionary=d) == r.tobytes() for r, f in zip(recs, frames)) if T.zstd() else None
        runs[name] = {"value": round(total / t / 1e9, 3), "ratio": round(total / comp, 4), "libzstd_verified": ok,
                      "roofline": leg_roofline(total + comp, kms, launches, "zh_lz_deep_kernel")}
    res = dict(runs["cover"])
    res.update({"unit": "GB/s", "level": C.LEVEL, "dict_bytes": len(cover),
                "workload": "C5: 4096 x 16 KiB JSON-like records, level 9 (LAZY2 deep chain matcher), 64 KiB COVER dictionary "
                            "trained on every 4th record; BatchedCompressor with the dictionary on the handle",
                "no_dict": runs["none"]})
    if threads and T.zstd():
        lz, el = C.libzstd_cdict(recs, cover, C.LEVEL)
        res["cpu_baseline"] = {"value": round(total / el / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "reference",
                               "sample": "libzstd ZSTD_compress_usingCDict level 9 with the same COVER dictionary, one thread, all 4096 records",
                               "ratio": round(total / lz, 4)}
    del d_recs
    return res


def decompress_leg(b, steps, world):
    """GPU decompression of the frames just produced, device-resident:
    zh_decode_kernel through nvcomp_zstd_batched_decompress_async_v5, timed with events on
    the launch stream after one warm-up; output compared with the input on the device."""
    import cuda_zstd

    n, dev = b.n, b.dev
    bd = cuda_zstd.BatchedDecompressor()
    back = torch.empty(max(n, 1) * CHUNK, dtype=torch.uint8, device=dev)
    ar = torch.arange(n, dtype=torch.int64, device=dev)
    back_ptrs = back.data_ptr() + ar * CHUNK
    dsizes = torch.zeros(n, dtype=torch.int64, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    temp = torch.empty(max(bd.temp_size(max(n, 1), CHUNK), 256), dtype=torch.uint8, device=dev)

    def run():
        if n:
            bd.decompress_async(b.out_ptrs, b.out_sizes, None, CHUNK, back_ptrs, dsizes, status, temp)

    run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ms = timed_events(run, steps)
    ok = bool((status == 0).all().item()) and bool((dsizes == CHUNK).all().item()) and torch.equal(back[: n * CHUNK], b.d_in)
    t = torch.tensor([ms, float(n), float(b.out_sizes.sum().item())], dtype=torch.float64, device=dev)
    okt = torch.tensor([0 if ok else 1], dtype=torch.int64, device=dev)
    if world > 1:
        tot = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(okt, op=dist.ReduceOp.SUM)
        n_all, comp = tot[1].item(), tot[2].item()
    else:
        n_all, comp = float(n), t[2].item()
    ms = t[0].item()
    del back, temp
    return {"value": round(n_all * CHUNK / (ms / 1e3) / 1e9, 3), "unit": "GB/s (decompressed bytes)", "kernel": "zh_decode_kernel",
            "ms_per_step": round(ms, 3), "steps": steps, "roundtrip_equal": okt.item() == 0,
            "hbm_GBps_algorithmic": round((n_all * CHUNK + comp) / (ms / 1e3) / 1e9, 2)}


def cpu_decompress_baseline(b, threads, gpu_gbs=None):
    """libzstd ZSTD_decompressDCtx (the reference's CPU decode route, src/cuda_zstd_manager.cu:
    3219-3344) over the rank-0 frames: `threads` threads (the value), one thread on the first
    1,024 frames, and the all-core figure as the compress legs derive it (VERDICT r5 missing #3):
    measured when the process may use every core, else the 1-thread rate x physical cores x the
    parallel efficiency measured at `threads`, x the SMT yield of two pinned sibling threads."""
    frames = b.d_out.cpu().numpy()
    sizes = b.out_sizes.cpu().numpy().astype(np.uint64)
    r = cpu_run(1, frames, b.n, threads, sizes=sizes, slot=b.slot)
    if r is None:
        return None
    gm = b.n * CHUNK / r["seconds"] / 1e9
    n1 = min(b.n, 1024)
    r1 = cpu_run(1, frames, n1, 1, passes=3, sizes=sizes, slot=b.slot)
    g1 = n1 * CHUNK / r1["seconds"] / 1e9 if r1 else None
    info = host_info()
    cores = info["physical_cores"] or threads
    hw = info["affinity_threads"] or threads
    measured_all = threads >= cores
    res = {"value": round(gm, 3), "unit": "GB/s (decompressed bytes)", "cores": threads, "kind": "reference",
           "sample": f"libzstd {r['version']} ZSTD_decompressDCtx of the {b.n} frames, {threads} threads, median of 5 sweeps"}
    if g1:
        eff = gm / (threads * g1)
        base_all = gm if measured_all else max(gm, g1 * cores * min(1.0, eff))
        smt = smt_yield(frames, mode=1, sizes=sizes, slot=b.slot, ref_g1=g1) if (hw > cores and not measured_all) else None
        smt_f = min(smt["value"], 2.0) if smt else (hw / cores if hw > cores else 1.0)
        all_hw = base_all * (smt_f if hw > cores and not measured_all else 1.0)
        res["single_thread"] = {"value": round(g1, 4), "unit": "GB/s (decompressed bytes)", "sample": f"the first {n1} frames, median of 3 sweeps"}
        res["all_core"] = {"value": round(all_hw, 2), "unit": "GB/s (decompressed bytes)", "measured": measured_all,
                           "physical_cores_value": round(base_all, 2), "hw_threads": hw, "smt_yield": smt,
                           "how": ("measured: one thread per physical core or more" if measured_all else
                                   f"1-thread rate x {cores} physical cores x the parallel efficiency {eff:.3f} measured at {threads} threads "
                                   f"= {base_all:.2f} GB/s, x {smt_f:.3f} for the second hardware thread of each core")}
        if gpu_gbs:
            res["gpu_speedup"] = {"vs_measured_threads": round(gpu_gbs / gm, 2), "vs_single_thread": round(gpu_gbs / g1, 1),
                                  "vs_all_core": round(gpu_gbs / all_hw, 3), "vs_all_physical_cores": round(gpu_gbs / base_all, 3)}
    return res


# ----------------------------------------------------------------------------- profiles
def _newest(pattern):
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    return files[-1] if files else None


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/*_rocprof_summary.json, written by tools/prof_summary.py: 2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of the microarchitecture guide)."""
    f = _newest("*_rocprof_summary.json")
    if not f:
        return None, None
    b = json.load(open(f)).get("kernels", {}).get(kernel, {}).get("hbm_bytes")
    return (int(b) if b else None), os.path.relpath(f, ROOT)


def issue_fraction(kernel):
    """VALU issue fraction of `kernel` from the newest committed SQ summary
    (profiles/*_sq_summary.json, tools/sq_summary.py): SQ_INSTS_VALU x 4 cycles over
    1024 SIMDs x the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs)."""
    f = _newest("*_sq_summary.json")
    if not f:
        return None
    k = json.load(open(f)).get("kernels", {}).get(kernel)
    if not k:
        return None
    return {"valu_issue_frac": k.get("valu_issue_frac"), "salu_per_valu": k.get("salu_per_valu"),
            "lds_bank_conflict_frac": k.get("lds_bank_conflict_frac"), "valu_insts_per_input_byte": k.get("valu_insts_per_input_byte"),
            "source": os.path.relpath(f, ROOT)}


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dataset", default="mix", choices=sorted(SEEDS))
    ap.add_argument("--chunks", type=int, default=CHUNKS, help="chunks in the batch (per GPU with --weak)")
    ap.add_argument("--weak", action="store_true", help="weak scaling: every rank compresses --chunks chunks of its own")
    ap.add_argument("--payload-gather", action="store_true", help="also time an RCCL gather of every rank's frames (N>1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the libzstd decode of every rank-0 frame after timing")
    ap.add_argument("--no-decompress", action="store_true", help="skip the GPU decompression leg")
    ap.add_argument("--no-legs", action="store_true", help="skip the C3-random, C2 and C5 legs (N=1)")
    ap.add_argument("--cpu-threads", default=None,
                    help="libzstd baseline threads: a number, or 'all' (the process affinity); default: every thread the "
                         "process may keep busy (affinity, capped by the cgroup quota and the pool share OMP_NUM_THREADS)")
    args = ap.parse_args()

    from cuda_zstd import launch

    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if not launch.rank_env_present():
        if args.gpus > 1:
            # C4 without a launcher around us: start one rank per GPU as child processes (before
            # any GPU call here, no exec) and pass rank 0's line through
            ndev = launch.visible_gpus()
            if args.gpus > ndev:
                sys.exit(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) are visible")
            sys.exit(launch.spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    rank, local, world = launch.rank_env()
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} from the launcher overrides --gpus {args.gpus}", file=sys.stderr)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import cuda_zstd
    from cuda_zstd import shard

    if args.weak:
        n_total = args.chunks * world
        lo, hi = shard.weak_range(rank, args.chunks)
        plan = shard.ShardPlan(world, n_total)  # equal slices: q = chunks
    else:
        n_total = args.chunks
        plan = shard.ShardPlan(world, n_total)
        lo, hi = plan.range(rank)
    host = gen_chunks(args.dataset, hi - lo, first=lo)
    b = Batch(host, dev)

    def step():
        b.compress()
        # RCCL all-gather of the per-chunk sizes -> global frame offsets (the only exchange)
        return plan.gather_offsets(b.out_sizes)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    cuda_zstd.profile_enable(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        all_sizes, offs = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    cuda_zstd.profile_enable(False)
    launches, kms = cuda_zstd.profile_collect()

    assert int((b.status != 0).sum().item()) == 0, "compression failed on some chunks"
    comp = int(b.out_sizes.sum().item())
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
    gathered_total = int(all_sizes.sum().item())  # == sum of every rank's frame bytes

    gather = None
    if args.payload_gather and world > 1:
        # frames of every rank into one image: all-gather of the padded slot array (q slots per rank)
        q = plan.q
        pad = torch.zeros(q * b.slot, dtype=torch.uint8, device=dev)
        pad[: b.n * b.slot] = b.d_out[: b.n * b.slot]
        img = torch.empty(world * q * b.slot, dtype=torch.uint8, device=dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        g0 = time.perf_counter()
        dist.all_gather_into_tensor(img, pad)
        torch.cuda.synchronize(dev)
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        gather = {"ms": round(gt.item() * 1e3, 3), "bytes_per_rank": int(q * b.slot),
                  "how": "RCCL all_gather_into_tensor of the padded frame slots (not part of value)"}
        del pad, img

    verified = None
    if not args.no_verify and rank == 0:
        verified = libzstd_roundtrip(b.d_out.cpu().numpy(), b.out_sizes.cpu().numpy(), b.slot, host)

    dec = None
    if not args.no_decompress:
        dec = decompress_leg(b, min(args.steps, 5), world)

    aff = len(os.sched_getaffinity(0))
    if args.cpu_threads == "all":
        threads = aff
    elif args.cpu_threads:
        threads = max(1, min(aff, int(args.cpu_threads)))
    else:
        threads = host_share()
    legs = {}
    if world == 1 and not args.no_legs and args.dataset == "mix" and args.chunks == CHUNKS:
        leg_threads = None if args.no_cpu_baseline else threads
        legs["c3_random"] = random_leg(dev, 5, leg_threads)
        for lv in (1, 2):
            legs[f"c3_level{lv}"] = level_leg(host, dev, lv, 5, leg_threads)
        legs["c2_64mib"] = c2_leg(dev, 5, leg_threads)
        legs["c5_level9_dict"] = c5_leg(dev, leg_threads)

    if rank == 0:
        total_in = float(n_total * CHUNK)
        gbs = total_in * args.steps / el / 1e9
        # dominant kernel roofline: algorithmic bytes per launch = sum over its chunks of (input + compressed)
        per_launch_bytes = b.n * CHUNK + comp
        dom, dom_ms = ("zh_lz_kernel", k1) if k1 >= k2 else ("entropy_stage", k2)
        achieved = per_launch_bytes / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0
        full = args.dataset == "mix" and b.n == CHUNKS
        traffic, traffic_src = pmc_traffic(dom) if full else (None, None)
        issue = issue_fraction(dom) if full else None
        # limiter: the larger of the kernel's HBM fraction (PMC traffic, else algorithmic bytes,
        # over its measured duration) and its VALU issue fraction (committed SQ summary)
        hbm_frac = ((traffic or per_launch_bytes) / (dom_ms / 1e3) / 1e9) / HBM_PEAK_GBS if dom_ms > 0 else 0.0
        iss = (issue or {}).get("valu_issue_frac")
        if issue and iss is not None:
            # the SQ summary prices a VALU at the 1-wave rate (4 cycles); the pipe's own rate is 2
            issue["valu_pipe_frac"] = round(iss * VALU_CYCLES_PIPE / VALU_CYCLES_1W, 4)
        if iss is None:
            bound, limiter = "unknown", f"unknown: no SQ summary for this workload (HBM {hbm_frac:.4f} of peak)"
        elif hbm_frac >= iss:
            bound, limiter = "hbm", f"hbm ({hbm_frac:.3f} of peak >= VALU issue {iss:.3f})"
        else:
            bound = "issue"
            limiter = (f"instruction issue / LDS latency, not HBM: VALU issue {iss:.3f} of the 1-wave rate "
                       f"({issue['valu_pipe_frac']:.3f} of the SIMD pipe), HBM {hbm_frac:.4f} of peak")
        line = {
            "metric": METRIC, "value": round(gbs, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "u8", "data": f"synthetic {args.dataset} corpus (tools/datagen.c, seed {SEEDS[args.dataset]:#x}), device-resident",
            "config": {"workload": f"C3{'' if world == 1 else '/C4'}: {n_total} x 64 KiB chunks ({total_in / 2**30:.2f} GiB), level 3, independent frames"
                                   + ("" if world == 1 else f", {'weak: per rank' if args.weak else 'strong: one batch split'} over {world} GPUs"),
                       "chunk_bytes": CHUNK, "chunks_total": n_total, "chunks_rank0": b.n, "level": 3, "ratio": round(total_in / comp_all, 4),
                       "kernel_ms": {"zh_lz_kernel": round(k1, 3), "entropy_stage": round(k2, 3)},
                       "parallelism": f"dp{world} (contiguous chunk shards, RCCL all-gather of sizes inside the step)",
                       "libzstd_verified": verified, "gathered_frame_bytes": gathered_total},
            # byte work, no MFMA: HBM is the only roofline peak; `bound` names what limits the
            # kernel ("issue" when its VALU issue fraction exceeds its HBM fraction)
            "roofline": {"kernel": dom, "bound": bound, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "algorithmic_bytes_per_launch": int(per_launch_bytes), "traffic_source": traffic_src,
                         "limiter": limiter,
                         "issue": issue},
        }
        if gather:
            line["payload_gather"] = gather
        if dec is not None:
            if not args.no_cpu_baseline and world == 1:
                dec["cpu_baseline"] = cpu_decompress_baseline(b, threads, dec["value"])
            line["decompress"] = dec
        if legs:
            line["legs"] = legs
        if not args.no_cpu_baseline and world == 1:
            cb = cpu_baseline(host, threads, gbs)
            line["cpu_baseline"] = cb
            # vs_baseline stays null: BASELINE.md publishes no number for this metric (the driver
            # contract); the GPU / libzstd ratios are cpu_baseline.gpu_speedup
            if cb:
                line["vs_cpu_all_core"] = cb["gpu_speedup"]["vs_all_core"]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
