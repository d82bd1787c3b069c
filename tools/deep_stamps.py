"""Diagnostic: per-phase cycles of zh_lz_deep_kernel (levels >= 9) from the -DZH_STAMPS build
(tools/libcuda_zstd_hip_stamps.so): C5-style 16 KiB JSON records without and with a 64 KiB
dictionary.  Not a benchmark."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CUDA_ZSTD_HIP_LIB"] = os.environ.get("STAMPS_LIB") or os.path.join(ROOT, "tools", "libcuda_zstd_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

import cuda_zstd
import zh_testlib as T

REC, N = 16384, 2048
recs = T.gen(T.DG_JSON, N, 0x5EED0005, REC)
d = cuda_zstd.Dictionary.train([recs[i * REC:(i + 1) * REC] for i in range(0, N, 4)], 65536)
dev = torch.from_numpy(recs).cuda()
L = ctypes.CDLL(os.environ["CUDA_ZSTD_HIP_LIB"])
L.zh_deep_fix_host.restype = ctypes.c_uint32
a256 = lambda v: (v + 255) // 256 * 256
WS = 13120 * 8 + 122880 + 256 + 4096
for use in (False, True):
    bc = cuda_zstd.BatchedCompressor(9, REC)
    if use:
        bc.set_dictionary(d)
    slot = (bc.max_out(REC) + 255) // 256 * 256
    out = torch.empty(N * slot, dtype=torch.uint8, device="cuda")
    ar = torch.arange(N, dtype=torch.int64, device="cuda")
    args = (dev.data_ptr() + ar * REC, torch.full((N,), REC, dtype=torch.int64, device="cuda"), REC, out.data_ptr() + ar * slot,
            torch.zeros(N, dtype=torch.int64, device="cuda"), torch.zeros(N, dtype=torch.int32, device="cuda"))
    temp = torch.empty(bc.temp_size_for([REC] * N), dtype=torch.uint8, device="cuda")
    L.zh_deep_fix_host()
    bc.compress_async(*args, temp)
    torch.cuda.synchronize()
    fix = L.zh_deep_fix_host()
    base = a256(temp.data_ptr()) - temp.data_ptr()
    off = a256(N * 56)
    off = a256(off + N * 24)
    off = a256(off + N * 4)
    off = a256(off + N * 8)
    off = a256(off + N * 4)
    off = a256(off + 0)
    off = a256(off + 4)
    blocks = base + off
    h = temp.cpu().numpy()
    m = np.array([h[blocks + b * WS + 13120 * 8 + 122880: blocks + b * WS + 13120 * 8 + 122880 + 256].view(np.uint32) for b in range(N)])
    st = m[:, 34:39].astype(np.float64)
    ph = np.diff(np.concatenate([np.zeros((N, 1)), st], 1), axis=1)
    names = ["stage+hash", "chains", "search", "take+walk", "emit"]
    print("dict" if use else "no dict", "nseq mean", m[:, 0].mean(), "mean cycles/record", int(st[:, 4].mean()), "fix-up steps", fix)
    for k, nm in enumerate(names):
        print(f"  {nm:12s} {ph[:, k].mean():10.0f}  {ph[:, k].mean() / st[:, 4].mean() * 100:5.1f}%")
    # demand-driven path (dbg[20..23] = m[24..28]): search rounds, positions searched, first walk, Jacobi
    dm = m[:, 24:28].astype(np.float64)
    if dm[:, 0].any():
        print(f"  demand path: search rounds {dm[:, 0].mean():.1f}, positions searched {dm[:, 1].mean():.0f} of {REC}"
              f" ({dm[:, 1].mean() / REC * 100:.1f}%), first walk {dm[:, 2].mean():.0f} cycles, Jacobi {dm[:, 3].mean():.0f}"
              " (search+take+walk above = set-up; emit = walk + Jacobi + records)")
        print(f"  Jacobi iterations {m[:, 28].astype(np.float64).mean():.2f}, slowest wave's first walk {m[:, 29].astype(np.float64).mean():.0f} cycles")
        ph4 = m[:, 4:8].astype(np.float64).mean(0)
        print(f"  wave 0 of the workgroup, summed over rounds: advance {ph4[0]:.0f}, post + barrier {ph4[1]:.0f}, search {ph4[2]:.0f},"
              f" barrier after search {ph4[3]:.0f} cycles")
