"""Diagnostic: per-phase cycle breakdown of zh_lz_kernel (wave 0 of each block),
from the -DZH_STAMPS build (tools/libcuda_zstd_hip_stamps.so).  Not a benchmark."""
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

kind = sys.argv[1] if len(sys.argv) > 1 else "mix"
n, cs = (int(sys.argv[2]) if len(sys.argv) > 2 else 2048), 65536
data = T.gen(T.KINDS[kind], n, 0x5EED0003, cs)
dev = torch.from_numpy(data).cuda()
bc = cuda_zstd.BatchedCompressor(int(os.environ.get("STAMPS_LEVEL", "3")), cs)
slot = (bc.max_out(cs) + 255) // 256 * 256
out = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
ar = torch.arange(n, dtype=torch.int64, device="cuda")
args = (dev.data_ptr() + ar * cs, torch.full((n,), cs, dtype=torch.int64, device="cuda"), cs, out.data_ptr() + ar * slot,
        torch.zeros(n, dtype=torch.int64, device="cuda"), torch.zeros(n, dtype=torch.int32, device="cuda"))
temp = torch.empty(bc.temp_size(n, cs), dtype=torch.uint8, device="cuda")
bc.compress_async(*args, temp)
torch.cuda.synchronize()
a256 = lambda v: (v + 255) // 256 * 256
base = a256(temp.data_ptr()) - temp.data_ptr()
off = a256(n * 56)  # sizeof(ZhBlockDesc)
off = a256(off + n * 24)
off = a256(off + n * 4)
off = a256(off + n * 8)
off = a256(off + n * 4)
off = a256(off + 0)
off = a256(off + 4)  # K1 block counter
blocks = base + off
WS = 13120 * 8 + 122880 + 256 + 4096
h = temp.cpu().numpy()
m0 = h[blocks + 13120 * 8 + 122880: blocks + 13120 * 8 + 122880 + 16].view(np.uint32)
print('block 0 meta (nseq, nlit, rle):', m0[:3].tolist(), 'temp', temp.numel(), 'blocks off', blocks, 'n*WS', n * WS)
raw = np.array([h[blocks + b * WS + 13120 * 8 + 122880 + 16: blocks + b * WS + 13120 * 8 + 122880 + 16 + 60 * 4].view(np.uint32) for b in range(n)])
st = raw[:, :6]
k2 = raw[:, 6:15].astype(np.float64)
names = ["stage", "A(P wait)", "B(lengths)", "J(walk+list)", "E(records+lits)", "rounds"]
tot = st[:, :5].sum(1).mean()
print(kind, "mean cycles/block (s_memtime units)", int(tot))
for k, nm in enumerate(names):
    print(f"  {nm:16s} mean {st[:, k].mean():12.0f}  share {st[:, k].mean() / tot * 100 if k < 5 else 0:5.1f}%")
print(f"  inserter busy (next window) {raw[:, 16].mean():12.0f}   R wait {raw[:, 21].mean():12.0f}  list + W1 {raw[:, 22].mean():12.0f}  catch-up + W2 {raw[:, 20].mean():12.0f}")

print(f"  wave 0 parse: span tops {raw[:, 55].mean():10.0f}  walk+Jacobi {raw[:, 56].mean():10.0f}  list {raw[:, 57].mean():10.0f}  catch-up+records {raw[:, 3].mean():10.0f}")
k2 = np.concatenate([k2, raw[:, 17:18].astype(np.float64)], 1)
k2n = ["lit_hist", "huf_build(serial)", "stream_sizes", "lit_streams", "merge", "repcode+codes", "fse_tables(serial)", "fse_pack", "tail", "fse_chains"]
t2 = k2.sum(1).mean()
print(kind, "K2 mean cycles/block", int(t2))
for k, nm in enumerate(k2n):
    print(f"  {nm:20s} mean {k2[:, k].mean():12.0f}  share {k2[:, k].mean() / t2 * 100:5.1f}%")
print(f"  of huf_build: parallel tree {np.array([h[blocks + b * WS + 13120 * 8 + 122880 + 16 + 42 * 4: blocks + b * WS + 13120 * 8 + 122880 + 16 + 43 * 4].view(np.uint32)[0] for b in range(n)]).mean():.0f}")
print(f"  K3 per block: cycles mean {raw[:, 46].mean():.0f} max {raw[:, 46].max()}  Jacobi rounds mean {raw[:, 47].mean():.2f} max {raw[:, 47].max()}"
      f"  reruns mean {raw[:, 48].mean():.1f}  nbSeq mean {raw[:, 49].mean():.0f} p99 {np.percentile(raw[:, 49], 99):.0f} max {raw[:, 49].max()}")
print(f"  K3 staging+warm-up cycles mean {raw[:, 50].mean():.0f} max {raw[:, 50].max()}")
t0, t1 = raw[:, 51].astype(np.int64), raw[:, 52].astype(np.int64)
ok = (t1 >= t0) & (raw[:, 49] > 0)
if ok.any():
    base_t = t0[ok].min()
    ev = sorted([(int(a - base_t), 1) for a in t0[ok]] + [(int(b - base_t), -1) for b in t1[ok]])
    cur = peak = 0
    for _, d in ev:
        cur += d
        peak = max(peak, cur)
    span = (t1[ok].max() - base_t)
    print(f"  K3 span {span / 100:.1f} us (100 MHz ticks), peak concurrent waves {peak}, mean concurrent {(t1[ok] - t0[ok]).sum() / span:.0f}, mean wave {(t1[ok] - t0[ok]).mean() / 100:.1f} us")
    st_ = np.sort(t0[ok] - base_t)
    print("  K3 wave start times (us) at 10/50/90/100 %:", [round(float(st_[int(q * (len(st_) - 1))]) / 100, 1) for q in (0.1, 0.5, 0.9, 1.0)])
slow = np.argsort(raw[:, 46])[-5:]
wb = np.concatenate([raw[:, 28:40], raw[:, 53:55]], 1).astype(np.float64)
print("  K1 length-phase cycles per worker wave (mean over blocks, waves 0..13; SIMD = wave % 4):", [int(x) for x in wb.mean(0)])
print("  slowest K3 blocks (cycles, rounds, reruns, nbSeq):", [(int(raw[b, 46]), int(raw[b, 47]), int(raw[b, 48]), int(raw[b, 49])) for b in slow])
print(f"  of fse_chains: serial chain steps only {raw[:, 18].mean():.0f}  raw seqs mean {raw[:, 19].mean():.0f}")
# wall clock per block (s_memrealtime, 100 MHz) and placement
rt = np.array([h[blocks + b * WS + 13120 * 8 + 122880 + 16 + 23 * 4: blocks + b * WS + 13120 * 8 + 122880 + 16 + 28 * 4].view(np.uint32) for b in range(n)]).astype(np.int64)
dur = (rt[:, 1] - rt[:, 0]) & 0xFFFFFFFF
print(f"  block wall (realtime 100MHz ticks) mean {dur.mean():.0f} = {dur.mean() * 10:.0f} ns; memtime mean {rt[:, 4].mean():.0f} -> clock {rt[:, 4].mean() / (dur.mean() * 10):.2f} GHz")
cu = (rt[:, 3] & 0xFFFFFFFF).astype(np.int64) * 1000 + ((rt[:, 2] >> 8) & 0xF) + 16 * ((rt[:, 2] >> 12) & 0x1) + 32 * ((rt[:, 2] >> 13) & 0x7)
t0 = rt[:, 0].min(); t1 = (rt[:, 0] + dur).max()
print(f"  span {(t1 - t0) * 10 / 1e3:.1f} us, distinct CUs {len(set(cu.tolist()))}, blocks/CU max {np.bincount(np.unique(cu, return_inverse=True)[1]).max()}")
busy = {}
for c, d in zip(cu.tolist(), dur.tolist()):
    busy[c] = busy.get(c, 0) + d
print(f"  per-CU busy fraction of span: mean {np.mean(list(busy.values())) / (t1 - t0):.3f}")
mx = np.array([h[blocks + b * WS + 13120 * 8 + 122880 + 16 + 40 * 4: blocks + b * WS + 13120 * 8 + 122880 + 16 + 42 * 4].view(np.uint32) for b in range(n)])
if kind:
    print(f"  B-work max over worker waves {mx[:, 0].mean():.0f}   inserter busy max {mx[:, 1].mean():.0f}  (per block)")
try:
    import ctypes as _ct
    _L = _ct.CDLL(os.environ["CUDA_ZSTD_HIP_LIB"])
    _h = (_ct.c_uint32 * 6)()
    _L.zh_hst_host(_h)
    print("  Huffman build phases (cycles summed over blocks; since process start): sort %d merge %d depths %d max_height %d codes %d" % tuple(_h[:5]))
except Exception as _e:  # noqa: BLE001
    print("  (no Huffman phase stamps)", _e)
