"""Diagnostic: per-phase cycle breakdown of zh_dec_exec_kernel (phase 3) (s_memtime, lane 0 of each
item) from the -DZH_STAMPS build (tools/libcuda_zstd_hip_stamps.so).  Not a benchmark.
Phases: 0 frame/raw blocks, 1 literals (Huffman), 2 sequence tables, 3 sequence
bitstream, 4 execution, 5 tail."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CUDA_ZSTD_HIP_LIB"] = os.path.join(ROOT, "tools", "libcuda_zstd_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

import cuda_zstd
import zh_testlib as T

kind = sys.argv[1] if len(sys.argv) > 1 else "mix"
n, cs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096, 65536
data = T.gen(T.KINDS[kind], n, 0x5EED0003, cs)
dev = torch.from_numpy(data).cuda()
bc = cuda_zstd.BatchedCompressor(3, cs)
slot = (bc.max_out(cs) + 255) // 256 * 256
comp = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
ar = torch.arange(n, dtype=torch.int64, device="cuda")
sizes = torch.full((n,), cs, dtype=torch.int64, device="cuda")
csz = torch.zeros(n, dtype=torch.int64, device="cuda")
temp = torch.empty(bc.temp_size(n, cs), dtype=torch.uint8, device="cuda")
bc.compress_async(dev.data_ptr() + ar * cs, sizes, cs, comp.data_ptr() + ar * slot, csz, None, temp)
bd = cuda_zstd.BatchedDecompressor()
back = torch.empty(n * cs, dtype=torch.uint8, device="cuda")
dsz = torch.zeros(n, dtype=torch.int64, device="cuda")
st = torch.zeros(n, dtype=torch.int32, device="cuda")
dtemp = torch.empty(bd.temp_size(n, cs), dtype=torch.uint8, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
bd.decompress_async(comp.data_ptr() + ar * slot, csz, None, cs, back.data_ptr() + ar * cs, dsz, st, dtemp)
e1.record()
torch.cuda.synchronize()
assert torch.equal(back, dev) and (st == 0).all()
# slot layout of DecLayout::make(n, cs) (csrc/zh_host.cpp)
a256 = lambda v: (v + 255) // 256 * 256
block_cap = min(max(cs, 64), 128 * 1024)
lit_bytes = a256(block_cap + 64)
seq_cap = block_cap // 3 + 2
slot_bytes = lit_bytes + a256(seq_cap * 8) + a256(5376)  # + hand-off record (ZH_DEC_HANDOFF_BYTES)
off = 0
for k in (8, 8, 8, 8, 8, 4):
    off = a256(off + n * k)
base = a256(dtemp.data_ptr()) - dtemp.data_ptr() + off
host = dtemp.cpu().numpy()
stv = np.stack([host[base + i * slot_bytes: base + i * slot_bytes + 64].view(np.uint64) for i in range(n)]).astype(np.float64)
# zh_dec_exec_kernel (-DZH_STAMPS): [0] cycles, [1] windows, [2] records + scan, [3] pass A,
# [4] pass B, [5] flush, [6] sequences, [7] bytes
x = stv
print(f"{kind}: {n} items, decode {e0.elapsed_time(e1):.2f} ms; exec kernel per item: cycles {x[:, 0].mean():.0f}, windows {x[:, 1].mean():.1f}, "
      f"sequences {x[:, 6].mean():.0f}, bytes {x[:, 7].mean():.0f}")
for k, nm in ((2, "records+scan"), (3, "pass A"), (4, "pass B"), (5, "flush+fence")):
    print(f"  {nm:14s} {x[:, k].mean():12.0f}  {100 * x[:, k].sum() / x[:, 0].sum():5.1f} %   per window {x[:, k].sum() / x[:, 1].sum():8.0f}")
