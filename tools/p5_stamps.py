"""Diagnostic: per-part cycle breakdown of the split pipeline's phase 5 (zh_decode_kernel) (s_memtime, lane 0 of each
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
# phase 5 (split pipeline, -DZH_STAMPS): the deferred items' record spare bytes at ho_off + 5248
ho_off = lit_bytes + a256(seq_cap * 8)
x = np.stack([host[base + i * slot_bytes + ho_off + 5248: base + i * slot_bytes + ho_off + 5248 + 48].view(np.uint64) for i in range(n)]).astype(np.float64)
names = ["frame header", "literals header", "Huffman weights", "Huffman table", "streams"]
tot = x[:, :5].sum(1)
print(f"{kind}: {n} items, decode {e0.elapsed_time(e1):.2f} ms; phase 5 per deferred item {tot.mean():.0f} cycles, literals {x[:, 5].mean():.0f} bytes")
for k, nm in enumerate(names):
    print(f"  {nm:16s} {x[:, k].mean():12.0f}  {100 * x[:, k].sum() / tot.sum():5.1f} %")
