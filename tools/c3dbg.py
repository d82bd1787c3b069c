import sys, os
sys.path.insert(0, 'custom-nvcomp-with-zstd_amd'); sys.path.insert(0, 'tests')
import torch, numpy as np, cuda_zstd, zh_testlib as T
n, cs = int(sys.argv[1]), 65536
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
data = T.gen(T.DG_MIX, n, 0x5EED0003, cs, first=first)
dev = torch.from_numpy(data).cuda()
bc = cuda_zstd.BatchedCompressor(3, cs)
slot = (bc.max_out(cs) + 255) // 256 * 256
comp = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
ar = torch.arange(n, dtype=torch.int64, device="cuda")
comp_ptrs = comp.data_ptr() + ar * slot
csizes = torch.zeros(n, dtype=torch.int64, device="cuda")
temp = torch.empty(bc.temp_size(n, cs), dtype=torch.uint8, device="cuda")
bc.compress_async(dev.data_ptr() + ar * cs, torch.full((n,), cs, dtype=torch.int64, device="cuda"), cs, comp_ptrs, csizes, None, temp)
torch.cuda.synchronize()
print("compressed", flush=True)
bd = cuda_zstd.BatchedDecompressor()
back = torch.zeros(n * cs, dtype=torch.uint8, device="cuda")
dsizes = torch.zeros(n, dtype=torch.int64, device="cuda")
status = torch.full((n,), -1, dtype=torch.int32, device="cuda")
dtemp = torch.empty(bd.temp_size(n, cs), dtype=torch.uint8, device="cuda")
bd.decompress_async(comp_ptrs, csizes, None, cs, back.data_ptr() + ar * cs, dsizes, status, dtemp)
torch.cuda.synchronize()
print("status ok", bool((status == 0).all()), "equal", torch.equal(back, dev), flush=True)
