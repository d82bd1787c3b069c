"""Diagnostic (-DZH_STAMPS build): how often the inserters' read-back finds a lane of one
ds_write_b16 that lost its slot to a lower position (fix-up rounds over a batch)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CUDA_ZSTD_HIP_LIB"] = os.path.join(ROOT, "tools", "libcuda_zstd_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch, cuda_zstd, zh_testlib as T
L = cuda_zstd.lib()
L.zh_fixups_host.restype = __import__("ctypes").c_uint
L.zh_fixups_host()
for kind in ("mix", "random", "text", "sym16"):
    n = 1024
    d = torch.from_numpy(T.gen(T.KINDS[kind], n, 0x5EED0003)).cuda()
    m = cuda_zstd.Manager(3)
    m.compress_batch([d[i * 65536:(i + 1) * 65536] for i in range(n)])
    torch.cuda.synchronize()
    f = L.zh_fixups_host()
    print(f"{kind}: {f} fix-up rounds over {n} blocks ({n * 512 * 2 * 2} inserter tile-stores)", flush=True)
