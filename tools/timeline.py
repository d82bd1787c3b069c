"""Diagnostic: K1's window-pipeline timeline per wave (-DZH_TIMELINE build, e.g. tools/libV_tl.so from
`bash tools/variants.sh build tl -DZH_TIMELINE`): s_memtime cycles per step in each phase, averaged
over every step of every block of one C3-style batch.  Worker waves 0..13: P wait | lengths |
parse/records | X wait | span tops + literals; inserter waves 14 (long) / 15 (short): P wait |
insertion (X taken between tiles included) | literal rounds (ZH_LIT_INS) | barriers after them | dump.
usage: CUDA_ZSTD_HIP_LIB=tools/libV_tl.so python3 tools/timeline.py [LEVEL] [CHUNKS] [KIND]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cuda_zstd  # noqa: E402
import zh_testlib as T  # noqa: E402

level = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
kind = sys.argv[3] if len(sys.argv) > 3 else "mix"
cs = 65536
L = cuda_zstd.lib()
L.zh_timeline_host.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_uint64 * 128)()
data = T.gen(T.KINDS[kind], n, 0x5EED0003, cs)
dev = torch.from_numpy(data).cuda()
bc = cuda_zstd.BatchedCompressor(level, cs)
slot = (bc.max_out(cs) + 255) // 256 * 256
out = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
ar = torch.arange(n, dtype=torch.int64, device="cuda")
args = (dev.data_ptr() + ar * cs, torch.full((n,), cs, dtype=torch.int64, device="cuda"), cs, out.data_ptr() + ar * slot,
        torch.zeros(n, dtype=torch.int64, device="cuda"), torch.zeros(n, dtype=torch.int32, device="cuda"))
temp = torch.empty(bc.temp_size(n, cs), dtype=torch.uint8, device="cuda")
bc.compress_async(*args, temp)
torch.cuda.synchronize()
L.zh_timeline_host(buf)  # reset
bc.compress_async(*args, temp)
torch.cuda.synchronize()
assert L.zh_timeline_host(buf) == 0
a = np.array(buf[:], dtype=np.float64).reshape(16, 8)
names_w = ["P_wait", "lengths", "parse_rec", "X_wait", "lits"]
names_i = ["P_wait", "insert", "lits", "X_after", "dump"]
res = {"level": level, "chunks": n, "kind": kind, "waves": {}}
for w in range(16):
    steps = a[w, 5]
    if steps == 0:
        continue
    per = a[w, :5] / steps
    nm = names_i if w >= 14 else names_w
    res["waves"][w] = {nm[i]: round(per[i]) for i in range(5) if nm[i] != "-"}
    res["waves"][w]["step"] = round(per.sum())
print(json.dumps(res))
for w, v in res["waves"].items():
    print(f"wave {int(w):2d} (SIMD {int(w) % 4}):", "  ".join(f"{k} {x:6d}" for k, x in v.items()))
