"""Debug: which inputs differ between the GPU LAZY2 parse and the oracle (level 9)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "custom-nvcomp-with-zstd_amd"))
import numpy as np, torch
import zh_testlib as T, cuda_zstd
m = cuda_zstd.Manager(9)
for kind in sorted(T.KINDS):
    for size in (65536, 32769, 100000, 300000):
        d = T.gen(T.KINDS[kind], 1, 44, size)
        got = m.compress(torch.from_numpy(d).cuda()).cpu().numpy().tobytes()
        want = T.oracle_frame(d, level=9)
        if got != want:
            # first differing byte and block structure
            k = next(i for i in range(min(len(got), len(want))) if got[i] != want[i]) if min(len(got), len(want)) else 0
            print(f"DIFF {kind} {size}: gpu {len(got)} oracle {len(want)} first diff at {k}", flush=True)
        else:
            print(f"ok {kind} {size}", flush=True)
