"""Diagnostic (not a test): K1 literal masks seen by the literal phase (-DZH_K1_DEBUG build,
tools/libcuda_zstd_hip_dbg.so) vs the masks implied by the oracle's parse, for one chunk."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CUDA_ZSTD_HIP_LIB"] = os.path.join(ROOT, "tools", "libcuda_zstd_hip_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import zh_testlib as T
import test_gpu_k1 as K
kind, idx = sys.argv[1], int(sys.argv[2])
d = T.gen(T.KINDS[kind], 1, 0x5EED0003, 65536, first=idx)
(recs, lits, rle), = K.k1_raw([d])
area = K.k1_raw.area
dbg = area[65536:65536 + 16 * 64 * 16].view(np.uint32).reshape(16, 64, 4)
seqs, last = K.oracle_parse(d)
islit = np.zeros(65536, bool)
pos = 0
for ll, ml, _ in seqs:
    islit[pos:pos + ll] = True
    pos += ll + ml
islit[pos:pos + last] = True
nbad = 0
for w in range(16):
    for r in range(64):
        lm = int(dbg[w, r, 0]) | (int(dbg[w, r, 1]) << 32)
        base = 4096 * w + 64 * r
        exp = sum(1 << k for k in range(64) if islit[base + k])
        if lm != exp:
            nbad += 1
            if nbad <= 8:
                print(f"window {w} seg {r} (pos {base}): lm {lm:016x} expected {exp:016x} diff {lm ^ exp:016x} lbr {dbg[w, r, 2]} nlit_tot {dbg[w, r, 3]}")
print("bad segments", nbad)
