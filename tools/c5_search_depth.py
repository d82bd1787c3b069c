"""C5 ratio sensitivity (CPU only, libzstd): how much of libzstd level 9's ratio on the C5
records (512 of the 4,096 x 16 KiB JSON-like records, seed 0x5EED0005) comes from its search
depth.  Prints the ratio for level 9, level 3 and strategies dfast/greedy/lazy/lazy2 at
searchLog 1, 2, 3, 5 (minMatch 4 and 5), without and with the 64 KiB ZDICT dictionary.
Numbers are quoted in DESIGN.md section 7."""
import ctypes, sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import zh_testlib as T
REC, N, SEED = 16384, 4096, 0x5EED0005
host = T.gen(T.DG_JSON, N, SEED, REC)
recs = [host[i*REC:(i+1)*REC] for i in range(N)]
train = recs[::4]
zd = T.zdict_train(train, 65536)
z = T.zstd(); vp = ctypes.c_void_p
z.ZSTD_createCCtx.restype = vp
z.ZSTD_CCtx_setParameter.argtypes = [vp, ctypes.c_int, ctypes.c_int]
z.ZSTD_CCtx_loadDictionary.argtypes = [vp, vp, ctypes.c_size_t]
z.ZSTD_compress2.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t]; z.ZSTD_compress2.restype = ctypes.c_size_t
z.ZSTD_CCtx_reset.argtypes = [vp, ctypes.c_int]
z.ZSTD_getDictID_fromDict.argtypes=[vp,ctypes.c_size_t]
z.ZSTD_getDictID_fromDict.restype=ctypes.c_uint
print("dict id", z.ZSTD_getDictID_fromDict(np.frombuffer(zd,np.uint8).ctypes.data, len(zd)), len(zd))
sub = recs[:512]
def run(d, params, level=9):
    c = z.ZSTD_createCCtx(); out = np.zeros(2*REC, np.uint8); tot = 0
    db = np.frombuffer(d, np.uint8).copy() if d else None
    for r in sub:
        z.ZSTD_CCtx_reset(c, 3)
        z.ZSTD_CCtx_setParameter(c, 100, level)
        for k, v in params.items(): z.ZSTD_CCtx_setParameter(c, k, v)
        if d: z.ZSTD_CCtx_loadDictionary(c, db.ctypes.data, len(d))
        s = z.ZSTD_compress2(c, out.ctypes.data, out.size, r.ctypes.data, r.size)
        assert not z.ZSTD_isError(s); tot += s
    return round(len(sub)*REC/tot, 3)
WL,HL,CL,SL,MM,TL,ST = 101,102,103,104,105,106,107
for name, d in (("none", None), ("zdict", zd)):
    print(name, "L9", run(d, {}), "L3", run(d, {}, 3))
    for st in (2,3,4,5):
        print(" strat", st, [run(d, {ST: st, SL: s, MM: mm}) for s in (1,2,3,5) for mm in (4,5)])
