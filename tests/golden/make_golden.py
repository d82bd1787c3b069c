"""Generates tests/golden/*.json from libzstd (the reference's CPU path and
third-party dependency; v1.4.9 at /opt/conda/lib/libzstd.so.1 in the build
container).  Fixtures are data (inputs + libzstd outputs); regenerate with
    python tests/golden/make_golden.py
The reference's own golden vectors (tests/test_fse_header.cu:57-66, 100-115,
tests/test_fse_encoding.cu:15-60) are written alongside."""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import zh_testlib as T  # noqa: E402

vp = ctypes.c_void_p
z = T.zstd()
assert z is not None
z.FSE_normalizeCount.restype = ctypes.c_size_t
z.FSE_writeNCount.restype = ctypes.c_size_t
z.HUF_buildCTable.restype = ctypes.c_size_t
z.HUF_writeCTable.restype = ctypes.c_size_t
z.FSE_optimalTableLog.restype = ctypes.c_uint
z.ZSTD_compressSequences.restype = ctypes.c_size_t
z.ZSTD_createCCtx.restype = vp
rng = np.random.default_rng(1234)


def is_err(r):
    return z.ZSTD_isError(ctypes.c_size_t(r)) != 0


def fse_cases(n=200):
    out = []
    for k in range(n):
        nsym = int(rng.integers(2, 53))
        if k % 4 == 0:
            counts = rng.integers(0, 3, nsym)
        elif k % 4 == 1:
            counts = (rng.zipf(1.5, nsym) * rng.integers(1, 50)).astype(np.int64)
        else:
            counts = rng.integers(0, 2000, nsym)
        counts = np.minimum(counts, 1 << 20).astype(np.uint32)
        counts[-1] = max(1, counts[-1])
        if counts.sum() < 2:
            counts[0] = 1
        total = int(counts.sum())
        maxsv = nsym - 1
        tl = int(z.FSE_optimalTableLog(ctypes.c_uint(9), ctypes.c_size_t(total), ctypes.c_uint(maxsv)))
        low = int(k % 3 != 0)
        norm = np.zeros(256, np.int16)
        c = np.ascontiguousarray(counts)
        r = z.FSE_normalizeCount(norm.ctypes.data_as(vp), ctypes.c_uint(tl), c.ctypes.data_as(vp), ctypes.c_size_t(total),
                                 ctypes.c_uint(maxsv), ctypes.c_uint(low))
        if is_err(r) or (counts == total).any():
            continue
        hdr = np.zeros(512, np.uint8)
        h = z.FSE_writeNCount(hdr.ctypes.data_as(vp), ctypes.c_size_t(512), norm.ctypes.data_as(vp), ctypes.c_uint(maxsv), ctypes.c_uint(tl))
        assert not is_err(h)
        out.append({"counts": counts.tolist(), "total": total, "maxsv": maxsv, "tablelog": tl, "lowprob": low,
                    "norm": norm[: maxsv + 1].tolist(), "ncount": bytes(hdr[:h]).hex()})
    return out


def huf_cases(n=150):
    out = []
    for k in range(n):
        nsym = int(rng.integers(2, 257))
        counts = np.minimum(rng.zipf(1.2 + 0.3 * (k % 5), nsym) * (1 + k % 7), 60000).astype(np.uint32)
        counts[rng.random(nsym) < 0.2] = 0
        counts[nsym - 1] = max(1, counts[nsym - 1])
        if (counts > 0).sum() < 2:
            counts[0] = 3
        maxsv = nsym - 1
        maxbits = 11
        ct = np.zeros(257 * 4, np.uint8)  # HUF_CElt {u16 val; u8 nbBits; pad}
        c = np.ascontiguousarray(counts)
        r = z.HUF_buildCTable(ct.ctypes.data_as(vp), c.ctypes.data_as(vp), ctypes.c_uint(maxsv), ctypes.c_uint(maxbits))
        if is_err(r):
            continue
        elts = ct.view(np.uint16).reshape(-1, 2)
        vals = elts[: maxsv + 1, 0].astype(int).tolist()
        nbs = (elts[: maxsv + 1, 1] & 0xFF).astype(int).tolist()
        hdr = np.zeros(512, np.uint8)
        h = z.HUF_writeCTable(hdr.ctypes.data_as(vp), ctypes.c_size_t(512), ct.ctypes.data_as(vp), ctypes.c_uint(maxsv), ctypes.c_uint(r))
        out.append({"counts": counts.tolist(), "maxsv": maxsv, "maxbits": maxbits, "huflog": int(r), "val": vals, "nbits": nbs,
                    "header": bytes(hdr[:h]).hex() if not is_err(h) else None})
    return out


class ZS(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint), ("litLength", ctypes.c_uint), ("matchLength", ctypes.c_uint), ("rep", ctypes.c_uint)]


def _block_case(o, cc, name, src, full):
    size = len(src)
    seqbuf = np.zeros((size // 5 + 2, 3), np.uint32)
    last = ctypes.c_uint32()
    ns = o.orc_lz_parse(src.ctypes.data_as(vp), ctypes.c_uint32(size), seqbuf.ctypes.data_as(vp), ctypes.byref(last))
    zs = (ZS * max(ns, 1))()
    for k in range(ns):
        zs[k].offset, zs[k].litLength, zs[k].matchLength = int(seqbuf[k, 2]), int(seqbuf[k, 0]), int(seqbuf[k, 1])
    z.ZSTD_CCtx_reset(vp(cc), 3)
    z.ZSTD_CCtx_setParameter(vp(cc), 100, 3)
    z.ZSTD_CCtx_setParameter(vp(cc), 1011, 0)
    buf = np.zeros(size * 2 + 512, np.uint8)
    r = z.ZSTD_compressSequences(vp(cc), buf.ctypes.data_as(vp), ctypes.c_size_t(len(buf)), zs, ctypes.c_size_t(ns),
                                 src.ctypes.data_as(vp), ctypes.c_size_t(size))
    assert not is_err(r)
    fr = bytes(buf[:r])
    fhd = fr[4]
    hs = 5 + (0 if (fhd >> 5) & 1 else 1) + [0, 1, 2, 4][fhd & 3] + [1 if (fhd >> 5) & 1 else 0, 2, 4, 8][fhd >> 6]
    c = {"name": name, "last_literals": last.value, "libzstd_block": fr[hs:].hex()}
    if full:  # 64 KiB: the input is regenerated from its generator, the parse pinned by its digest
        import hashlib
        c["nseq"] = int(ns)
        c["sequences_sha256"] = hashlib.sha256(seqbuf[:ns].astype("<u4").tobytes()).hexdigest()
    else:
        c["input"] = src.tobytes().hex()
        c["sequences"] = seqbuf[:ns].tolist()
    return c


def block_cases():
    """libzstd ZSTD_compressSequences (noBlockDelimiters) on the oracle's own parse:
    pins the oracle's entropy stage byte-for-byte.  Small inputs (<= 8 KiB) carry their
    bytes; the 64 KiB blocks of the metric's chunk size (4-stream Huffman, FSE-compressed
    weights, large-nbSeq FSE tables) are named by their tools/datagen.c generator."""
    o = T.oracle()
    cc = z.ZSTD_createCCtx()
    out = []
    for name, kind, size, seed in [("text", T.DG_TEXT, 8192, 1), ("csv", T.DG_CSV, 6000, 2), ("json", T.DG_JSON, 8192, 3),
                                   ("exe", T.DG_EXE, 5000, 4), ("sensor", T.DG_SENSOR, 8192, 5), ("source", T.DG_SOURCE, 7000, 6),
                                   ("sym16", T.DG_SYM16, 4096, 7), ("text_small", T.DG_TEXT, 700, 8),
                                   ("sym16_seq", T.DG_SYM16, 4096, 10)]:  # (sym16 seed 7: no match in the probe window)
        out.append(_block_case(o, cc, name, T.gen(kind, 1, seed, size), False))
    for kname in ("mix", "text", "exe", "sensor", "json", "csv", "source", "sym16"):
        for first in (0, 5):
            c = _block_case(o, cc, f"{kname}_64k_{first}", T.gen(T.KINDS[kname], 1, 0x5EED0003, 65536, first=first), True)
            c["gen"] = {"kind": kname, "seed": 0x5EED0003, "size": 65536, "first": first}
            out.append(c)
    return out


def main():
    ver = int(z.ZSTD_versionNumber())
    only = sys.argv[1:]  # e.g. "blocks": regenerate only the entropy-block fixtures (they follow the LZ parameters)
    if not only or "fse" in only:
        json.dump({"libzstd_version": ver, "cases": fse_cases()}, open(os.path.join(HERE, "fse_normalize_ncount.json"), "w"))
    if not only or "huf" in only:
        json.dump({"libzstd_version": ver, "cases": huf_cases()}, open(os.path.join(HERE, "huf_ctable.json"), "w"))
    if not only or "blocks" in only:
        json.dump({"libzstd_version": ver, "cases": block_cases()}, open(os.path.join(HERE, "entropy_blocks.json"), "w"))
    ref = {
        "source": "reference tests/test_fse_header.cu:57-66,100-115; tests/test_fse_encoding.cu:15-60; tests/test_compressible_data.cu:272,311,325,363",
        "ncount": [{"norm": [16, 16], "maxsv": 1, "tablelog": 5, "bytes": "103f"},
                   {"norm": [-1, 31], "maxsv": 1, "tablelog": 5, "bytes": "007e"}],
        "ctable_delta_nbbits": {"norm": [1, 1, 1, 1], "tablelog": 2, "deltaNbBits": 131068},
        "ratio_floors_64k": {"json": 1.3, "period8": 1.5, "zeros": 10.0, "ff": 500.0},
    }
    json.dump(ref, open(os.path.join(HERE, "reference_vectors.json"), "w"), indent=1)
    print("golden fixtures written; libzstd", ver)


if __name__ == "__main__":
    main()
