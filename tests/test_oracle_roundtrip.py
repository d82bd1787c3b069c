"""Oracle frames decode with stock libzstd to the original bytes; ratio floors of
the reference's tests/test_compressible_data.cu hold."""
import json
import os

import numpy as np
import pytest

import zh_testlib as T


@pytest.mark.parametrize("name", sorted(T.special_inputs().keys()))
def test_special_inputs_roundtrip(libzstd, name):
    data = T.special_inputs()[name]
    fr = T.oracle_frame(data)
    assert T.zstd_decompress(fr, len(data)) == data.tobytes()


@pytest.mark.parametrize("kind", sorted(T.KINDS))
def test_corpora_roundtrip(libzstd, kind):
    data = T.gen(T.KINDS[kind], 6, 0x5EED0003)
    for i in range(6):
        c = data[i * 65536:(i + 1) * 65536]
        assert T.zstd_decompress(T.oracle_frame(c), 65536) == c.tobytes()


def test_multiblock_frame_roundtrip(libzstd):
    # > 64 KiB: several device blocks in one frame, later blocks start with unknown repcodes
    data = np.concatenate([T.gen(T.DG_TEXT, 3, 5, 65536), T.gen(T.DG_CSV, 1, 6, 50000), T.gen(T.DG_RANDOM, 1, 7, 9000)])
    for bs in (128 * 1024, 1 << 20):
        fr = T.oracle_frame(data, block_size=bs)
        assert T.zstd_decompress(fr, len(data)) == data.tobytes()


def test_reference_ratio_floors():
    floors = json.load(open(os.path.join(T.GOLDEN, "reference_vectors.json")))["ratio_floors_64k"]
    s = T.special_inputs()
    json_chunk = T.gen(T.DG_JSON, 1, 3, 65536)
    for name, data in (("json", json_chunk), ("period8", s["period8_64k"]), ("zeros", s["zeros_64k"]), ("ff", s["ff_64k"])):
        assert len(data) / len(T.oracle_frame(data)) > floors[name], name


def test_ratio_vs_libzstd_level3(libzstd):
    """Not a parity bar (the parse is a deterministic GPU design), but track it:
    on the Silesia-like mix the oracle is within 10% of libzstd -3."""
    import ctypes
    data = T.gen(T.DG_MIX, 32, 0x5EED0003)
    ours = sum(len(T.oracle_frame(data[i * 65536:(i + 1) * 65536])) for i in range(32))
    out = np.zeros(80000, np.uint8)
    ref = 0
    for i in range(32):
        src = np.ascontiguousarray(data[i * 65536:(i + 1) * 65536])
        ref += libzstd.ZSTD_compress(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(80000), src.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(65536), 3)
    assert ref / ours > 0.90


def test_level1_stride_ratio_and_roundtrip(libzstd):
    """Level 1 looks matches up at every ZH_L1_STRIDE-th position (K1 mode 2):
    its frames decode with libzstd, and on the C3 mix it stays within 2 % of libzstd level 1 on the
    same chunks while level 3 stays at or above libzstd level 3 (oracle on 128 chunks: ~2.50 vs
    libzstd L1 ~2.53, level 3 ~2.80 vs ~2.79)."""
    n = 128
    data = T.gen(T.DG_MIX, n, 0x5EED0003)
    chunks = [data[i * 65536:(i + 1) * 65536] for i in range(n)]
    f1 = [T.oracle_frame(c, level=1) for c in chunks]
    for c, f in zip(chunks[:16], f1[:16]):
        assert T.zstd_decompress(f, len(c)) == c.tobytes()
    ours1 = sum(len(f) for f in f1)
    ours3 = sum(len(T.oracle_frame(c, level=3)) for c in chunks)
    ref1 = sum(len(T.zstd_compress(c.tobytes(), 1)) for c in chunks)
    ref3 = sum(len(T.zstd_compress(c.tobytes(), 3)) for c in chunks)
    assert ref1 / ours1 > 0.98, (ref1, ours1)
    assert ref3 / ours3 >= 1.0, (ref3, ours3)
    assert ours1 > ours3  # level 1 trades ratio for speed


def test_lazy2_parse_roundtrip_and_gain(libzstd):
    """Level >= 9 (LAZY2 parse): frames decode with libzstd and the parse gains on JSON records."""
    data = T.gen(T.DG_JSON, 8, 0x5EED0005, 16384)
    l3 = l9 = 0
    for i in range(8):
        c = data[i * 16384:(i + 1) * 16384]
        f9 = T.oracle_frame(c, level=9)
        assert T.zstd_decompress(f9, len(c)) == c.tobytes()
        l9 += len(f9)
        l3 += len(T.oracle_frame(c))
    assert l9 < l3


def _prefixed(kind, pre, seed):
    rng = np.random.default_rng(seed)
    c = T.gen(T.KINDS[kind], 1, 200 + seed, 65536).copy()
    c[:pre] = rng.integers(0, 256, pre, dtype=np.uint8)
    return c


@pytest.mark.parametrize("kind", ["text", "json", "mix"])
def test_random_prefix_ratio_vs_libzstd(libzstd, kind):
    """64 KiB chunks whose first 1-8 KiB are random (the incompressibility
    probe used to leave them literal-only: JSON with a 2 KiB prefix 1.55 vs libzstd L3 5.39).  The
    repeat scan resurrects them and the miss skip resumes at the first matching tiles: every chunk
    within 5 % of libzstd level 3 (the GPU frames equal these, tests/test_gpu_probe.py)."""
    for pre in (1024, 2048, 4096, 8192):
        for i in range(2):
            c = _prefixed(kind, pre, 31 * i + pre)
            f = T.oracle_frame(c)
            assert T.zstd_decompress(f, len(c)) == c.tobytes()
            z = len(T.zstd_compress(c, 3))
            assert len(f) * 0.95 <= z, (kind, pre, i, len(f), z)


def test_repeat_scan_restatement():
    """orc_repeat_scan against a direct Python statement of ZH_SCAN_* (include/zstd_hip_params.h)
    on small buffers: random (no repeats), a copied stretch, a dictionary-like prefix."""
    import ctypes
    O = T.oracle()
    O.orc_repeat_scan.restype = ctypes.c_uint32
    O.orc_repeat_scan.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    m24 = lambda a, b: ((a & 0xFFFFFF) * (b & 0xFFFFFF)) & 0xFFFFFFFF

    def ssum(v):
        return (m24(v, 0x9E3779) + m24(v >> 24, 0x85EBCA) + m24(v >> 48, 0xC2B2AE)) & 0xFFFFFFFF

    def py_scan(b, pre):
        n = len(b)
        lim = n - 8 if n > 8 else 0
        E = {}
        for q in range(0, lim, 4):
            t = ssum(int.from_bytes(b[q:q + 8], "little"))
            e = ((t << 14) & 0xFFFF0000) | q
            s = t >> 18
            E[s] = min(E.get(s, 0xFFFFFFFF), e)
        c = 0
        for p in range(pre, lim, 3):
            t = ssum(int.from_bytes(b[p:p + 8], "little"))
            x = (E.get(t >> 18, 0xFFFFFFFF) - ((t << 14) & 0xFFFF0000)) & 0xFFFFFFFF
            c += x < p
        return c

    rng = np.random.default_rng(3)
    r = rng.integers(0, 256, 12000, dtype=np.uint8)
    cp = r.copy()
    cp[7000:9000] = cp[1001:3001]
    txt = T.gen(T.DG_TEXT, 1, 9, 9000)
    for b, pre in ((r, 0), (cp, 0), (cp, 5000), (txt, 0), (txt, 4321)):
        b = np.ascontiguousarray(b)
        assert O.orc_repeat_scan(b.ctypes.data, pre, len(b)) == py_scan(b.tobytes(), pre)
    assert py_scan(r.tobytes(), 0) == 0 and py_scan(cp.tobytes(), 0) > 100


def test_dictionary_unaligned_history_no_cliff(libzstd):
    """one byte of dictionary size moved the probe window to a single block position and
    made a 16 KiB JSON record with 4 random leading bytes 4.4x larger (10,071 vs 2,300 B)."""
    rng = np.random.default_rng(23)
    rec = T.gen(T.DG_JSON, 1, 0x5EED0105, 16384).copy()
    rec[:4] = rng.integers(0, 256, 4, dtype=np.uint8)
    content = T.gen(T.DG_JSON, 1, 0x5EED0106, 40000)
    sizes = []
    for dn in (32767, 32768):
        dct = content[:dn].tobytes()
        f = T.oracle_frame(rec, dictionary=dct)
        assert T.zstd_decompress(f, len(rec), dictionary=dct) == rec.tobytes()
        sizes.append(len(f))
    assert max(sizes) <= 1.1 * min(sizes), sizes
