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
