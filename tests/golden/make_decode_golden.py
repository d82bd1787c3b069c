"""Generate tests/golden/decode_frames.json: libzstd 1.4.9 frames (the reference's own
CPU codec, src/cuda_zstd_manager.cu:1643-1645, 3277-3313) that exercise every part of
the decoder, with the SHA-256 of the bytes they decode to.

Inputs come from tools/datagen.c or seeded numpy builders; the fixture holds only the
frames, the decoded sizes and their SHA-256, so the tests need neither libzstd nor the
builders to check a decode.  One vector is the reference's own golden
frame, tests/test_fse_canonical.cu:20-24 (Huffman literals with FSE-compressed weights);
it is truncated (48 bytes of a frame whose block announces 211), so the expectation is
libzstd's: an error.

    python tests/golden/make_decode_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import zh_testlib as T  # noqa: E402

REF_CANONICAL = ("28b52ffd60f4009d0600869e3107f00d9999399f7b2e002e002e003f1a151d22554454020037c5446ca9322305"
                 "e180e2")

# (name, kind, seed, size, libzstd parameters)
CASES = [
    ("iota_1k_l1", "iota", 0, 1024, dict(level=1)),  # reference tests/test_rfc8878_integration.cu:236
    ("text_20k_l1", "text", 21, 20000, dict(level=1)),
    ("text_20k_l19", "text", 22, 20000, dict(level=19)),
    ("json_30k_l12_checksum", "json", 23, 30000, dict(level=12, checksum=True)),
    ("exe_10k_l3_nofcs", "exe", 24, 10000, dict(level=3, content_size=False)),
    ("sensor_50k_l5_window1k", "sensor", 25, 50000, dict(level=5, window_log=10)),
    ("csv_300k_l19_multiblock", "csv", 26, 300000, dict(level=19)),  # (csv compresses ~6x)
    ("source_200k_l7_multiblock_checksum", "source", 27, 200000, dict(level=7, checksum=True)),
    ("sym16_64k_l3", "sym16", 28, 65536, dict(level=3)),
    ("random_5k_l3", "random", 29, 5000, dict(level=3)),
    ("zeros_100k_l3", "zeros", 0, 100000, dict(level=3)),
    ("empty_l3", "zeros", 0, 0, dict(level=3)),
    # shapes found with tests/zh_frames.py to reach the remaining decoder paths
    ("zeros_then_rand_l3_rle_block", "rand_then_zeros", 1, 0, dict(level=3)),
    ("sym16_2k_l1_no_sequences", "sym16_small", 1, 2000, dict(level=1)),
    ("sym16_2k_l3_ml_rle", "sym16_small", 1, 2000, dict(level=3)),
    ("runs_l3_direct_weights", "runs_small", 1, 0, dict(level=3)),
    ("rows_l1_ll_of_rle_repeat", "rows", 2, 0, dict(level=1)),
    ("rows_l3_ml_rle_repeat", "rows", 2, 0, dict(level=3)),
    ("slices_l19_rle_literals", "slices_q", 3, 0, dict(level=19)),
    ("rows_l9_ml_repeat", "rows", 2, 0, dict(level=9)),
    ("json_300k_l9_treeless_ml_repeat", "json", 5, 300000, dict(level=9)),
]


def make_input(kind, seed, size):
    rng = np.random.default_rng(seed)
    if kind == "rand_then_zeros":
        return np.concatenate([np.zeros(262144, np.uint8), rng.integers(0, 256, 100, dtype=np.uint8)])
    if kind == "sym16_small":
        return rng.integers(0, 16, size, dtype=np.uint8) + 65
    if kind == "runs_small":
        return np.concatenate([np.full(rng.integers(1, 4), rng.integers(0, 8), np.uint8) for _ in range(3000)])
    if kind == "rows":  # 64-byte rows, each the previous one with one byte changed
        r, out = rng.integers(0, 256, 64, dtype=np.uint8), []
        for _ in range(5000):
            r = r.copy()
            r[rng.integers(0, 64)] = rng.integers(0, 256)
            out.append(r)
        return np.concatenate(out)
    if kind == "slices_q":  # a text block, then slices of it separated by 0x01 (literals all 0x01)
        base = T.gen(T.DG_TEXT, 1, seed, 131072)
        parts = [base]
        for _ in range(1500):
            s = rng.integers(0, 131072 - 80)
            parts += [base[s:s + rng.integers(20, 70)], np.array([1], np.uint8)]
        return np.concatenate(parts)
    if kind == "iota":
        return (np.arange(size) % 256).astype(np.uint8)
    if kind == "zeros":
        return np.zeros(size, np.uint8)
    return T.gen(T.KINDS[kind], 1, seed, size) if size else np.zeros(0, np.uint8)


def main():
    assert T.zstd() is not None, "needs libzstd"
    out = {"libzstd_version": int(T.zstd().ZSTD_versionNumber()), "vectors": []}
    # the reference's vector is the first 48 bytes of a frame whose block header announces
    # 211 bytes: libzstd rejects it ("Src size is incorrect"), and so must the decoder
    ref = bytes.fromhex(REF_CANONICAL)
    try:
        T.zstd_decompress(ref, 1 << 16)
        raise SystemExit("libzstd accepted the truncated reference vector")
    except AssertionError as e:
        err = str(e)
    out["vectors"].append({"name": "reference_test_fse_canonical_truncated", "source": "reference tests/test_fse_canonical.cu:20-24",
                           "frame": REF_CANONICAL, "expect_error": err})
    for name, kind, seed, size, kw in CASES:
        data = make_input(kind, seed, size)
        frame = T.zstd_compress(data, **kw)
        assert T.zstd_decompress(frame, max(len(data), 1)) == data.tobytes()
        out["vectors"].append({"name": name, "kind": kind, "seed": seed, "size": len(data), "params": kw, "frame": frame.hex(),
                               "sha256": hashlib.sha256(data.tobytes()).hexdigest()})
    with open(os.path.join(HERE, "decode_frames.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(sum(len(v["frame"]) // 2 for v in out["vectors"]), "frame bytes")


if __name__ == "__main__":
    main()
