"""Dictionaries, CPU side: the oracle's dictionary frames decode with stock
libzstd (ZSTD_decompress_usingDict) for raw-content and formatted (ZDICT) dictionaries and name
the dictionary by its RFC Dictionary_ID; the C ABI's dictionary parser agrees with the oracle's;
the COVER trainer (replacing the reference's n-gram trainer, src/cuda_zstd_dictionary.cu:179-415)
is deterministic and helps the ratio.  GPU parity is tests/test_gpu_dict.py."""
import pytest

import zh_frames
import zh_testlib as T

pytestmark = pytest.mark.skipif(T.zstd() is None, reason="libzstd absent")

SIZES = [1, 7, 100, 4095, 16384, 50000, 65536, 70000, 200000]


def _split(a, size):
    return [a[i:i + size] for i in range(0, len(a), size)]


@pytest.fixture(scope="module")
def samples():
    return _split(T.gen(T.DG_JSON, 512, 0x5EED0005, 4096), 4096)


@pytest.fixture(scope="module")
def zdict(samples):
    return T.zdict_train(samples, 16384)


@pytest.fixture(scope="module")
def cover(samples):
    import cuda_zstd

    return cuda_zstd.Dictionary.train(samples, 16384).content()


def capi_layout(buf):
    import cuda_zstd

    try:
        return cuda_zstd.Dictionary.load(buf).layout()
    except cuda_zstd.ZstdError:
        return None


def test_dict_layouts(zdict, cover):
    lz = T.dict_layout(zdict)
    assert lz is not None and lz[0] != 0 and 8 < lz[1] < len(zdict)
    assert T.dict_layout(cover) == (0, 0)  # raw content
    cut = zdict[:lz[1] - 13]  # ends inside the repcodes
    bad_rep = bytearray(zdict)
    bad_rep[lz[1] - 12:lz[1] - 8] = b"\0\0\0\0"  # repcode 0 (libzstd: dictionary_corrupted)
    for b in (cut, bytes(bad_rep)):
        assert T.dict_layout(b) is None and capi_layout(b) is None
    assert capi_layout(zdict) == lz and capi_layout(cover) == (0, 0)


@pytest.mark.parametrize("kind", ["zdict", "cover"])
def test_oracle_dict_frames_decode_with_libzstd(kind, zdict, cover):
    d = zdict if kind == "zdict" else cover
    did = T.dict_layout(d)[0]
    src = T.gen(T.DG_JSON, 1, 0x5EED0105, 200000)
    for n in SIZES:
        data = src[:n]
        for ck in (False, True):
            f = T.oracle_frame(data, checksum=ck, dictionary=d)
            assert zh_frames.walk(f)[0]["dict_id"] == did
            assert T.zstd_decompress(f, n, dictionary=d) == data.tobytes(), (kind, n, ck)


@pytest.mark.parametrize("kind", ["zdict", "cover"])
def test_dictionary_improves_ratio(kind, zdict, cover):
    d = zdict if kind == "zdict" else cover
    held = _split(T.gen(T.DG_JSON, 64, 0x5EED0205, 4096), 4096)
    plain = sum(len(T.oracle_frame(r)) for r in held)
    with_d = sum(len(T.oracle_frame(r, dictionary=d)) for r in held)
    assert with_d < 0.85 * plain, (with_d, plain)


def test_cover_trainer(samples, cover):
    import cuda_zstd

    assert cuda_zstd.Dictionary.train(samples, 16384).content() == cover  # deterministic
    assert 0 < len(cover) <= 16384
    corpus = b"".join(s.tobytes() for s in samples)
    probes = list(range(0, len(cover) - 32, 251))
    assert sum(cover[o:o + 32] in corpus for o in probes) >= 0.9 * len(probes)  # segments of the samples


def test_dictionary_handle_bytes(zdict, cover):
    import cuda_zstd

    for d in (zdict, cover):
        assert cuda_zstd.Dictionary.load(d).content() == d


def test_deep_matcher_sees_whole_64k_dictionary():
    """Levels >= 9 (the deep matcher) stage the whole last 64 KiB of the dictionary content in front
    of a record's first block (ZH_DEEP_PRE; VERDICT r2 missing #2): a 16 KiB record made of bytes
    from the dictionary's FIRST 8 KiB -- outside the 64 KiB - 16 KiB tail that level 3's K1 stages
    -- compresses to almost nothing at level 9 and not at level 3; both decode with libzstd."""
    import numpy as np

    d = T.gen(T.DG_RANDOM, 1, 0x5EED0901, 65536).tobytes()
    a = np.frombuffer(d, dtype=np.uint8)
    rec = np.concatenate([a[100:8292], a[200:8392]])
    assert len(rec) == 16384
    f9 = T.oracle_frame(rec, dictionary=d, level=9)
    f3 = T.oracle_frame(rec, dictionary=d, level=3)
    for f in (f9, f3):
        assert T.zstd_decompress(f, len(rec), dictionary=d) == rec.tobytes()
    assert len(f9) < 200 and len(f3) > 8000, (len(f9), len(f3))


@pytest.mark.parametrize("kind", ["zdict", "cover"])
def test_dictionary_helps_large_records_level3(kind, zdict, cover):
    """Level 3 dictionary frames over 32 KiB are cut into 32 KiB blocks (ZH_FRAME_BLOCK
    split_dict; advisor r3): the first block is staged behind 32 KiB of the dictionary instead of
    64 KiB - n, so 48-64 KiB records still gain from the dictionary (a 64 KiB record used to see
    none of it).  Measured on records whose content comes from the dictionary's sample corpus."""
    d = zdict if kind == "zdict" else cover
    for n in (49152, 61440, 65536):
        recs = [T.gen(T.DG_JSON, 1, 0x5EED0305, n, first=i) for i in range(4)]
        plain = sum(len(T.oracle_frame(r)) for r in recs)
        with_d = sum(len(T.oracle_frame(r, dictionary=d)) for r in recs)
        assert with_d < 0.97 * plain, (n, with_d, plain)
        for r in recs:
            f = T.oracle_frame(r, dictionary=d)
            assert len(zh_frames.walk(f)) == 2  # two 32 KiB blocks
            assert T.zstd_decompress(f, n, dictionary=d) == r.tobytes()
