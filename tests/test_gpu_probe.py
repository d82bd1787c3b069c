"""The incompressibility probe without its ratio cliff: a block the
probe finds no match in is literal-only only when the repeat scan (ZH_SCAN_*, oracle
orc_repeat_scan) also finds no repeated 8-byte strings; otherwise K1 redoes the block without the
probe.  A miss-skip window whose first tiles find a match is searched whole.  GPU == oracle on the
same inputs (K1's records and literals, and whole frames), frames decode with libzstd, and chunks
with a random prefix compress within 5 % of libzstd level 3 (the reference's route for 64 KiB
chunks is ZSTD_compress, src/cuda_zstd_manager.cu:1604-1645)."""
import numpy as np
import pytest

import zh_testlib as T
from test_gpu_k1 import BLOCK, K1HIST, _compare, k1_raw, oracle_parse

pytestmark = pytest.mark.gpu

W = 2048
PREFIXES = (1024, 2048, 3000, 4096, 6144, 8192)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def _prefixed(kind, pre, seed):
    rng = np.random.default_rng(seed)
    c = T.gen(T.KINDS[kind], 1, 200 + seed, BLOCK).copy()
    c[:pre] = rng.integers(0, 256, pre, dtype=np.uint8)
    return c


def test_k1_resurrected_blocks_vs_oracle():
    """Blocks the probe ends that the scan resurrects (random prefixes over text / JSON / mix, a
    repeated random pattern), blocks that stay literal-only (random, 16 symbols, a random block with
    a few repeats), and short / ragged ones."""
    rng = np.random.default_rng(21)
    rnd = rng.integers(0, 256, BLOCK, dtype=np.uint8)
    datas, names = [], []

    def add(nm, d):
        names.append(nm)
        datas.append(np.ascontiguousarray(d, dtype=np.uint8))

    for kind in ("text", "json", "mix"):
        for pre in (W, 3000, 8192, 30000):
            add(f"{kind}+rand{pre}", _prefixed(kind, pre, pre))
    add("rand_period4096", np.tile(rnd[:4096], 16))
    add("rand_period3000", np.tile(rnd[:3000], 22)[:BLOCK])
    few = rnd.copy()
    few[50000:50040] = few[10000:10040]  # 32 repeated positions: below the scan's threshold
    add("rand_few_repeats", few)
    add("random", rnd)
    add("sym16", T.gen(T.DG_SYM16, 1, 7, BLOCK))
    add("json+rand_ragged", _prefixed("json", 2500, 3)[:40001])
    add("rand_then_copy_5000", np.concatenate([rnd[:2 * W + 8], rnd[:5000]])[:BLOCK])
    _compare(datas, names)
    got = k1_raw(datas)
    state = {nm: rle for (_, _, rle), nm in zip(got, names)}
    for nm in ("random", "rand_few_repeats"):
        assert state[nm] == K1HIST, f"{nm}: expected the literal-only block"
    for nm in ("json+rand3000", "text+rand8192", "mix+rand2048", "rand_period4096"):
        assert state[nm] != K1HIST, f"{nm}: expected the scan to resurrect the block"


def test_k1_miss_skip_resume_vs_oracle():
    """Miss-skip windows (after a window without matches) search their first ZH_SKIP_TILES tiles; a
    match among them resumes the whole window.  Text opens the block (no probe), random follows, and
    a copy of an earlier stretch lands in the first tiles of a skip window (at its first position,
    the last one of the searched tiles, just past them) or text resumes there."""
    rng = np.random.default_rng(22)
    text = T.gen(T.DG_TEXT, 1, 0x5EED0029, BLOCK)
    rnd = rng.integers(0, 256, BLOCK, dtype=np.uint8)
    datas, names = [], []
    for win in (8, 13):
        base = win * W
        for at, ln in ((0, 16), (128, 8), (250, 16), (255, 9), (256, 16), (300, 40)):
            d = np.concatenate([text[:2 * W], rnd[2 * W:]]).copy()
            src = base + 10 if at >= 128 else base - 3 * W + 10  # an earlier searched tile
            d[base + at:base + at + ln] = d[src:src + ln]
            names.append(f"w{win}@{at}+{ln}")
            datas.append(d)
        d = np.concatenate([text[:2 * W], rnd[2 * W:base + 100], text[2 * W:]])[:BLOCK].copy()
        names.append(f"w{win}text@100")
        datas.append(d)
    _compare(datas, names)
    # the resume actually happened somewhere: a match inside a window after the first skip window
    hits = 0
    for d in datas:
        seqs, _ = oracle_parse(d)
        pos = 0
        for ll, ml, _o in seqs:
            pos += ll
            hits += pos >= 8 * W and (pos % W) >= 2 * 128
            pos += ml
    assert hits > 0


@pytest.mark.parametrize("kind", ["text", "json", "mix"])
def test_prefix_chunks_ratio_vs_libzstd(torch_cuda, libzstd, kind):
    """64 KiB chunks with 1-8 KiB random prefixes (an embedded compressed or encrypted header):
    every GPU frame equals the oracle's, decodes with libzstd, and is at most 1 / 0.95 of
    libzstd level 3's frame for that chunk."""
    import cuda_zstd

    datas = [_prefixed(kind, pre, 31 * i + pre) for pre in PREFIXES for i in range(4)]
    outs = cuda_zstd.Manager(3).compress_batch([torch_cuda.from_numpy(d.copy()).cuda() for d in datas])
    for k, (o, d) in enumerate(zip(outs, datas)):
        got = o.cpu().numpy().tobytes()
        assert got == T.oracle_frame(d), f"chunk {k}: GPU frame != oracle"
        assert T.zstd_decompress(got, len(d)) == d.tobytes()
        z = len(T.zstd_compress(d, 3))
        assert len(got) * 0.95 <= z, f"chunk {k} (prefix {PREFIXES[k // 4]}): {len(got)} B vs libzstd L3 {z} B"


def test_dictionary_unaligned_history_no_cliff(torch_cuda):
    """a 16 KiB JSON record with 4 random leading bytes and a raw dictionary of
    32,767 / 32,768 bytes -- the probe window held one block position for the odd size.  Frames equal
    the oracle's and the two sizes are within 10 % of each other."""
    import cuda_zstd

    rng = np.random.default_rng(23)
    rec = T.gen(T.DG_JSON, 1, 0x5EED0105, 16384).copy()
    rec[:4] = rng.integers(0, 256, 4, dtype=np.uint8)
    content = T.gen(T.DG_JSON, 1, 0x5EED0106, 40000)
    sizes = []
    for dn in (32767, 32768, 20001):
        dct = content[:dn].tobytes()
        m = cuda_zstd.Manager(3)
        m.set_dictionary(cuda_zstd.Dictionary.load(dct))
        f = m.compress(torch_cuda.from_numpy(rec.copy()).cuda()).cpu().numpy().tobytes()
        assert f == T.oracle_frame(rec, dictionary=dct), dn
        assert T.zstd_decompress(f, len(rec), dictionary=dct) == rec.tobytes()
        sizes.append(len(f))
    assert max(sizes[:2]) <= 1.1 * min(sizes[:2]), sizes
