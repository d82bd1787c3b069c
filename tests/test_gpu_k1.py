"""GPU parity of the LZ stage alone: K1's raw output (sequence records + literal bytes, read
back through the library's zh_test_lz hook) equals the oracle's parse
(oracle/zstd_oracle.c orc_lz_parse: tile-lagged dual hash, lazy-1 parse, catch-up) on the
same inputs.  Finer-grained than the frame tests: a mismatch names the first differing
sequence.  K1's records carry the walk's cumulative literal count and the catch-up length; consecutive
same-offset records with no literals between them are merged (K2 merges them the same way)."""
import ctypes

import numpy as np
import pytest

import zh_testlib as T

pytestmark = pytest.mark.gpu

BLOCK = 65536
K1HIST, K1_HIST_OFF = 2, 65536  # ZH_META_K1HIST, ZH_K1_HIST_OFF (zh_common.h)


def k1_raw(datas):
    import torch

    import cuda_zstd

    L = cuda_zstd.lib()
    n = len(datas)
    stride = BLOCK
    buf = np.zeros(n * stride, dtype=np.uint8)
    for i, d in enumerate(datas):
        buf[i * stride:i * stride + len(d)] = d
    dev = torch.from_numpy(buf).cuda()
    sizes = np.array([len(d) for d in datas], dtype=np.uint32)
    # per-item sizes the hook copies back (ZH_SEQ_CAP, ZH_LIT_BYTES), from the library itself
    cap, area_b = ctypes.c_uint32(), ctypes.c_uint32()
    L.zh_test_lz_sizes(ctypes.byref(cap), ctypes.byref(area_b))
    SEQ_CAP, LIT_AREA = cap.value, area_b.value
    recs = np.zeros(n * SEQ_CAP, dtype=np.uint64)
    lits = np.zeros(n * LIT_AREA, dtype=np.uint8)
    meta = np.zeros(n * 4, dtype=np.uint32)
    f = L.zh_test_lz
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p]
    torch.cuda.synchronize()
    rc = f(dev.data_ptr(), n, stride, sizes.ctypes.data, 0, recs.ctypes.data, lits.ctypes.data, meta.ctypes.data)
    assert rc == 0
    out = []
    for i in range(n):
        ns, nl, rle = (int(x) for x in meta[4 * i:4 * i + 3])
        r = recs[i * SEQ_CAP:i * SEQ_CAP + ns]
        area = lits[i * LIT_AREA:(i + 1) * LIT_AREA]
        if rle == K1HIST:  # literals = the block itself; K1's sub-histograms after the first 64 KiB
            out.append((r, area[K1_HIST_OFF:K1_HIST_OFF + 16 * 1024].view(np.uint32).reshape(16, 256).sum(0), rle))
        else:
            out.append((r, area[:nl].tobytes(), rle))
    k1_raw.area = lits
    return out


def merged(recs):
    """K1 records -> (ll, ml, off) with same-offset continuations merged.  A record holds the
    walk's literal count before the match, its length, its catch-up e (bytes of the literal run
    before it that join the match) and its offset."""
    seqs, prev = [], 0
    for v in recs:
        v = int(v)
        cum, ln, e, off = v & 0x1FFFF, (v >> 17) & 0x7F, (v >> 24) & 0xFFF, (v >> 36) & 0x1FFFF
        ll, ml = cum - prev - e, ln + e
        prev = cum
        if seqs and ll == 0 and seqs[-1][2] == off:
            seqs[-1][1] += ml
        else:
            seqs.append([ll, ml, off])
    return [tuple(s) for s in seqs], prev


def oracle_parse(d):
    O = T.oracle()
    d = np.ascontiguousarray(d, dtype=np.uint8)
    seq = (ctypes.c_uint32 * (3 * (len(d) // 5 + 2)))()
    last = ctypes.c_uint32(0)
    ns = O.orc_lz_parse(d.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(d)), seq, ctypes.byref(last))
    return [(seq[3 * i], seq[3 * i + 1], seq[3 * i + 2]) for i in range(ns)], last.value


def expected_literals(d, seqs, last):
    out, pos = bytearray(), 0
    for ll, ml, _ in seqs:
        out += bytes(d[pos:pos + ll])
        pos += ll + ml
    out += bytes(d[pos:pos + last])
    return bytes(out)


def _compare(datas, names):
    got = k1_raw(datas)
    for (recs, lits, rle), d, nm in zip(got, datas, names):
        if rle == K1HIST:
            # the incompressibility probe ended the block: no sequences, every byte a literal, read
            # by K2 from the source; K1 left the literal histogram
            want, last = oracle_parse(d)
            assert want == [] and last == len(d), f"{nm}: K1 ended the block at the probe, the oracle did not"
            assert len(recs) == 0
            assert np.array_equal(lits, np.bincount(d, minlength=256)), f"{nm}: K1 literal histogram"
            continue
        if rle:
            assert len(d) >= 2 and (d == d[0]).all(), f"{nm}: RLE flag on a non-RLE block"
            continue
        want, last = oracle_parse(d)
        have, cum_end = merged(recs)
        if have != want:
            k = next((i for i, (a, b) in enumerate(zip(have, want)) if a != b), min(len(have), len(want)))
            pos = sum(a + b for a, b, _ in want[:k])
            raise AssertionError(f"{nm}: sequence {k} (position {pos}) GPU {have[k:k + 3]} oracle {want[k:k + 3]}; "
                                 f"counts {len(have)} vs {len(want)}")
        exp = expected_literals(d, want, last)
        if lits != exp:
            k = next((i for i, (a, b) in enumerate(zip(lits, exp)) if a != b), min(len(lits), len(exp)))
            raise AssertionError(f"{nm}: literal bytes differ at literal {k} of {len(lits)} (oracle {len(exp)}): "
                                 f"GPU {lits[k:k + 12].hex()} oracle {exp[k:k + 12].hex()}")


def test_k1_corpora_vs_oracle():
    names, datas = [], []
    for kname in ("mix", "text", "source", "csv", "exe", "sensor", "json", "random", "sym16"):
        for i in range(3):
            names.append(f"{kname}[{i}]")
            datas.append(T.gen(T.KINDS[kname], 1, 0x5EED0003, BLOCK, first=i))
    _compare(datas, names)


def test_k1_miss_skip_transitions_vs_oracle():
    """Blocks that enter and leave the miss-skip mode (oracle orc_lz_parse_pre: a window after a
    window without matches searches only its first tiles): random stretches between text,
    random with a repeat of an earlier stretch, text inside random at window offsets."""
    rng = np.random.default_rng(11)
    text = T.gen(T.DG_TEXT, 1, 0x5EED0009, BLOCK)
    rnd = rng.integers(0, 256, BLOCK, dtype=np.uint8)
    datas, names = [], []

    def add(nm, d):
        names.append(nm)
        datas.append(np.ascontiguousarray(d[:BLOCK], dtype=np.uint8))

    add("rand16k+text", np.concatenate([rnd[:16384], text[:49152]]))
    add("text8k+rand40k+text", np.concatenate([text[:8192], rnd[:40960], text[8192:24576]]))
    rep = rnd.copy()
    rep[40000:52000] = rep[1000:13000]
    add("rand+repeat", rep)
    for off in (9 * 2048 + 100, 9 * 2048 + 300, 20 * 2048 - 50):
        d = rnd.copy()
        d[off:off + 6000] = text[:6000]
        add(f"rand+text@{off}", d)
    add("rand_ragged", rnd[:30001])
    _compare(datas, names)


def test_k1_probe_vs_oracle():
    """The incompressibility probe (ZH_PROBE_WINDOWS, oracle orc_lz_parse_pre): a block whose
    parse takes no match in its first windows takes no sequences at all.  Blocks that die at the
    probe, blocks whose probe windows just reach compressible bytes, text with a random stretch
    after the probe (the miss skip, not the probe), and short blocks with no window past the probe."""
    rng = np.random.default_rng(12)
    text = T.gen(T.DG_TEXT, 1, 0x5EED0019, BLOCK)
    rnd = rng.integers(0, 256, BLOCK, dtype=np.uint8)
    W = 2048
    datas, names = [], []

    def add(nm, d):
        names.append(nm)
        datas.append(np.ascontiguousarray(d, dtype=np.uint8))

    # (boundaries of one and of two probe windows)
    for cut in (W - 200, W - 1, W, W + 1, 2 * W - 200, 2 * W, 2 * W + 1, 3 * W):
        add(f"rand{cut}+text", np.concatenate([rnd[:cut], text[:BLOCK - cut]]))
    add("text4k+rand+text", np.concatenate([text[:4096], rnd[:40960], text[4096:24576]]))
    for at in (1100, W + 100):  # one repeat inside the first window / inside the second
        half = rnd[:2 * W].copy()
        half[at:at + 300] = half[100:400]
        add(f"rand+repeat@{at}", np.concatenate([half, rnd[2 * W:]]))
    for n in (W + 8, W + 9, 2 * W + 8, 2 * W + 9, 3 * W + 8, 3 * W + 9, 5000):
        add(f"rand_{n}", rnd[:n])
    _compare(datas, names)


def test_k1_special_and_ragged_vs_oracle():
    items = T.special_inputs()
    names = sorted(k for k in items if 0 < len(items[k]) <= BLOCK)
    datas = [items[k] for k in names]
    rng = np.random.default_rng(5)
    for n in (1, 7, 63, 64, 65, 4095, 4096, 4097, 8191, 12345, 40000, 65535):
        names.append(f"text{n}")
        datas.append(T.gen(T.DG_TEXT, 1, int(rng.integers(1 << 30)), 65536)[:n].copy())
    _compare(datas, names)


def test_ins_check_variant_never_repairs(tmp_path):
    """The determinism guard (DESIGN §2 K1 inserters): K1's hash tables rely on
    gfx950 leaving the highest lane's value when lanes of one ds_write_b16 hit the same slot.  The
    -DZH_INS_CHECK build reads every slot back and repairs a lost store.  Run the C3 sample and the
    corpora batch through that build (child process, CUDA_ZSTD_HIP_LIB): the repair path must fire 0
    times and its frames must equal this (default) build's."""
    import os
    import subprocess
    import sys

    import ins_check_data as D

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "custom-nvcomp-with-zstd_amd", "libcuda_zstd_hip_inscheck.so")
    assert os.path.exists(so), "build() makes the check variant"
    env = dict(os.environ, CUDA_ZSTD_HIP_LIB=so)
    out = tmp_path / "ic.npz"
    subprocess.run([sys.executable, os.path.join(root, "tests", "ins_check_worker.py"), str(out)], env=env, check=True, timeout=300)
    r = np.load(out)
    assert int(r["repairs"][0]) == 0, "the inserter repair path fired: same-slot lane order differs from the oracle's"
    for level in D.LEVELS:
        want = D.compress(level)
        sizes = r[f"sizes{level}"]
        assert sizes.tolist() == [len(f) for f in want], level
        assert r[f"frames{level}"].tobytes() == b"".join(want), level
