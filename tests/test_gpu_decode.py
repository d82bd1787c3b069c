"""GPU decoder (zh_decode.hip): bit-exact decodes on the MI355X.

Parity anchors: the original bytes (our own frames and libzstd frames round-trip), the
committed libzstd fixtures (tests/golden/decode_frames.json: SHA-256 of the expected
output, every decoder path), and libzstd's accept/reject decision on damaged frames.
Mirrors the reference's CPU-compress -> GPU-decompress tests
(tests/test_rfc8878_integration.cu:117-222), inference API tests
(tests/test_inference_api.cu:90-143, 307-381, 530-593) and batch tests."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import zh_testlib as T

pytestmark = pytest.mark.gpu

CORRUPT, TOO_SMALL, CHECKSUM, GENERIC = 6, 7, 10, 1


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def mgr(torch_cuda):
    import cuda_zstd

    return cuda_zstd.Manager(3)


def _dev(torch, b):
    a = np.frombuffer(bytes(b), np.uint8).copy()
    return torch.from_numpy(a if a.size else np.zeros(1, np.uint8)).cuda()[: len(b)]


def _decode(torch, mgr, frames, caps):
    outs, st = mgr.decompress_batch([_dev(torch, f) for f in frames], caps, raise_on_error=False)
    return [o.cpu().numpy().tobytes() for o in outs], st


def test_golden_fixture_frames(torch_cuda, mgr):
    vecs = json.load(open(os.path.join(T.GOLDEN, "decode_frames.json")))["vectors"]
    frames = [bytes.fromhex(v["frame"]) for v in vecs]
    caps = [max(v.get("size", 1 << 16), 1) for v in vecs]
    outs, st = _decode(torch_cuda, mgr, frames, caps)
    for v, o, s in zip(vecs, outs, st):
        if "expect_error" in v:
            assert s == CORRUPT, v["name"]
            continue
        assert s == 0, (v["name"], s)
        assert len(o) == v["size"] and hashlib.sha256(o).hexdigest() == v["sha256"], v["name"]


def test_own_frames_roundtrip(torch_cuda, mgr):
    items = T.special_inputs()
    datas = [items[k] for k in sorted(items)]
    for kind in sorted(T.KINDS):
        d = T.gen(T.KINDS[kind], 6, 0x5EED0003, first=40)
        datas += [d[i * 65536:(i + 1) * 65536] for i in range(6)]
    rng = np.random.default_rng(8)
    datas += [T.gen(T.DG_MIX, 1, 500 + i, int(s)) for i, s in enumerate(rng.integers(1, 65537, 20))]
    frames = mgr.compress_batch([torch_cuda.from_numpy(np.ascontiguousarray(d)).cuda() for d in datas])
    outs, st = mgr.decompress_batch(frames, [len(d) for d in datas], raise_on_error=False)
    assert st == [0] * len(datas)
    for k, (o, d) in enumerate(zip(outs, datas)):
        assert o.cpu().numpy().tobytes() == np.ascontiguousarray(d).tobytes(), f"item {k}"


def test_own_multiblock_frames(torch_cuda, mgr):
    data = np.concatenate([T.gen(T.DG_TEXT, 3, 5, 65536), T.gen(T.DG_CSV, 1, 6, 50000), T.gen(T.DG_RANDOM, 1, 7, 9000), np.zeros(70000, np.uint8)])
    frame = mgr.compress(torch_cuda.from_numpy(data).cuda())
    assert mgr.decompress(frame, len(data)).cpu().numpy().tobytes() == data.tobytes()


@pytest.mark.parametrize("level", [1, 3, 5, 9, 12, 19])
def test_libzstd_frames_by_level(torch_cuda, mgr, libzstd, level):
    """CPU (libzstd) compress -> GPU decompress (reference tests/test_rfc8878_integration.cu:117)."""
    datas = [(np.arange(1024) % 256).astype(np.uint8)]
    for kind in ("text", "mix", "json", "exe", "sensor", "sym16", "random", "csv"):
        datas.append(T.gen(T.KINDS[kind], 1, 900 + level, 65536))
    datas += [T.gen(T.DG_SOURCE, 1, 31, 1), T.gen(T.DG_SOURCE, 1, 32, 100), T.gen(T.DG_TEXT, 1, 33, 333333)]
    frames = [T.zstd_compress(d, level=level) for d in datas]
    outs, st = _decode(torch_cuda, mgr, frames, [len(d) for d in datas])
    assert st == [0] * len(datas)
    for k, (o, d) in enumerate(zip(outs, datas)):
        assert o == d.tobytes(), f"level {level} item {k}"


def test_libzstd_frame_options(torch_cuda, mgr, libzstd):
    d = T.gen(T.DG_TEXT, 1, 41, 200000)
    variants = [dict(level=3, checksum=True), dict(level=3, content_size=False), dict(level=5, window_log=10),
                dict(level=19, checksum=True, content_size=False), dict(level=1, window_log=12)]
    frames = [T.zstd_compress(d, **kw) for kw in variants]
    outs, st = _decode(torch_cuda, mgr, frames, [len(d)] * len(frames))
    assert st == [0] * len(frames)
    assert all(o == d.tobytes() for o in outs)


def test_concatenated_and_skippable_frames(torch_cuda, mgr, libzstd):
    a, b = T.gen(T.DG_JSON, 1, 51, 30000), T.gen(T.DG_EXE, 1, 52, 20000)
    skip = (0x184D2A53).to_bytes(4, "little") + (7).to_bytes(4, "little") + b"metadat"
    buf = skip + T.zstd_compress(a, level=3) + skip + T.oracle_frame(b) + skip
    outs, st = _decode(torch_cuda, mgr, [buf], [len(a) + len(b)])
    assert st == [0] and outs[0] == a.tobytes() + b.tobytes()


def test_decode_errors(torch_cuda, mgr, libzstd):
    d = T.gen(T.DG_TEXT, 1, 61, 50000)
    good = T.zstd_compress(d, level=3, checksum=True)
    bad_sum = bytearray(good)
    bad_sum[-1] ^= 0xFF
    frames = [good[:len(good) // 2], good[:10], b"\x00\x01\x02\x03\x04\x05\x06\x07", bytes(bad_sum), good, good]
    caps = [len(d), len(d), 100, len(d), len(d) - 1, len(d)]
    outs, st = _decode(torch_cuda, mgr, frames, caps)
    assert st[0] == CORRUPT and st[1] == CORRUPT
    assert st[2] == GENERIC  # ERROR_INVALID_MAGIC maps to the generic nvcomp code
    assert st[3] == CHECKSUM
    assert st[4] == TOO_SMALL
    assert st[5] == 0 and outs[5] == d.tobytes()


def test_damaged_frames_agree_with_libzstd(torch_cuda, mgr, libzstd):
    """Byte flips: the decoder never faults, rejects what libzstd rejects when the damage
    breaks the format, and when both accept, both produce the same bytes."""
    rng = np.random.default_rng(71)
    srcs = [T.zstd_compress(T.gen(T.DG_TEXT, 1, 72, 20000), level=19), T.oracle_frame(T.gen(T.DG_MIX, 1, 73, 30000)),
            T.zstd_compress(T.gen(T.DG_JSON, 1, 74, 25000), level=3)]
    frames, caps = [], []
    for i in range(150):
        f = bytearray(srcs[i % 3])
        for _ in range(1 + i % 3):
            f[rng.integers(0, len(f))] ^= int(rng.integers(1, 256))
        frames.append(bytes(f))
        caps.append(40000)
    outs, st = _decode(torch_cuda, mgr, frames, caps)
    z = T.zstd()
    agree = 0
    for f, o, s in zip(frames, outs, st):
        src = np.frombuffer(f, np.uint8).copy()
        dst = np.zeros(40000, np.uint8)
        r = z.ZSTD_decompress(dst.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(40000), src.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(len(src)))
        ok_ref = not z.ZSTD_isError(r)
        if s == 0 and ok_ref:
            assert o == dst[:r].tobytes()
        agree += (s == 0) == ok_ref
    assert agree >= 140, agree


def test_inference_api(torch_cuda, libzstd):
    """decompress_to_preallocated / decompress_async_no_sync semantics through the C ABI
    (reference tests/test_inference_api.cu): stream-ordered size, invalid arguments."""
    import cuda_zstd

    L = cuda_zstd.lib()
    m = L.cuda_zstd_create_manager(3)
    d = T.gen(T.DG_SOURCE, 1, 81, 256 * 1024)
    frame = _dev(torch_cuda, T.zstd_compress(d, level=3))
    out = torch_cuda.empty(len(d), dtype=torch_cuda.uint8, device="cuda")
    ws = torch_cuda.empty(L.cuda_zstd_get_decompress_workspace_size(m, frame.numel()), dtype=torch_cuda.uint8, device="cuda")
    sz = ctypes.c_size_t(len(d))
    assert L.cuda_zstd_decompress(m, frame.data_ptr(), frame.numel(), out.data_ptr(), ctypes.byref(sz), ws.data_ptr(), ws.numel(), None) == 0
    assert sz.value == len(d) and out.cpu().numpy().tobytes() == d.tobytes()
    # null pointers -> invalid parameter; short workspace -> buffer too small
    assert L.cuda_zstd_decompress(m, None, frame.numel(), out.data_ptr(), ctypes.byref(sz), ws.data_ptr(), ws.numel(), None) == 2
    assert L.cuda_zstd_decompress(m, frame.data_ptr(), frame.numel(), out.data_ptr(), ctypes.byref(sz), ws.data_ptr(), 1024, None) == 7
    small = ctypes.c_size_t(1000)
    assert L.cuda_zstd_decompress(m, frame.data_ptr(), frame.numel(), out.data_ptr(), ctypes.byref(small), ws.data_ptr(), ws.numel(), None) == 7
    L.cuda_zstd_destroy_manager(m)


def test_device_batched_api_roundtrip(torch_cuda):
    """nvcomp_zstd_batched_{compress,decompress}_async_v5 back to back on one stream, no host
    round trip in between; per-chunk capacities on the device."""
    import cuda_zstd

    n, cs = 512, 65536
    data = T.gen(T.DG_MIX, n, 0x5EED0003, cs, first=2000)
    dev = torch_cuda.from_numpy(data).cuda()
    bc = cuda_zstd.BatchedCompressor(3, cs)
    slot = (bc.max_out(cs) + 255) // 256 * 256
    comp = torch_cuda.empty(n * slot, dtype=torch_cuda.uint8, device="cuda")
    ar = torch_cuda.arange(n, dtype=torch_cuda.int64, device="cuda")
    in_ptrs, comp_ptrs = dev.data_ptr() + ar * cs, comp.data_ptr() + ar * slot
    sizes = torch_cuda.full((n,), cs, dtype=torch_cuda.int64, device="cuda")
    csizes = torch_cuda.zeros(n, dtype=torch_cuda.int64, device="cuda")
    temp = torch_cuda.empty(bc.temp_size(n, cs), dtype=torch_cuda.uint8, device="cuda")
    bc.compress_async(in_ptrs, sizes, cs, comp_ptrs, csizes, None, temp)
    bd = cuda_zstd.BatchedDecompressor()
    back = torch_cuda.zeros(n * cs, dtype=torch_cuda.uint8, device="cuda")
    back_ptrs = back.data_ptr() + ar * cs
    dsizes = torch_cuda.zeros(n, dtype=torch_cuda.int64, device="cuda")
    status = torch_cuda.full((n,), -1, dtype=torch_cuda.int32, device="cuda")
    dtemp = torch_cuda.empty(bd.temp_size(n, cs), dtype=torch_cuda.uint8, device="cuda")
    bd.decompress_async(comp_ptrs, csizes, sizes, cs, back_ptrs, dsizes, status, dtemp)
    torch_cuda.cuda.synchronize()
    assert (status == 0).all().item() and (dsizes == cs).all().item()
    assert torch_cuda.equal(back, dev)


def test_hybrid_device_decompress(torch_cuda, libzstd):
    """HybridEngine (AUTO): device-resident frames go to the GPU decoder."""
    import cuda_zstd

    L = cuda_zstd.lib()
    L.cuda_zstd_hybrid_create_default.restype = ctypes.c_void_p
    L.cuda_zstd_hybrid_destroy.argtypes = [ctypes.c_void_p]
    L.cuda_zstd_hybrid_decompress.restype = ctypes.c_int
    L.cuda_zstd_hybrid_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    e = L.cuda_zstd_hybrid_create_default()
    d = T.gen(T.DG_CSV, 1, 91, 100000)
    frame = _dev(torch_cuda, T.zstd_compress(d, level=7))
    out = torch_cuda.empty(len(d), dtype=torch_cuda.uint8, device="cuda")
    sz = ctypes.c_size_t(len(d))
    UNKNOWN = 3  # DataLocation::UNKNOWN: detect
    assert L.cuda_zstd_hybrid_decompress(e, frame.data_ptr(), frame.numel(), out.data_ptr(), ctypes.byref(sz), UNKNOWN, UNKNOWN, None, None) == 0
    assert sz.value == len(d) and out.cpu().numpy().tobytes() == d.tobytes()
    L.cuda_zstd_hybrid_destroy(e)


def test_c2_64mib_frame_decode(torch_cuda, mgr):
    """BASELINE config 2's frame (64 MiB, 1024 blocks, one workgroup walks them)."""
    data = T.gen(T.DG_SYM16, 1024, 0x5EED0002)
    dev = torch_cuda.from_numpy(data).cuda()
    frame = mgr.compress(dev)
    back = mgr.decompress(frame, len(data))
    assert torch_cuda.equal(back, dev)


def test_c3_full_batch_decode(torch_cuda):
    """BASELINE config 3 at full size: 16384 x 64 KiB compressed and decompressed on the
    GPU, compared on the device (size-independent round-trip property)."""
    import cuda_zstd

    n, cs = 16384, 65536
    data = T.gen(T.DG_MIX, n, 0x5EED0003, cs)
    dev = torch_cuda.from_numpy(data).cuda()
    del data
    bc = cuda_zstd.BatchedCompressor(3, cs)
    slot = (bc.max_out(cs) + 255) // 256 * 256
    comp = torch_cuda.empty(n * slot, dtype=torch_cuda.uint8, device="cuda")
    ar = torch_cuda.arange(n, dtype=torch_cuda.int64, device="cuda")
    in_ptrs, comp_ptrs = dev.data_ptr() + ar * cs, comp.data_ptr() + ar * slot
    sizes = torch_cuda.full((n,), cs, dtype=torch_cuda.int64, device="cuda")
    csizes = torch_cuda.zeros(n, dtype=torch_cuda.int64, device="cuda")
    temp = torch_cuda.empty(bc.temp_size(n, cs), dtype=torch_cuda.uint8, device="cuda")
    bc.compress_async(in_ptrs, sizes, cs, comp_ptrs, csizes, None, temp)
    del temp
    bd = cuda_zstd.BatchedDecompressor()
    back = torch_cuda.zeros(n * cs, dtype=torch_cuda.uint8, device="cuda")
    dsizes = torch_cuda.zeros(n, dtype=torch_cuda.int64, device="cuda")
    status = torch_cuda.full((n,), -1, dtype=torch_cuda.int32, device="cuda")
    dtemp = torch_cuda.empty(bd.temp_size(n, cs), dtype=torch_cuda.uint8, device="cuda")
    bd.decompress_async(comp_ptrs, csizes, None, cs, back.data_ptr() + ar * cs, dsizes, status, dtemp)
    torch_cuda.cuda.synchronize()
    assert (status == 0).all().item() and (dsizes == cs).all().item()
    assert torch_cuda.equal(back, dev)


def test_split_pipeline_mixed_batch_matches_small_batches(torch_cuda, mgr, libzstd):
    """Batches of >= 2048 buffers take the split pipeline (zh_decode.hip launch_decompress:
    a tables-only pass, the sequence kernel beside the literals pass, execution); smaller ones
    the one-pass phase 1.  A 2,304-buffer batch mixing deferrable frames (this library's and
    libzstd's), raw / RLE / multi-block frames, damaged frames (some fail only in the literals
    pass, after the tables pass deferred them) and truncated ones must give every buffer the
    same status and bytes as the same frames decoded 576 at a time, and agree with libzstd."""
    rng = np.random.default_rng(2304)
    frames = []
    own = [T.gen(T.DG_MIX, 1, 900 + i, 65536) for i in range(6)]
    own_frames = [bytes(f.cpu().numpy().tobytes()) for f in mgr.compress_batch([torch_cuda.from_numpy(np.ascontiguousarray(d)).cuda() for d in own])]
    z_frames = [T.zstd_compress(T.gen(k, 1, 950 + j, s), level=lv)
                for j, (k, s, lv) in enumerate([(T.DG_TEXT, 30000, 1), (T.DG_JSON, 65536, 3), (T.DG_SOURCE, 50000, 9),
                                                 (T.DG_CSV, 40000, 19), (T.DG_RANDOM, 20000, 3), (T.DG_TEXT, 200000, 3)])]
    z_frames.append(T.zstd_compress(np.zeros(60000, np.uint8), level=3))
    pool = own_frames + z_frames
    for i in range(2304):
        f = bytearray(pool[i % len(pool)])
        kind = i % 7
        if kind == 5:  # damaged: a few byte flips past the frame header
            for _ in range(1 + i % 3):
                f[int(rng.integers(6, len(f)))] ^= int(rng.integers(1, 256))
        elif kind == 6 and i % 14 == 6:  # truncated
            f = f[: int(rng.integers(1, len(f)))]
        frames.append(bytes(f))
    caps = [262144] * len(frames)
    outs, st = _decode(torch_cuda, mgr, frames, caps)
    small_o, small_s = [], []
    for k in range(0, len(frames), 576):
        o, s = _decode(torch_cuda, mgr, frames[k:k + 576], caps[k:k + 576])
        small_o += o
        small_s += s
    assert st == small_s
    for k, (a, b, s) in enumerate(zip(outs, small_o, st)):
        if s == 0:
            assert a == b, f"item {k}"
    z = T.zstd()
    agree = 0
    for f, o, s in zip(frames, outs, st):
        src = np.frombuffer(f, np.uint8).copy()
        dst = np.zeros(262144, np.uint8)
        r = z.ZSTD_decompress(dst.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(262144), src.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(len(src)))
        ok_ref = not z.ZSTD_isError(r)
        if s == 0 and ok_ref:
            assert o == dst[:r].tobytes()
        agree += (s == 0) == ok_ref
    assert agree >= len(frames) - 40, agree
    assert sum(1 for s in st if s == 0) >= 1900
