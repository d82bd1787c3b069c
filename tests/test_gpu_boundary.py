"""The reference's own call shapes on the drop-in boundary (§8f F1
inference API), on the GPU:

* NvcompV5BatchManager::compress_async with device pointer arrays, host input sizes and a
  device size array (reference tests/test_nvcomp_batch.cu:132-134), then decompress_async
  with device arrays -- through the C++ API (tests/cpp/boundary.cpp);
* CompressionConfig::cpu_threshold routing (reference src/cuda_zstd_manager.cu:1604-1668):
  a 64 KiB device item below a 1 MiB threshold takes the libzstd route, a 2 MiB one the GPU;
  per item in compress_batch (the reference's per-item compress() loop, :5744-5768);
* the single-buffer C entry nvcomp_zstd_compress_async_v5 / nvcomp_zstd_decompress_async_v5;
* the inference flow (allocate_inference_workspace + decompress_to_preallocated, reference
  tests/test_inference_api.cu:398-410) with outputs below 128 KiB.
GPU frames must equal the oracle's; every frame must decode with libzstd."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import zh_testlib as T

pytestmark = pytest.mark.gpu
DRIVER = os.path.join(T.ROOT, "tests", "cpp", "boundary")


def _chunks():
    sizes = [65536, 65536, 40001, 1000, 65536, 12345, 9]
    return [T.gen(k, 1, 900 + i, s) for i, (k, s) in enumerate(zip([T.DG_MIX, T.DG_TEXT, T.DG_JSON, T.DG_EXE, T.DG_RANDOM, T.DG_CSV, T.DG_MIX], sizes))]


def _run(mode, datas, tmp_path, *extra):
    assert os.path.exists(DRIVER), "tests/cpp/boundary not built (__graft_entry__.build())"
    (tmp_path / "in.bin").write_bytes(b"".join(d.tobytes() for d in datas))
    (tmp_path / "sizes.bin").write_bytes(np.array([len(d) for d in datas], np.uint64).tobytes())
    r = subprocess.run([DRIVER, mode, str(tmp_path), *extra], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, f"boundary {mode}: rc {r.returncode}\n{r.stdout}\n{r.stderr}"
    fs = np.frombuffer((tmp_path / "fsizes.bin").read_bytes(), np.uint64)
    blob = (tmp_path / "frames.bin").read_bytes()
    offs = np.concatenate([[0], np.cumsum(fs)]).astype(np.int64)
    return [blob[offs[i]:offs[i + 1]] for i in range(len(fs))]


def test_nvcomp_batch_device_arrays(tmp_path, libzstd):
    datas = _chunks()
    frames = _run("nvcomp", datas, tmp_path)
    for k, (f, d) in enumerate(zip(frames, datas)):
        assert f == T.oracle_frame(d), f"item {k}"
        assert T.zstd_decompress(f, len(d)) == d.tobytes()
    assert (tmp_path / "back.bin").read_bytes() == b"".join(d.tobytes() for d in datas)


def test_cpu_threshold_routing(tmp_path, libzstd):
    small = T.gen(T.DG_MIX, 1, 0x5EED0003, 65536)
    big = T.gen(T.DG_MIX, 32, 0x5EED0003, 65536)  # 2 MiB: at/above the threshold -> GPU
    frames = _run("threshold", [small, big], tmp_path, str(1 << 20))
    # below the threshold: libzstd's own frame (the reference's CPU route), not the GPU's
    assert frames[0] != T.oracle_frame(small)
    cands = set()
    for p in ("/opt/conda/lib/libzstd.so.1", "libzstd.so.1", "/usr/lib/x86_64-linux-gnu/libzstd.so.1"):
        try:
            L = ctypes.CDLL(p)
        except OSError:
            continue
        L.ZSTD_compress.restype = ctypes.c_size_t
        L.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        out = np.zeros(70000, np.uint8)
        r = L.ZSTD_compress(out.ctypes.data, 70000, small.ctypes.data, len(small), 3)
        cands.add(out[:r].tobytes())
    assert frames[0] in cands, "CPU-routed frame is not libzstd ZSTD_compress(level 3)"
    assert T.zstd_decompress(frames[0], len(small)) == small.tobytes()
    assert frames[1] == T.oracle_frame(big)
    assert T.zstd_decompress(frames[1], len(big)) == big.tobytes()
    # threshold 0 (the default): the 64 KiB item goes to the GPU
    frames0 = _run("threshold", [small], tmp_path, "0")
    assert frames0[0] == T.oracle_frame(small)


def _libzstd_l3(d):
    """ZSTD_compress(level 3) frames of d from every libzstd on the box (the CPU route's output)."""
    cands = set()
    for p in ("/opt/conda/lib/libzstd.so.1", "libzstd.so.1", "/usr/lib/x86_64-linux-gnu/libzstd.so.1"):
        try:
            L = ctypes.CDLL(p)
        except OSError:
            continue
        L.ZSTD_compress.restype = ctypes.c_size_t
        L.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        cap = len(d) + (len(d) >> 7) + 1024
        out = np.zeros(cap, np.uint8)
        r = L.ZSTD_compress(out.ctypes.data, cap, d.ctypes.data, len(d), 3)
        cands.add(out[:r].tobytes())
    return cands


def test_compress_batch_per_item_threshold(tmp_path, libzstd):
    """ZstdBatchManager::compress_batch with cpu_threshold = 48 KiB over mixed sizes: items
    below it equal libzstd ZSTD_compress(3) (the reference's per-item compress() route), the
    rest equal the oracle's GPU frame; all decode."""
    datas = _chunks() + [T.gen(T.DG_MIX, 1, 950, 300000)]
    thr = 48 * 1024
    frames = _run("batch_threshold", datas, tmp_path, str(thr))
    for k, (f, d) in enumerate(zip(frames, datas)):
        if len(d) < thr:
            assert f in _libzstd_l3(d), f"item {k} ({len(d)} B): not the libzstd route"
        else:
            assert f == T.oracle_frame(d), f"item {k} ({len(d)} B)"
        assert T.zstd_decompress(f, len(d)) == d.tobytes()
    # threshold 0: every item on the GPU
    frames0 = _run("batch_threshold", datas, tmp_path, "0")
    for k, (f, d) in enumerate(zip(frames0, datas)):
        assert f == T.oracle_frame(d), f"item {k}"


def test_inference_workspace(tmp_path, libzstd):
    datas = [T.gen(T.DG_TEXT, 1, 77, 65536), T.gen(T.DG_JSON, 1, 78, 5000), T.gen(T.DG_MIX, 1, 79, 65536 * 3 + 17)]
    frames = _run("inference", datas, tmp_path)
    for f, d in zip(frames, datas):
        assert f == T.oracle_frame(d)
    assert (tmp_path / "back.bin").read_bytes() == b"".join(d.tobytes() for d in datas)


def test_nvcomp_single_buffer_c_api(libzstd):
    import torch

    import cuda_zstd

    L = cuda_zstd.lib()
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.nvcomp_zstd_create_manager_v5.restype = vp
    L.nvcomp_zstd_create_manager_v5.argtypes = [ctypes.c_int]
    L.nvcomp_zstd_destroy_manager_v5.argtypes = [vp]
    L.nvcomp_zstd_get_compress_temp_size_v5.restype = sz
    L.nvcomp_zstd_get_compress_temp_size_v5.argtypes = [vp, sz]
    L.nvcomp_zstd_get_decompress_temp_size_v5.restype = sz
    L.nvcomp_zstd_get_decompress_temp_size_v5.argtypes = [vp, sz]
    L.nvcomp_zstd_compress_async_v5.argtypes = [vp, vp, sz, vp, ctypes.POINTER(sz), vp, sz, vp]
    L.nvcomp_zstd_decompress_async_v5.argtypes = [vp, vp, sz, vp, ctypes.POINTER(sz), vp, sz, vp]
    h = L.nvcomp_zstd_create_manager_v5(3)
    assert h
    try:
        for n in (65536, 1 << 20, 777):
            d = T.gen(T.DG_MIX, 1, 4242, n)
            din = torch.from_numpy(d).cuda()
            out = torch.empty(cuda_zstd.max_compressed_size(n), dtype=torch.uint8, device="cuda")
            tmp = torch.empty(L.nvcomp_zstd_get_compress_temp_size_v5(h, n), dtype=torch.uint8, device="cuda")
            cs = sz(out.numel())
            s = torch.cuda.current_stream().cuda_stream
            assert L.nvcomp_zstd_compress_async_v5(h, din.data_ptr(), n, out.data_ptr(), ctypes.byref(cs), tmp.data_ptr(), tmp.numel(), s) == 0
            frame = out[: cs.value].cpu().numpy().tobytes()  # output valid on return (reference semantics)
            assert frame == T.oracle_frame(d)
            assert T.zstd_decompress(frame, n) == d.tobytes()
            back = torch.empty(n, dtype=torch.uint8, device="cuda")
            dt = torch.empty(L.nvcomp_zstd_get_decompress_temp_size_v5(h, cs.value), dtype=torch.uint8, device="cuda")
            us = sz(n)
            assert L.nvcomp_zstd_decompress_async_v5(h, out.data_ptr(), cs.value, back.data_ptr(), ctypes.byref(us), dt.data_ptr(), dt.numel(), s) == 0
            assert us.value == n and torch.equal(back, din)
    finally:
        L.nvcomp_zstd_destroy_manager_v5(h)


@pytest.mark.parametrize("formatted", [False, True])
@pytest.mark.parametrize("history", [0, 1])
def test_streaming_with_dictionary(tmp_path, libzstd, formatted, history):
    """ZstdStreamingManager::set_dictionary, then compress_chunk (history 0) or
    compress_chunk_with_history (1) over 5 chunks and decompress_chunk in order: the stream
    comes back (chunks of their own decode with the dictionary, not with the decoded window;
    advisor round 2).  Chunks of their own equal the oracle's frame with the dictionary and
    decode with libzstd ZSTD_decompress_usingDict."""
    recs = [T.gen(T.DG_JSON, 1, 0x5EED0005, 16384, first=i) for i in range(64)]
    dct = T.zdict_train(recs, 32768) if formatted else b"".join(r.tobytes() for r in recs[:2])
    datas = [T.gen(T.DG_JSON, 1, 0x5EED0005, n, first=100 + i) for i, n in enumerate([16384, 40000, 65536, 777, 30000])]
    (tmp_path / "dict.bin").write_bytes(dct)
    frames = _run("stream_dict", datas, tmp_path, str(history))
    assert (tmp_path / "back.bin").read_bytes() == b"".join(d.tobytes() for d in datas)
    if not history:
        for k, (f, d) in enumerate(zip(frames, datas)):
            assert f == T.oracle_frame(d, dictionary=dct), f"chunk {k}"
            assert T.zstd_decompress(f, len(d), dictionary=dct) == d.tobytes()


@pytest.mark.parametrize("formatted", [False, True])
def test_cxx_extra_surface(tmp_path, libzstd, formatted):
    """The rest of the reference's C++ boundary (VERDICT r3 missing #1), called by
    tests/cpp/boundary.cpp: compress_with_dict / decompress_with_dict frames equal the
    oracle's frame with the dictionary and decode with libzstd ZSTD_decompress_usingDict;
    a workspace from allocate_compression_workspace gives the same frames; the error API,
    HybridEngine move ops / decompress_batch / profiling and hybrid_decompress are checked
    inside the driver."""
    recs = [T.gen(T.DG_JSON, 1, 0x5EED0005, 16384, first=i) for i in range(64)]
    dct = T.zdict_train(recs, 32768) if formatted else b"".join(r.tobytes() for r in recs[:2])
    datas = [T.gen(T.DG_JSON, 1, 0x5EED0005, n, first=200 + i) for i, n in enumerate([16384, 65536, 777, 30000])]
    (tmp_path / "dict.bin").write_bytes(dct)
    frames = _run("cxx_extra", datas, tmp_path)
    assert (tmp_path / "back.bin").read_bytes() == b"".join(d.tobytes() for d in datas)
    for k, (f, d) in enumerate(zip(frames, datas)):
        assert f == T.oracle_frame(d, dictionary=dct), f"item {k}"
        assert T.zstd_decompress(f, len(d), dictionary=dct) == d.tobytes()


@pytest.mark.parametrize("formatted,flag", [(True, 1), (False, 1), (True, 2), (False, 2)])
def test_streaming_history_second_manager(tmp_path, libzstd, formatted, flag):
    """Frames from compress_chunk_with_history (dictionary set) decode in a SECOND, decode-only
    streaming manager with the same dictionary (advisor r3) once it is told the session has history
    (init_decompression_with_history, flag 1): history frames carry no Dictionary_ID, and neither
    does a dictionary frame written without one (test_streaming_idless_dictionary_frames).
    flag 2: the decoder is NOT told (plain init_decompression) and the frames carry a
    content checksum; each fails against the dictionary (corrupt, or a wrong checksum) and is decoded
    again against the decoded window, so the bytes come back right instead of silently wrong."""
    recs = [T.gen(T.DG_JSON, 1, 0x5EED0005, 16384, first=i) for i in range(64)]
    dct = T.zdict_train(recs, 32768) if formatted else b"".join(r.tobytes() for r in recs[:2])
    datas = [T.gen(T.DG_JSON, 1, 0x5EED0005, n, first=300 + i) for i, n in enumerate([16384, 40000, 65536, 777, 30000])]
    (tmp_path / "dict.bin").write_bytes(dct)
    _run("stream_split", datas, tmp_path, str(flag))
    assert (tmp_path / "back.bin").read_bytes() == b"".join(d.tobytes() for d in datas)


@pytest.mark.parametrize("level", [3, 5])
def test_static_batched_temp_size_levels(libzstd, level):
    """nvcomp_zstd_batched_compress_get_temp_size_v5 (static) covers levels below 5
    without a dictionary; at level 5 (the deep matcher's scratch slots) a workspace of that size
    is refused with 7 before anything is launched, and the handle's own size
    (nvcomp_zstd_batch_get_batched_temp_size_v5) works.  Frames equal the oracle's at that level."""
    import torch

    import cuda_zstd

    L = cuda_zstd.lib()
    datas = [T.gen(T.DG_MIX, 1, 0x5EED0003, 65536, first=i) for i in range(6)]
    n, chunk = len(datas), 65536
    c = cuda_zstd.BatchedCompressor(level, chunk)
    static = L.nvcomp_zstd_batched_compress_get_temp_size_v5(n, chunk)
    own = c.temp_size(n, chunk)
    assert (own == static) if level < 5 else (own > static)
    src = torch.from_numpy(np.concatenate(datas)).cuda()
    cap = L.nvcomp_zstd_batch_get_max_compressed_chunk_size_v5(c._h, chunk)
    out = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
    ptrs = torch.tensor([src.data_ptr() + i * chunk for i in range(n)], dtype=torch.int64, device="cuda")
    optr = torch.tensor([out.data_ptr() + i * cap for i in range(n)], dtype=torch.int64, device="cuda")
    sizes = torch.full((n,), chunk, dtype=torch.int64, device="cuda")
    osz = torch.zeros(n, dtype=torch.int64, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    if level >= 5:
        small = torch.zeros(static, dtype=torch.uint8, device="cuda")
        with pytest.raises(cuda_zstd.ZstdError) as e:
            c.compress_async(ptrs, sizes, chunk, optr, osz, st, small)
        assert e.value.code == 7
        assert int(osz.sum().item()) == 0  # nothing was launched
    temp = torch.zeros(own, dtype=torch.uint8, device="cuda")
    c.compress_async(ptrs, sizes, chunk, optr, osz, st, temp)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for i, d in enumerate(datas):
        f = o[i * cap:i * cap + int(osz[i].item())].tobytes()
        assert f == T.oracle_frame(d, level=level), f"item {i}"
        assert T.zstd_decompress(f, len(d)) == d.tobytes()
    c.close()


def test_streaming_idless_dictionary_frames(tmp_path, libzstd):
    """libzstd frames compressed with a formatted dictionary but without its ID in the
    header (ZSTD_c_dictIDFlag = 0) decode, one after another, in a streaming manager with that
    dictionary set and no history session -- each against the dictionary, not the previous output."""
    import ctypes

    z = libzstd
    recs = [T.gen(T.DG_JSON, 1, 0x5EED0005, 16384, first=i) for i in range(64)]
    dct = T.zdict_train(recs, 32768)
    datas = [T.gen(T.DG_JSON, 1, 0x5EED0005, n, first=400 + i) for i, n in enumerate([16384, 9000, 30000, 16384])]
    z.ZSTD_createCCtx.restype = ctypes.c_void_p
    z.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
    z.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    z.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
    z.ZSTD_CCtx_loadDictionary.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    z.ZSTD_CCtx_loadDictionary.restype = ctypes.c_size_t
    z.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    z.ZSTD_compress2.restype = ctypes.c_size_t
    frames = []
    db = np.frombuffer(dct, np.uint8).copy()
    for d in datas:
        cctx = z.ZSTD_createCCtx()
        assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cctx, 100, 3))
        assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cctx, 202, 0))  # ZSTD_c_dictIDFlag
        assert not z.ZSTD_isError(z.ZSTD_CCtx_loadDictionary(cctx, db.ctypes.data, len(db)))
        out = np.zeros(len(d) + 1024, np.uint8)
        r = z.ZSTD_compress2(cctx, out.ctypes.data, len(out), d.ctypes.data, len(d))
        z.ZSTD_freeCCtx(cctx)
        assert not z.ZSTD_isError(r)
        f = out[:r].copy()
        assert f[4] & 3 == 0  # Frame_Header_Descriptor: no Dictionary_ID field
        frames.append(f)
    (tmp_path / "dict.bin").write_bytes(dct)
    (tmp_path / "usizes.bin").write_bytes(np.array([len(d) for d in datas], np.uint64).tobytes())
    _run("stream_ext", frames, tmp_path)
    assert (tmp_path / "back.bin").read_bytes() == b"".join(d.tobytes() for d in datas)
