"""Config C1: HybridEngine FORCE_CPU on a 1 MiB dickens-like text,
host buffers only, through the C ABI (reference src/cuda_zstd_hybrid.cu:779-832,
402-458: the CPU route is libzstd ZSTD_compress at the configured level).  Runs here
without a GPU: host-to-host copies never touch HIP."""
import ctypes

import numpy as np

import zh_testlib as T

FORCE_CPU = 3  # HybridMode::FORCE_CPU (include/cuda_zstd_types.h)
HOST = 0


class Cfg(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_uint), ("cpu_size_threshold", ctypes.c_size_t), ("gpu_device_threshold", ctypes.c_size_t),
                ("compression_level", ctypes.c_int), ("enable_profiling", ctypes.c_int), ("cpu_thread_count", ctypes.c_uint)]


class Res(ctypes.Structure):
    _fields_ = [("backend_used", ctypes.c_uint), ("input_location", ctypes.c_uint), ("output_location", ctypes.c_uint),
                ("total_time_ms", ctypes.c_double), ("transfer_time_ms", ctypes.c_double), ("compute_time_ms", ctypes.c_double),
                ("throughput_mbps", ctypes.c_double), ("input_bytes", ctypes.c_size_t), ("output_bytes", ctypes.c_size_t),
                ("compression_ratio", ctypes.c_float)]


def test_c1_force_cpu_roundtrip(libzstd):
    import cuda_zstd

    L = cuda_zstd.lib()
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.cuda_zstd_hybrid_create.restype = vp
    L.cuda_zstd_hybrid_create.argtypes = [ctypes.POINTER(Cfg)]
    L.cuda_zstd_hybrid_compress.restype = ctypes.c_int
    L.cuda_zstd_hybrid_compress.argtypes = [vp, vp, sz, vp, ctypes.POINTER(sz), ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(Res), vp]
    L.cuda_zstd_hybrid_decompress.restype = ctypes.c_int
    L.cuda_zstd_hybrid_decompress.argtypes = L.cuda_zstd_hybrid_compress.argtypes
    L.cuda_zstd_hybrid_destroy.argtypes = [vp]
    L.cuda_zstd_hybrid_query_routing.restype = ctypes.c_uint
    L.cuda_zstd_hybrid_query_routing.argtypes = [vp, sz, ctypes.c_uint, ctypes.c_uint, ctypes.c_int]
    cfg = Cfg(FORCE_CPU, 0, 0, 3, 0, 1)
    e = L.cuda_zstd_hybrid_create(ctypes.byref(cfg))
    assert e
    try:
        data = T.gen(T.KINDS["text"], 1, 0x5EED0001, 1 << 20)
        out = np.zeros(libzstd.ZSTD_compressBound(ctypes.c_size_t(data.size)), np.uint8)
        osz = sz(out.size)
        r = Res()
        assert L.cuda_zstd_hybrid_query_routing(e, data.size, HOST, HOST, 1) == 0  # CPU_LIBZSTD
        rc = L.cuda_zstd_hybrid_compress(e, data.ctypes.data, data.size, out.ctypes.data, ctypes.byref(osz), HOST, HOST, ctypes.byref(r), None)
        assert rc == 0 and r.backend_used == 0
        frame = out[:osz.value].tobytes()
        # the CPU route is libzstd itself: byte-identical to ZSTD_compress(level 3)
        want = np.zeros(out.size, np.uint8)
        w = libzstd.ZSTD_compress(want.ctypes.data_as(vp), sz(want.size), data.ctypes.data_as(vp), sz(data.size), 3)
        assert frame == want[:w].tobytes()
        assert data.size / len(frame) > 2.0
        back = np.zeros(data.size, np.uint8)
        bsz = sz(back.size)
        rc = L.cuda_zstd_hybrid_decompress(e, out.ctypes.data, osz.value, back.ctypes.data, ctypes.byref(bsz), HOST, HOST, None, None)
        assert rc == 0 and bsz.value == data.size and np.array_equal(back, data)
    finally:
        L.cuda_zstd_hybrid_destroy(e)


def test_metadata_frame_host():
    """Skippable metadata frame (reference SkippableFrameHeader + CustomMetadataFrame,
    src/cuda_zstd_manager.cu:309-318, 391-412): libzstd skips it, extract_metadata reads the
    level and the following frame's header (host buffers, no GPU)."""
    import cuda_zstd

    data = T.gen(T.DG_TEXT, 1, 5, 100000)
    meta = cuda_zstd.metadata_frame(9)
    assert len(meta) == 16 and meta[:4] == bytes.fromhex("502a4d18")
    frame = T.oracle_frame(data, checksum=True)
    blob = meta + frame
    if T.zstd() is not None:
        assert T.zstd_decompress(blob, len(data)) == data.tobytes()
    m = cuda_zstd.extract_metadata(blob)
    assert m == {"level": 9, "uncompressed_size": len(data), "dictionary_id": 0, "checksum": True}
    assert cuda_zstd.extract_metadata(frame)["level"] == 3
