"""Test helpers: ctypes access to the oracle (CPU restatement), libzstd (the
reference's own dependency, used as the decoder / stage oracle) and the seeded
synthetic-data generator.  Test infrastructure only."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "custom-nvcomp-with-zstd_amd")
ORACLE_SO = os.environ.get("ZH_ORACLE_SO") or os.path.join(ROOT, "oracle", "liboracle.so")
DATAGEN_SO = os.path.join(ROOT, "tools", "libdatagen.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

DG_MIX, DG_RANDOM, DG_SYM16, DG_TEXT, DG_JSON, DG_SOURCE, DG_CSV, DG_EXE, DG_SENSOR = range(9)
KINDS = {"mix": DG_MIX, "random": DG_RANDOM, "sym16": DG_SYM16, "text": DG_TEXT, "json": DG_JSON, "source": DG_SOURCE,
         "csv": DG_CSV, "exe": DG_EXE, "sensor": DG_SENSOR}

vp = ctypes.c_void_p
_o = _d = _z = None


def oracle():
    global _o
    if _o is None:
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_compress_frame.restype = ctypes.c_size_t
        L.orc_compress_frame.argtypes = [vp, ctypes.c_size_t, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_fse_normalize.restype = ctypes.c_int
        L.orc_fse_write_ncount.restype = ctypes.c_size_t
        L.orc_huf_build_ctable.restype = ctypes.c_uint32
        L.orc_huf_write_ctable.restype = ctypes.c_size_t
        L.orc_compress_literals.restype = ctypes.c_size_t
        L.orc_lz_parse.restype = ctypes.c_size_t
        L.orc_compress_block.restype = ctypes.c_size_t
        L.orc_max_compressed_size.restype = ctypes.c_size_t
        L.orc_fse_optimal_table_log.restype = ctypes.c_uint32
        L.orc_compress_frame_ck.restype = ctypes.c_size_t
        L.orc_compress_frame_ck.argtypes = [vp, ctypes.c_size_t, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.orc_compress_frame_dict.restype = ctypes.c_size_t
        L.orc_compress_frame_dict.argtypes = [vp, ctypes.c_size_t, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, vp,
                                              ctypes.c_size_t]
        L.orc_compress_frame_lv.restype = ctypes.c_size_t
        L.orc_compress_frame_lv.argtypes = [vp, ctypes.c_size_t, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, vp,
                                            ctypes.c_size_t, ctypes.c_int]
        L.orc_dict_layout.restype = ctypes.c_int
        L.orc_dict_layout.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_size_t)]
        L.orc_xxh64.restype = ctypes.c_uint64
        L.orc_xxh64.argtypes = [vp, ctypes.c_uint64]
        _o = L
    return _o


def datagen():
    global _d
    if _d is None:
        _d = ctypes.CDLL(DATAGEN_SO)
    return _d


# RTLD_DEEPBIND: the image's calls to its own exported functions bind inside that image.  A
# process can hold two libzstd images -- this one (by path, 1.4.9) and the system's 1.4.8 in the
# global scope when a preloaded tool links it (rocprofv3's libraries do) -- and without it the
# library's PLT calls (ZSTD_freeCCtx's frees among them) resolved into the other image's 1.4.8
# code and layouts: the r04f SIGSEGV in free <- ZSTD_freeCCtx under the profiler.
# AddressSanitizer refuses RTLD_DEEPBIND dlopens: a sanitizer run sets ZH_NO_DEEPBIND=1.
LIBZSTD_MODE = os.RTLD_NOW | os.RTLD_LOCAL | (0 if os.environ.get("ZH_NO_DEEPBIND") else getattr(os, "RTLD_DEEPBIND", 0))


def find_libzstd():
    for p in ("/opt/conda/lib/libzstd.so.1", "libzstd.so.1", "/usr/lib/x86_64-linux-gnu/libzstd.so.1"):
        try:
            return ctypes.CDLL(p, mode=LIBZSTD_MODE)
        except OSError:
            continue
    return None


def libzstd_images():
    """Paths of the libzstd images mapped into this process (/proc/self/maps)."""
    out = []
    try:
        for line in open("/proc/self/maps"):
            f = line.split()
            if len(f) >= 6 and "libzstd" in f[5] and f[5] not in out:
                out.append(f[5])
    except OSError:
        pass
    return out


def zstd():
    global _z
    if _z is None:
        L = find_libzstd()
        if L is None:
            return None
        L.ZSTD_decompress.restype = ctypes.c_size_t
        L.ZSTD_compress.restype = ctypes.c_size_t
        L.ZSTD_isError.restype = ctypes.c_uint
        L.ZSTD_getErrorName.restype = ctypes.c_char_p
        L.ZSTD_versionNumber.restype = ctypes.c_uint
        _z = L
    return _z


def gen(kind, nchunks, seed, chunk_size=65536, first=0):
    a = np.zeros(nchunks * chunk_size, np.uint8)
    datagen().dg_fill(a.ctypes.data_as(vp), ctypes.c_size_t(nchunks), ctypes.c_size_t(chunk_size), ctypes.c_uint64(seed),
                      ctypes.c_int(kind), ctypes.c_uint64(first))
    return a


def level_window_log(level):
    """Window log of a level (apply_level_parameters, zh_host.cpp; reference src/cuda_zstd_types.cpp:860-950)."""
    return 18 if level <= 1 else 19 if level <= 3 else 20 if level <= 6 else 22 if level <= 9 else 23


def oracle_frame(data, block_size=128 * 1024, window_log=None, checksum=False, dictionary=None, level=3):
    if window_log is None:
        window_log = level_window_log(level)
    data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data)
    cap = int(oracle().orc_max_compressed_size(ctypes.c_uint64(len(data)))) + 64
    out = np.zeros(cap, np.uint8)
    d = np.frombuffer(bytes(dictionary), np.uint8).copy() if dictionary else None
    n = oracle().orc_compress_frame_lv(out.ctypes.data_as(vp), cap, data.ctypes.data_as(vp), len(data), block_size, window_log, int(checksum),
                                       d.ctypes.data_as(vp) if d is not None else None, 0 if d is None else len(d), level)
    assert n > 0
    return out[:n].tobytes()


def zstd_decompress(frame, size, dictionary=None):
    z = zstd()
    assert z is not None, "libzstd not available"
    src = np.frombuffer(frame, np.uint8).copy()
    dst = np.zeros(max(size, 1), np.uint8)
    if dictionary is None:
        r = z.ZSTD_decompress(dst.ctypes.data_as(vp), ctypes.c_size_t(len(dst)), src.ctypes.data_as(vp), ctypes.c_size_t(len(src)))
    else:  # ZSTD_decompress_usingDict: raw content or a formatted dictionary
        z.ZSTD_createDCtx.restype = vp
        z.ZSTD_freeDCtx.argtypes = [vp]
        z.ZSTD_decompress_usingDict.restype = ctypes.c_size_t
        z.ZSTD_decompress_usingDict.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp, ctypes.c_size_t]
        dct = np.frombuffer(bytes(dictionary), np.uint8).copy()
        dctx = z.ZSTD_createDCtx()
        r = z.ZSTD_decompress_usingDict(dctx, dst.ctypes.data, len(dst), src.ctypes.data, len(src), dct.ctypes.data, len(dct))
        z.ZSTD_freeDCtx(dctx)
    if z.ZSTD_isError(r):
        raise AssertionError("libzstd: " + z.ZSTD_getErrorName(r).decode())
    return dst[:r].tobytes()


def zstd_compress(data, level=3, checksum=False, content_size=True, window_log=0):
    """libzstd frame of `data` (ZSTD_compress2 with the given frame parameters).
    ZSTD_cParameter values of zstd.h 1.4.x: compressionLevel 100, windowLog 101,
    contentSizeFlag 200, checksumFlag 201."""
    z = zstd()
    assert z is not None, "libzstd not available"
    z.ZSTD_createCCtx.restype = vp
    z.ZSTD_freeCCtx.argtypes = [vp]
    z.ZSTD_CCtx_setParameter.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    z.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
    z.ZSTD_compress2.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t]
    z.ZSTD_compress2.restype = ctypes.c_size_t
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    src = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
    cctx = z.ZSTD_createCCtx()
    params = [(100, level), (201, int(checksum)), (200, int(content_size))] + ([(101, window_log)] if window_log else [])
    for p, v in params:
        assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cctx, p, v))
    cap = int(z.ZSTD_compressBound(ctypes.c_size_t(len(src)))) + 64
    out = np.zeros(cap, np.uint8)
    r = z.ZSTD_compress2(cctx, out.ctypes.data, cap, src.ctypes.data if len(src) else None, len(src))
    z.ZSTD_freeCCtx(cctx)
    assert not z.ZSTD_isError(r), z.ZSTD_getErrorName(r)
    return out[:r].tobytes()


def special_inputs():
    """Edge cases the reference tests exercise (tests/test_compressible_data.cu:22-101,
    tests/test_c_api_edge_cases.cu): tiny, ragged, zeros, 0xFF, periodic, random."""
    rng = np.random.default_rng(42)
    out = {
        "one": np.array([7], np.uint8),
        "seven": np.frombuffer(b"abcdefg", np.uint8).copy(),
        "nine": np.frombuffer(b"abcdefghi", np.uint8).copy(),
        "two_same": np.array([5, 5], np.uint8),
        "zeros_64k": np.zeros(65536, np.uint8),
        "ff_64k": np.full(65536, 255, np.uint8),
        "period8_64k": np.tile(np.arange(8, dtype=np.uint8), 8192),
        "iota_4k": (np.arange(4097) % 256).astype(np.uint8),
        "random_64k": rng.integers(0, 256, 65536, dtype=np.uint8),
        "random_300": rng.integers(0, 256, 300, dtype=np.uint8),
        "text_ragged": gen(DG_TEXT, 1, 11, 40001),
        "json_4095": gen(DG_JSON, 1, 12, 4095),
        "csv_65535": gen(DG_CSV, 1, 13, 65535),
        "exe_777": gen(DG_EXE, 1, 14, 777),
        "sensor_64k": gen(DG_SENSOR, 1, 15, 65536),
        "sym16_64k": gen(DG_SYM16, 1, 0x5EED0002, 65536),
        "long_repeat": np.tile(rng.integers(0, 256, 1000, dtype=np.uint8), 66)[:65536].copy(),
        "runs": np.repeat(rng.integers(0, 4, 700, dtype=np.uint8), 97)[:65536].copy(),
    }
    return out


def dict_layout(buf):
    """(Dictionary_ID, content offset) by the oracle's RFC 8878 §5 parser; None if malformed."""
    b = np.frombuffer(bytes(buf), np.uint8).copy()
    did, off = ctypes.c_uint32(), ctypes.c_size_t()
    r = oracle().orc_dict_layout(b.ctypes.data_as(vp), len(b), ctypes.byref(did), ctypes.byref(off))
    return None if r else (did.value, off.value)


def zdict_train(samples, capacity):
    """libzstd ZDICT_trainFromBuffer (a formatted dictionary) over host samples."""
    z = zstd()
    assert z is not None, "libzstd not available"
    z.ZDICT_trainFromBuffer.restype = ctypes.c_size_t
    z.ZDICT_trainFromBuffer.argtypes = [vp, ctypes.c_size_t, vp, ctypes.POINTER(ctypes.c_size_t), ctypes.c_uint]
    z.ZDICT_isError.restype = ctypes.c_uint
    raw = [bytes(s) for s in samples]
    buf = np.frombuffer(b"".join(raw), np.uint8).copy()
    sizes = (ctypes.c_size_t * len(raw))(*[len(r) for r in raw])
    out = np.zeros(capacity, np.uint8)
    r = z.ZDICT_trainFromBuffer(out.ctypes.data_as(vp), capacity, buf.ctypes.data_as(vp), sizes, len(raw))
    assert not z.ZDICT_isError(r), "ZDICT_trainFromBuffer failed"
    return out[:r].tobytes()


def zstd_compress_dict(data, dictionary, level=3):
    """libzstd ZSTD_compress_usingDict frame of `data`."""
    z = zstd()
    assert z is not None, "libzstd not available"
    z.ZSTD_createCCtx.restype = vp
    z.ZSTD_freeCCtx.argtypes = [vp]
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compress_usingDict.restype = ctypes.c_size_t
    z.ZSTD_compress_usingDict.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.c_int]
    src = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
    dct = np.frombuffer(bytes(dictionary), np.uint8).copy()
    cap = int(z.ZSTD_compressBound(ctypes.c_size_t(len(src)))) + 64
    out = np.zeros(cap, np.uint8)
    cctx = z.ZSTD_createCCtx()
    r = z.ZSTD_compress_usingDict(cctx, out.ctypes.data, cap, src.ctypes.data if len(src) else None, len(src), dct.ctypes.data, len(dct), level)
    z.ZSTD_freeCCtx(cctx)
    assert not z.ZSTD_isError(r), z.ZSTD_getErrorName(r)
    return out[:r].tobytes()
