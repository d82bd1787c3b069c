"""The Python binding against the reference's own Python tests (python/tests/test_basic.py:
round trips of bytes / bytearray / memoryview / numpy, levels, Manager as a context manager,
batches, HybridEngine, errors, edge cases) and the F4 streaming manager: chunks compressed with
the stream's history are byte-identical to the oracle's frame with that history as a raw-content
dictionary, decode with libzstd ZSTD_decompress_usingDict, and decode in order on the GPU."""
import numpy as np
import pytest

import zh_testlib as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cz():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import cuda_zstd

    return cuda_zstd


SMALL = b"hello world! " * 80


def test_roundtrip_host_types(cz):
    medium = T.gen(T.DG_TEXT, 1, 1, 100_000).tobytes()
    large = T.gen(T.DG_MIX, 1, 2, 3_000_000).tobytes()
    for d in (SMALL, medium, large):
        c = cz.compress(d)
        assert isinstance(c, bytes) and c == T.oracle_frame(np.frombuffer(d, np.uint8))
        assert cz.decompress(c) == d
    assert cz.decompress(cz.compress(bytearray(SMALL))) == SMALL
    assert cz.decompress(cz.compress(memoryview(SMALL))) == SMALL
    a = np.frombuffer(medium, np.uint8)
    assert cz.decompress(cz.compress(a)) == medium


@pytest.mark.parametrize("level", [1, 3, 9, 19])
def test_levels_roundtrip(cz, level):
    d = T.gen(T.DG_JSON, 1, 3, 70_000).tobytes()
    assert cz.decompress(cz.compress(d, level=level)) == d


def test_manager_context_batch_and_close(cz):
    batch = [T.gen(k, 1, 10 + k, s).tobytes() for k, s in ((T.DG_TEXT, 5000), (T.DG_CSV, 65536), (T.DG_EXE, 1), (T.DG_MIX, 200_000))]
    with cz.Manager(level=3) as m:
        assert m.get_level() == 3 and "level=3" in repr(m)
        cs = m.compress_batch(batch)
        assert [len(c) for c in cs] and all(isinstance(c, bytes) for c in cs)
        assert m.decompress_batch(cs) == batch
    assert cz.decompress_batch(cz.compress_batch(batch)) == batch
    m = cz.Manager(3)
    m.close()
    with pytest.raises(RuntimeError):
        m.compress(b"data")


def test_errors_and_edges(cz):
    with pytest.raises(RuntimeError):
        cz.decompress(b"this is not compressed data!!!")
    c = cz.compress(SMALL)
    with pytest.raises(RuntimeError):
        cz.decompress(c[: len(c) // 2])
    assert cz.decompress(cz.compress(b"x")) == b"x"
    z = b"\x00" * 100_000
    cz_ = cz.compress(z)
    assert len(cz_) < len(z) // 10 and cz.decompress(cz_) == z
    allb = bytes(range(256)) * 40
    assert cz.decompress(cz.compress(allb)) == allb
    assert cz.validate_compressed_data(c) and not cz.validate_compressed_data(b"nope nope")
    assert cz.estimate_compressed_size(65536) == 65536 + 257 + 3 + 512
    assert cz.is_cuda_available() and cz.get_cuda_device_info()["total_memory"] > 0
    assert (cz.MIN_LEVEL, cz.MAX_LEVEL, cz.DEFAULT_LEVEL) == (1, 22, 3)


def test_hybrid_engine(cz, libzstd):
    d = T.gen(T.DG_TEXT, 1, 0x5EED0001, 1 << 20).tobytes()
    with cz.HybridEngine(3) as e:
        c = e.compress(d)
        assert e.decompress(c) == d
        assert e.last_result.backend_used in (cz.CPU_LIBZSTD, cz.GPU_KERNELS, cz.CPU_PARALLEL)
        assert T.zstd_decompress(c, len(d)) == d
    for mode in (cz.FORCE_CPU, cz.FORCE_GPU):
        e = cz.HybridEngine(cz.HybridConfig(mode, 1 << 20, 0, 3, 0, 0))
        c = e.compress(d)
        assert e.last_result.backend_used == (cz.CPU_LIBZSTD if mode == cz.FORCE_CPU else cz.GPU_KERNELS)
        if mode == cz.FORCE_GPU:
            assert c == T.oracle_frame(np.frombuffer(d, np.uint8))
        assert cz.hybrid_decompress(c) == d
    assert cz.hybrid_decompress(cz.hybrid_compress(SMALL)) == SMALL


def test_metadata_frame_on_device(cz):
    import torch

    d = T.gen(T.DG_MIX, 1, 11, 200_000)
    m = cz.Manager(3)
    f = m.compress(torch.from_numpy(d).cuda())
    blob = torch.cat([torch.frombuffer(bytearray(cz.metadata_frame(7)), dtype=torch.uint8).cuda(), f])
    md = cz.extract_metadata(blob)
    assert md["level"] == 7 and md["uncompressed_size"] == len(d)
    assert m.decompress(blob).cpu().numpy().tobytes() == d.tobytes()


@pytest.mark.parametrize("level", [3, 9])
def test_streaming_with_history(cz, libzstd, level):
    """F4: a 600 KiB JSON-like stream in chunks of mixed sizes; chunk k with history equals
    the oracle frame of chunk k with the last <= 64 KiB of the stream before it as a raw-content
    dictionary, decodes with libzstd using that history, and the streaming decoder returns the
    stream in order.  With history the stream compresses better than chunk by chunk.  Level 9
    (the deep matcher) stages up to 64 KiB of history + a 64 KiB block: its links stay in the
    global scratch slot (the search's slot-only variant)."""
    import torch

    stream = T.gen(T.DG_JSON, 1, 0x5EED0005, 600_000)
    sizes = [10_000, 30_000, 65_536, 100_000, 1, 40_000, 200_000, 16_384]
    sizes.append(len(stream) - sum(sizes))
    s = cz.StreamingManager(level)
    plain = cz.StreamingManager(level)
    frames, pos, tot_h, tot_p = [], 0, 0, 0
    for n in sizes:
        chunk = stream[pos:pos + n]
        hist = stream[max(0, pos - 65536):pos].tobytes()
        f = s.compress_chunk(torch.from_numpy(chunk.copy()).cuda(), with_history=True).cpu().numpy().tobytes()
        assert f == T.oracle_frame(chunk, dictionary=hist if hist else None, level=level), (pos, n)
        assert T.zstd_decompress(f, n, dictionary=hist if hist else None) == chunk.tobytes()
        tot_h += len(f)
        tot_p += plain.compress_chunk(torch.from_numpy(chunk.copy()).cuda(), with_history=False).numel()
        frames.append(f)
        pos += n
    assert tot_h < tot_p
    d = cz.StreamingManager(3)
    back = b"".join(d.decompress_chunk(torch.frombuffer(bytearray(f), dtype=torch.uint8).cuda()).cpu().numpy().tobytes() for f in frames)
    assert back == stream.tobytes()
