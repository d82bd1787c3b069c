"""Decoder fixtures on the CPU (no GPU): the committed libzstd frames
(tests/golden/decode_frames.json, made by tests/golden/make_decode_golden.py) decode with
libzstd to the recorded digests, and together they reach every decoder path of
zh_decode.hip (block types, literal types, stream counts, weight encodings, the four
sequence-table modes for each table, checksum, frames without content size, window
descriptors).  The GPU test (test_gpu_decode.py) decodes the same frames."""
import ctypes
import hashlib
import json
import os

import pytest

import zh_frames as F
import zh_testlib as T

FIX = os.path.join(T.GOLDEN, "decode_frames.json")

ALL_PATHS = {"block_compressed", "block_raw", "block_rle", "checksum", "huf_1stream", "huf_4stream", "lit_huffman", "lit_raw", "lit_rle",
             "lit_treeless", "ll_fse", "ll_predefined", "ll_repeat", "ll_rle", "ml_fse", "ml_predefined", "ml_repeat", "ml_rle", "no_fcs",
             "no_sequences", "of_fse", "of_predefined", "of_repeat", "of_rle", "weights_direct", "weights_fse", "window_descriptor"}


def vectors():
    return json.load(open(FIX))["vectors"]


def test_fixture_covers_every_decoder_path():
    frames = [bytes.fromhex(v["frame"]) for v in vectors() if "expect_error" not in v]
    assert F.features(frames) >= ALL_PATHS, ALL_PATHS - F.features(frames)


def test_fixture_digests_with_libzstd(libzstd):
    for v in vectors():
        frame = bytes.fromhex(v["frame"])
        if "expect_error" in v:
            with pytest.raises(AssertionError):
                T.zstd_decompress(frame, 1 << 16)
            continue
        out = T.zstd_decompress(frame, max(v["size"], 1))
        assert len(out) == v["size"] and hashlib.sha256(out).hexdigest() == v["sha256"], v["name"]


def test_walker_on_own_frames():
    """The oracle's (= the GPU compressor's) frames: single segment, no checksum, 64 KiB
    blocks; RLE blocks for constant input."""
    zeros = F.walk(T.oracle_frame(bytes(65536)))
    assert [b["type"] for b in zeros] == ["rle"]
    text = F.walk(T.oracle_frame(T.gen(T.DG_TEXT, 1, 1, 65536)))
    assert text[0]["type"] == "compressed" and text[0]["lit"] == "huffman" and text[0]["streams"] == 4


def test_decompress_workspace_sizes():
    import cuda_zstd

    L = cuda_zstd.lib()
    m = L.cuda_zstd_create_manager(3)
    one = L.cuda_zstd_get_decompress_workspace_size(m, 1000)
    assert 128 * 1024 < one < 1 << 20  # one slot: 128 KiB of literals + sequence records
    n = 16
    sizes = (ctypes.c_size_t * n)(*([1000] * n))
    assert L.cuda_zstd_get_batch_decompress_workspace_size(m, sizes, n) < n * one + 4096
    small = L.nvcomp_zstd_batched_decompress_get_temp_size_v5(n, 65536)
    assert small < L.nvcomp_zstd_batched_decompress_get_temp_size_v5(n, 1 << 20)  # slots sized by the chunk bound
    L.cuda_zstd_destroy_manager(m)
