"""Python binding of libcuda_zstd_hip.so (gfx950 Zstandard compressor).

Mirrors the reference's Python package (python/cuda_zstd/__init__.py:90-120,
python/src/binding.cpp:151-976): ``Manager`` (compress / decompress /
compress_batch / decompress_batch), ``HybridEngine``, module-level ``compress``,
``decompress``, ``compress_batch``, ``decompress_batch``, ``hybrid_compress``,
``hybrid_decompress``, ``validate_compressed_data``, ``estimate_compressed_size``,
``is_cuda_available``, ``get_cuda_device_info`` and the level constants -- plus a
``StreamingManager`` and the dictionary / batched device entries, all over the
library's C ABI (include/cuda_zstd_capi.h).  Host inputs (bytes, bytearray, numpy)
give host ``bytes`` back, as the reference's binding does; torch device tensors stay
on the device.  PyTorch is only used for device memory and streams.

The product path never falls back to a CPU implementation: if the shared
library or a GPU is missing, every call raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CUDA_ZSTD_HIP_LIB") or os.path.join(os.path.dirname(_HERE), "libcuda_zstd_hip.so")

# nvcomp-style return codes (reference src/cuda_zstd_nvcomp.cpp:75-96)
OK, INVALID, OOM, DEVICE_ERROR, CORRUPT, TOO_SMALL, CHECKSUM, COMPRESSION = 0, 2, 3, 4, 6, 7, 10, 12

_lib = None


class ZstdError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {error_string(code)} (code {code})")


def lib() -> ctypes.CDLL:
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with __graft_entry__.build() (make -C custom-nvcomp-with-zstd_amd)")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        psz, pvp, pi = ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(i)
        sig = {
            "cuda_zstd_create_manager": (vp, [i]),
            "cuda_zstd_destroy_manager": (None, [vp]),
            "cuda_zstd_compress": (i, [vp, vp, sz, vp, psz, vp, sz, vp]),
            "cuda_zstd_decompress": (i, [vp, vp, sz, vp, psz, vp, sz, vp]),
            "cuda_zstd_get_compress_workspace_size": (sz, [vp, sz]),
            "cuda_zstd_get_decompress_workspace_size": (sz, [vp, sz]),
            "cuda_zstd_get_max_compressed_size": (sz, [vp, sz]),
            "cuda_zstd_get_batch_compress_workspace_size": (sz, [vp, psz, sz]),
            "cuda_zstd_compress_batch": (i, [vp, pvp, psz, sz, pvp, psz, pi, vp, sz, vp]),
            "cuda_zstd_get_error_string": (ctypes.c_char_p, [i]),
            "cuda_zstd_is_error": (i, [i]),
            "cuda_zstd_train_dictionary": (vp, [pvp, psz, sz, sz]),
            "cuda_zstd_load_dictionary": (vp, [vp, sz]),
            "cuda_zstd_destroy_dictionary": (None, [vp]),
            "cuda_zstd_set_dictionary": (i, [vp, vp]),
            "cuda_zstd_clear_dictionary": (i, [vp]),
            "cuda_zstd_get_dictionary_content": (sz, [vp, vp, sz]),
            "cuda_zstd_get_dictionary_layout": (i, [vp, ctypes.POINTER(ctypes.c_uint), psz]),
            "nvcomp_zstd_batch_create_v5": (vp, [i, ctypes.c_uint, i]),
            "nvcomp_zstd_batch_destroy_v5": (None, [vp]),
            "nvcomp_zstd_batch_get_compress_temp_size_v5": (sz, [vp, psz, sz]),
            "nvcomp_zstd_batch_get_max_compressed_chunk_size_v5": (sz, [vp, sz]),
            "nvcomp_zstd_batch_compress_async_v5": (i, [vp, vp, vp, sz, vp, vp, vp, sz, vp]),
            "nvcomp_zstd_batched_compress_get_temp_size_v5": (sz, [sz, sz]),
            "nvcomp_zstd_batch_get_batched_temp_size_v5": (sz, [vp, sz, sz]),
            "nvcomp_zstd_batch_set_dictionary_v5": (i, [vp, vp]),
            "nvcomp_zstd_batched_compress_async_v5": (i, [vp, vp, vp, sz, sz, vp, vp, vp, vp, sz, vp]),
            "cuda_zstd_get_batch_decompress_workspace_size": (sz, [vp, psz, sz]),
            "cuda_zstd_decompress_batch": (i, [vp, pvp, psz, sz, pvp, psz, pi, vp, sz, vp]),
            "nvcomp_zstd_batch_get_decompress_temp_size_v5": (sz, [vp, psz, sz]),
            "nvcomp_zstd_batch_decompress_async_v5": (i, [vp, vp, vp, sz, vp, vp, vp, sz, vp]),
            "nvcomp_zstd_batched_decompress_get_temp_size_v5": (sz, [sz, sz]),
            "nvcomp_zstd_batched_decompress_async_v5": (i, [vp, vp, vp, vp, sz, sz, vp, vp, vp, vp, sz, vp]),
            "cuda_zstd_write_metadata_frame": (i, [vp, sz, i, psz, vp]),
            "cuda_zstd_stream_create": (vp, [i]),
            "cuda_zstd_stream_destroy": (None, [vp]),
            "cuda_zstd_stream_compress_chunk": (i, [vp, vp, sz, vp, psz, i, i, vp]),
            "cuda_zstd_stream_decompress_chunk": (i, [vp, vp, sz, vp, psz, pi, vp]),
            "cuda_zstd_stream_reset": (i, [vp]),
            "cuda_zstd_hybrid_create": (vp, [vp]),
            "cuda_zstd_hybrid_create_default": (vp, []),
            "cuda_zstd_hybrid_destroy": (None, [vp]),
            "cuda_zstd_hybrid_compress": (i, [vp, vp, sz, vp, psz, ctypes.c_uint, ctypes.c_uint, vp, vp]),
            "cuda_zstd_hybrid_decompress": (i, [vp, vp, sz, vp, psz, ctypes.c_uint, ctypes.c_uint, vp, vp]),
            "cuda_zstd_hybrid_max_compressed_size": (sz, [vp, sz]),
            "cuda_zstd_hybrid_query_routing": (ctypes.c_uint, [vp, sz, ctypes.c_uint, ctypes.c_uint, i]),
            "cuda_zstd_extract_metadata": (i, [vp, sz, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint), pi]),
            "cuda_zstd_hip_version": (ctypes.c_char_p, []),
            "cuda_zstd_hip_profile_enable": (None, [i]),
            "cuda_zstd_hip_profile_collect": (i, [ctypes.POINTER(ctypes.c_double)]),
            "cuda_zstd_hip_kernel_lds_bytes": (ctypes.c_uint, [i]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def error_string(code: int) -> str:
    return lib().cuda_zstd_get_error_string(code).decode()


def _torch():
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError("cuda_zstd: no GPU visible (the gfx950 path has no CPU fallback)")
    return torch


def _stream_ptr(stream) -> int:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def max_compressed_size(n: int) -> int:
    """reference estimate_compressed_size (src/cuda_zstd_types.cpp:831-853)."""
    nb = max(1, (n + 128 * 1024 - 1) // (128 * 1024))
    return n + n // 255 + nb * 3 + 512


MIN_LEVEL, MAX_LEVEL, DEFAULT_LEVEL = 1, 22, 3
__version__ = "0.2.0"


def _is_host(x) -> bool:
    return isinstance(x, (bytes, bytearray, memoryview)) or type(x).__module__.startswith("numpy")


def _to_device(x):
    """Host bytes-like / numpy -> uint8 device tensor (the reference binding's H2D)."""
    torch = _torch()
    import numpy as np

    a = np.frombuffer(bytes(x), np.uint8) if isinstance(x, (bytes, bytearray, memoryview)) else np.ascontiguousarray(x).view(np.uint8).reshape(-1)
    if a.size == 0:
        return torch.empty(0, dtype=torch.uint8, device="cuda")
    return torch.from_numpy(a.copy()).cuda()


def _host_bytes(t) -> bytes:
    return t.cpu().numpy().tobytes() if t.numel() else b""


def _frame_size(frame) -> int:
    """Content size from the frame header (after any skippable frames), like the reference's
    get_decompressed_size path of PyManager.decompress; 16x the input when it is absent."""
    try:
        return extract_metadata(frame)["uncompressed_size"] or frame.numel() * 16
    except ZstdError:
        return max(frame.numel() * 16, 1024)


class Manager:
    """C-ABI manager handle (reference PyManager, python/src/binding.cpp:151-329).

    Device tensors in -> device tensors out; host bytes / numpy in -> bytes out."""

    def __init__(self, level: int = 3):
        self.level = level
        self._h = lib().cuda_zstd_create_manager(level)
        if not self._h:
            raise ZstdError(INVALID, "cuda_zstd_create_manager")
        self._ws = None

    def close(self):
        if self._h:
            lib().cuda_zstd_destroy_manager(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown: module globals may already be gone
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __repr__(self):
        return f"<cuda_zstd.Manager level={self.level}>"

    def get_level(self) -> int:
        return self.level

    def _workspace(self, nbytes: int):
        torch = _torch()
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device="cuda")
        return self._ws

    def compress(self, data, stream=None):
        """Compress a contiguous uint8 device tensor into one zstd frame (device tensor); host
        bytes-like / numpy input gives bytes (reference PyManager.compress)."""
        if _is_host(data):
            return _host_bytes(self.compress(_to_device(data), stream))
        torch = _torch()
        data = data.contiguous().view(torch.uint8)
        n = data.numel()
        out = torch.empty(max_compressed_size(n), dtype=torch.uint8, device=data.device)
        ws_n = lib().cuda_zstd_get_compress_workspace_size(self._h, n)
        ws = self._workspace(ws_n)
        size = ctypes.c_size_t(out.numel())
        rc = lib().cuda_zstd_compress(self._h, data.data_ptr(), n, out.data_ptr(), ctypes.byref(size), ws.data_ptr(), ws.numel(), _stream_ptr(stream))
        if rc:
            raise ZstdError(rc, "cuda_zstd_compress")
        return out[: size.value]

    def compress_batch(self, chunks: Sequence, stream=None) -> List:
        """ZstdBatchManager::compress_batch over a list of uint8 device tensors (host inputs:
        a list of bytes back)."""
        if len(chunks) and all(_is_host(c) for c in chunks):
            return [_host_bytes(o) for o in self.compress_batch([_to_device(c) for c in chunks], stream)]
        torch = _torch()
        n = len(chunks)
        ins = [c.contiguous().view(torch.uint8) for c in chunks]
        sizes = [t.numel() for t in ins]
        caps = [max_compressed_size(s) for s in sizes]
        offs = [0]
        for c in caps:
            offs.append(offs[-1] + ((c + 255) // 256) * 256)
        out = torch.empty(offs[-1], dtype=torch.uint8, device="cuda")
        in_ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
        out_ptrs = (ctypes.c_void_p * n)(*[out.data_ptr() + o for o in offs[:-1]])
        in_sz = (ctypes.c_size_t * n)(*sizes)
        out_sz = (ctypes.c_size_t * n)(*caps)
        st = (ctypes.c_int * n)()
        ws_n = lib().cuda_zstd_get_batch_compress_workspace_size(self._h, in_sz, n)
        ws = self._workspace(ws_n)
        rc = lib().cuda_zstd_compress_batch(self._h, in_ptrs, in_sz, n, out_ptrs, out_sz, st, ws.data_ptr(), ws.numel(), _stream_ptr(stream))
        if rc and all(s == OK for s in st):
            raise ZstdError(rc, "cuda_zstd_compress_batch")
        res = []
        for k in range(n):
            if st[k] != OK:
                raise ZstdError(st[k], f"cuda_zstd_compress_batch item {k}")
            res.append(out[offs[k] : offs[k] + out_sz[k]])
        return res


    def set_dictionary(self, d: "Dictionary"):
        """ZstdManager::set_dictionary: later compress / decompress calls use `d`."""
        rc = lib().cuda_zstd_set_dictionary(self._h, d._h)
        if rc:
            raise ZstdError(rc, "cuda_zstd_set_dictionary")

    def clear_dictionary(self):
        rc = lib().cuda_zstd_clear_dictionary(self._h)
        if rc:
            raise ZstdError(rc, "cuda_zstd_clear_dictionary")

    def decompress(self, frame, capacity: int = None, stream=None):
        """GPU-decode one device buffer (frames, concatenated) into a new device tensor of
        at most `capacity` bytes (cuda_zstd_decompress); capacity None: the frame header's
        content size.  Host bytes in -> bytes out (reference PyManager.decompress)."""
        if _is_host(frame):
            return _host_bytes(self.decompress(_to_device(frame), capacity, stream))
        auto = capacity is None
        if auto:
            capacity = _frame_size(frame)
        torch = _torch()
        frame = frame.contiguous().view(torch.uint8)
        # a derived capacity (the first frame's content size, or 16x the input without one)
        # grows on BUFFER_TOO_SMALL: concatenated frames, frames without a content size
        for _ in range(4 if auto else 1):
            out = torch.empty(max(capacity, 1), dtype=torch.uint8, device=frame.device)
            ws = self._workspace(lib().cuda_zstd_get_decompress_workspace_size(self._h, frame.numel()))
            size = ctypes.c_size_t(capacity)
            rc = lib().cuda_zstd_decompress(self._h, frame.data_ptr(), frame.numel(), out.data_ptr(), ctypes.byref(size), ws.data_ptr(),
                                            ws.numel(), _stream_ptr(stream))
            if rc == TOO_SMALL and auto:
                capacity *= 4
                continue
            if rc:
                raise ZstdError(rc, "cuda_zstd_decompress")
            return out[: size.value]
        raise ZstdError(TOO_SMALL, "cuda_zstd_decompress")

    def decompress_batch(self, frames: Sequence, capacities: Sequence[int] = None, stream=None, raise_on_error=True):
        """ZstdBatchManager::decompress_batch over device tensors: one GPU launch for all.
        Returns the decoded tensors (and, with raise_on_error=False, the nvcomp codes).
        capacities None: each frame header's content size; host inputs give bytes back."""
        if len(frames) and all(_is_host(f) for f in frames):
            outs = self.decompress_batch([_to_device(f) for f in frames], capacities, stream, raise_on_error)
            if raise_on_error:
                return [_host_bytes(o) for o in outs]
            return [_host_bytes(o) for o in outs[0]], outs[1]
        if capacities is None:
            capacities = [_frame_size(f) for f in frames]
        torch = _torch()
        n = len(frames)
        ins = [f.contiguous().view(torch.uint8) for f in frames]
        offs = [0]
        for c in capacities:
            offs.append(offs[-1] + ((max(c, 1) + 255) // 256) * 256)
        out = torch.empty(max(offs[-1], 256), dtype=torch.uint8, device="cuda")
        in_ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
        out_ptrs = (ctypes.c_void_p * n)(*[out.data_ptr() + o for o in offs[:-1]])
        in_sz = (ctypes.c_size_t * n)(*[t.numel() for t in ins])
        out_sz = (ctypes.c_size_t * n)(*capacities)
        st = (ctypes.c_int * n)()
        ws = self._workspace(lib().cuda_zstd_get_batch_decompress_workspace_size(self._h, in_sz, n))
        rc = lib().cuda_zstd_decompress_batch(self._h, in_ptrs, in_sz, n, out_ptrs, out_sz, st, ws.data_ptr(), ws.numel(), _stream_ptr(stream))
        if rc and all(s == OK for s in st):
            raise ZstdError(rc, "cuda_zstd_decompress_batch")
        res = [out[offs[k] : offs[k] + out_sz[k]] for k in range(n)]
        if raise_on_error:
            for k in range(n):
                if st[k] != OK:
                    raise ZstdError(st[k], f"cuda_zstd_decompress_batch item {k}")
            return res
        return res, list(st)


class Dictionary:
    """Dictionary handle (reference dictionary::Dictionary, include/cuda_zstd_dictionary.h:101;
    DictionaryTrainer::train_dictionary, DictionaryManager::load_dictionary :292).  Raw content,
    or a formatted RFC 8878 §5 dictionary such as ZDICT_trainFromBuffer's."""

    def __init__(self, handle, what: str = "dictionary"):
        if not handle:
            raise ZstdError(INVALID, what)
        self._h = handle

    @classmethod
    def train(cls, samples, dict_size: int) -> "Dictionary":
        """COVER training over host samples (bytes-like / uint8 arrays) -> raw content."""
        raw = [bytes(s) for s in samples]
        bufs = [ctypes.create_string_buffer(b, max(len(b), 1)) for b in raw]
        n = len(raw)
        ptrs = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
        sizes = (ctypes.c_size_t * n)(*[len(b) for b in raw])
        return cls(lib().cuda_zstd_train_dictionary(ptrs, sizes, n, dict_size), "cuda_zstd_train_dictionary")

    @classmethod
    def load(cls, buf) -> "Dictionary":
        b = bytes(buf)
        cb = ctypes.create_string_buffer(b, max(len(b), 1))
        return cls(lib().cuda_zstd_load_dictionary(cb, len(b)), "cuda_zstd_load_dictionary")

    def content(self) -> bytes:
        n = lib().cuda_zstd_get_dictionary_content(self._h, None, 0)
        cb = ctypes.create_string_buffer(max(n, 1))
        lib().cuda_zstd_get_dictionary_content(self._h, cb, n)
        return cb.raw[:n]

    def layout(self):
        """(Dictionary_ID, content offset); (0, 0) for raw content."""
        did, off = ctypes.c_uint(), ctypes.c_size_t()
        rc = lib().cuda_zstd_get_dictionary_layout(self._h, ctypes.byref(did), ctypes.byref(off))
        if rc:
            raise ZstdError(rc, "cuda_zstd_get_dictionary_layout")
        return did.value, off.value

    def close(self):
        if self._h:
            lib().cuda_zstd_destroy_dictionary(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


class BatchedDecompressor:
    """Stream-ordered batched GPU decompression over device arrays
    (nvcomp_zstd_batched_decompress_async_v5).  Used by bench.py --decompress."""

    def __init__(self):
        self._h = lib().nvcomp_zstd_batch_create_v5(3, 64 * 1024, 0)
        if not self._h:
            raise ZstdError(INVALID, "nvcomp_zstd_batch_create_v5")

    def close(self):
        if self._h:
            lib().nvcomp_zstd_batch_destroy_v5(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def temp_size(num_chunks: int, max_out: int) -> int:
        return lib().nvcomp_zstd_batched_decompress_get_temp_size_v5(num_chunks, max_out)

    def decompress_async(self, d_in_ptrs, d_in_sizes, d_out_caps, max_out, d_out_ptrs, d_out_sizes, d_status, temp, stream=None):
        n = d_in_ptrs.numel()
        rc = lib().nvcomp_zstd_batched_decompress_async_v5(
            self._h, d_in_ptrs.data_ptr(), d_in_sizes.data_ptr(), d_out_caps.data_ptr() if d_out_caps is not None else None, max_out, n,
            d_out_ptrs.data_ptr(), d_out_sizes.data_ptr(), d_status.data_ptr() if d_status is not None else None, temp.data_ptr(), temp.numel(),
            _stream_ptr(stream))
        if rc:
            raise ZstdError(rc, "nvcomp_zstd_batched_decompress_async_v5")


class BatchedCompressor:
    """Stream-ordered batched compression of equal-capacity chunk slots
    (nvcomp_zstd_batched_compress_async_v5).  Used by bench.py."""

    def __init__(self, level: int = 3, chunk_size: int = 64 * 1024, checksum: bool = False):
        self._h = lib().nvcomp_zstd_batch_create_v5(level, chunk_size, 1 if checksum else 0)
        if not self._h:
            raise ZstdError(INVALID, "nvcomp_zstd_batch_create_v5")
        self.chunk_size = chunk_size

    def close(self):
        if self._h:
            lib().nvcomp_zstd_batch_destroy_v5(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def temp_size(self, num_chunks: int, max_chunk: int) -> int:
        """Workspace of compress_async for this handle's level and dictionary."""
        return lib().nvcomp_zstd_batch_get_batched_temp_size_v5(self._h, num_chunks, max_chunk)

    def temp_size_for(self, chunk_sizes) -> int:
        """Workspace for these chunk sizes under the handle's current dictionary."""
        n = len(chunk_sizes)
        arr = (ctypes.c_size_t * n)(*chunk_sizes)
        return lib().nvcomp_zstd_batch_get_compress_temp_size_v5(self._h, arr, n)

    def set_dictionary(self, d: "Dictionary"):
        rc = lib().nvcomp_zstd_batch_set_dictionary_v5(self._h, d._h)
        if rc:
            raise ZstdError(rc, "nvcomp_zstd_batch_set_dictionary_v5")

    def max_out(self, max_chunk: int) -> int:
        return lib().nvcomp_zstd_batch_get_max_compressed_chunk_size_v5(self._h, max_chunk)

    def compress_async(self, d_in_ptrs, d_in_sizes, max_chunk, d_out_ptrs, d_out_sizes, d_status, temp, stream=None):
        n = d_in_ptrs.numel()
        rc = lib().nvcomp_zstd_batched_compress_async_v5(
            self._h, d_in_ptrs.data_ptr(), d_in_sizes.data_ptr(), max_chunk, n, d_out_ptrs.data_ptr(), d_out_sizes.data_ptr(),
            d_status.data_ptr() if d_status is not None else None, temp.data_ptr(), temp.numel(), _stream_ptr(stream))
        if rc:
            raise ZstdError(rc, "nvcomp_zstd_batched_compress_async_v5")


class StreamingManager:
    """ZstdStreamingManager over the C ABI (cuda_zstd_stream_*; reference
    include/cuda_zstd_manager.h:300-352).  Each chunk is a complete frame; with_history=True is
    compress_chunk_with_history (the preceding <= 64 KiB of the stream as history, reference
    src/cuda_zstd_manager.cu:6327-6418); decompress_chunk keeps the decoded window, so chunks
    must be decoded in stream order.  Device tensors."""

    def __init__(self, level: int = 3):
        self._h = lib().cuda_zstd_stream_create(level)
        if not self._h:
            raise ZstdError(INVALID, "cuda_zstd_stream_create")

    def close(self):
        if self._h:
            lib().cuda_zstd_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compress_chunk(self, data, with_history: bool = True, is_last: bool = False, stream=None):
        torch = _torch()
        data = data.contiguous().view(torch.uint8)
        out = torch.empty(max_compressed_size(data.numel()), dtype=torch.uint8, device=data.device)
        size = ctypes.c_size_t(out.numel())
        rc = lib().cuda_zstd_stream_compress_chunk(self._h, data.data_ptr(), data.numel(), out.data_ptr(), ctypes.byref(size), int(with_history),
                                                   int(is_last), _stream_ptr(stream))
        if rc:
            raise ZstdError(rc, "cuda_zstd_stream_compress_chunk")
        return out[: size.value]

    def decompress_chunk(self, frame, capacity: int = None, stream=None):
        torch = _torch()
        frame = frame.contiguous().view(torch.uint8)
        auto = capacity is None
        if auto:
            capacity = _frame_size(frame)
        for _ in range(4 if auto else 1):  # (a derived capacity grows on BUFFER_TOO_SMALL)
            out = torch.empty(max(capacity, 1), dtype=torch.uint8, device=frame.device)
            size = ctypes.c_size_t(capacity)
            last = ctypes.c_int()
            rc = lib().cuda_zstd_stream_decompress_chunk(self._h, frame.data_ptr(), frame.numel(), out.data_ptr(), ctypes.byref(size),
                                                         ctypes.byref(last), _stream_ptr(stream))
            if rc == TOO_SMALL and auto:
                capacity *= 4
                continue
            if rc:
                raise ZstdError(rc, "cuda_zstd_stream_decompress_chunk")
            return out[: size.value]
        raise ZstdError(TOO_SMALL, "cuda_zstd_stream_decompress_chunk")

    def reset(self):
        rc = lib().cuda_zstd_stream_reset(self._h)
        if rc:
            raise ZstdError(rc, "cuda_zstd_stream_reset")


# HybridEngine (reference PyHybridEngine, python/src/binding.cpp:331-545, over
# cuda_zstd_hybrid_*): host buffers in and out; the engine routes between libzstd on the host
# and the GPU (cuda_zstd_hybrid_query_routing tells which).
HOST, DEVICE, MANAGED, UNKNOWN = 0, 1, 2, 3  # DataLocation
AUTO, PREFER_CPU, PREFER_GPU, FORCE_CPU, FORCE_GPU, ADAPTIVE = range(6)  # HybridMode
CPU_LIBZSTD, GPU_KERNELS, CPU_PARALLEL = 0, 1, 2  # ExecutionBackend


class HybridConfig(ctypes.Structure):
    """cuda_zstd_hybrid_config_t (reference HybridConfig, include/cuda_zstd_hybrid.h:45-70)."""
    _fields_ = [("mode", ctypes.c_uint), ("cpu_size_threshold", ctypes.c_size_t), ("gpu_device_threshold", ctypes.c_size_t),
                ("compression_level", ctypes.c_int), ("enable_profiling", ctypes.c_int), ("cpu_thread_count", ctypes.c_uint)]


class HybridResult(ctypes.Structure):
    _fields_ = [("backend_used", ctypes.c_uint), ("input_location", ctypes.c_uint), ("output_location", ctypes.c_uint),
                ("total_time_ms", ctypes.c_double), ("transfer_time_ms", ctypes.c_double), ("compute_time_ms", ctypes.c_double),
                ("throughput_mbps", ctypes.c_double), ("input_bytes", ctypes.c_size_t), ("output_bytes", ctypes.c_size_t),
                ("compression_ratio", ctypes.c_float)]


class HybridEngine:
    def __init__(self, level_or_config=3):
        if isinstance(level_or_config, HybridConfig):
            self.config = level_or_config
        else:
            self.config = HybridConfig(AUTO, 1 << 20, 0, int(level_or_config), 0, 0)
        self._h = lib().cuda_zstd_hybrid_create(ctypes.byref(self.config))
        if not self._h:
            raise ZstdError(INVALID, "cuda_zstd_hybrid_create")
        self.last_result = None

    def close(self):
        if self._h:
            lib().cuda_zstd_hybrid_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __repr__(self):
        return f"<cuda_zstd.HybridEngine level={self.config.compression_level}>"

    def get_level(self) -> int:
        return self.config.compression_level

    def get_config(self) -> HybridConfig:
        return self.config

    def query_routing(self, size: int, input_loc: int = HOST, output_loc: int = HOST, is_compression: bool = True) -> int:
        return lib().cuda_zstd_hybrid_query_routing(self._h, size, input_loc, output_loc, int(is_compression))

    def compress(self, data) -> bytes:
        b = bytes(data)
        if not b:
            return b""
        src = ctypes.create_string_buffer(b, len(b))
        cap = lib().cuda_zstd_hybrid_max_compressed_size(self._h, len(b))
        dst = ctypes.create_string_buffer(cap)
        size, res = ctypes.c_size_t(cap), HybridResult()
        rc = lib().cuda_zstd_hybrid_compress(self._h, src, len(b), dst, ctypes.byref(size), HOST, HOST, ctypes.byref(res), None)
        if rc:
            raise ZstdError(rc, "hybrid compress")
        self.last_result = res
        return dst.raw[: size.value]

    def decompress(self, data) -> bytes:
        b = bytes(data)
        if not b:
            return b""
        try:
            cap = extract_metadata(b)["uncompressed_size"] or max(16 * len(b), 1024)
        except ZstdError:
            cap = max(16 * len(b), 1024)
        src = ctypes.create_string_buffer(b, len(b))
        for _ in range(3):  # grow on BUFFER_TOO_SMALL, as the reference binding does
            dst = ctypes.create_string_buffer(max(cap, 1))
            size, res = ctypes.c_size_t(cap), HybridResult()
            rc = lib().cuda_zstd_hybrid_decompress(self._h, src, len(b), dst, ctypes.byref(size), HOST, HOST, ctypes.byref(res), None)
            if rc == 0:
                self.last_result = res
                return dst.raw[: size.value]
            if rc != TOO_SMALL:
                raise ZstdError(rc, "hybrid decompress")
            cap *= 4
        raise ZstdError(TOO_SMALL, "hybrid decompress")


def compress(data, level: int = 3, stream=None):
    return Manager(level).compress(data, stream)


def compress_batch(chunks, level: int = 3, stream=None):
    return Manager(level).compress_batch(chunks, stream)


def decompress(frame, capacity: int = None, stream=None):
    return Manager(3).decompress(frame, capacity, stream)


def decompress_batch(frames, capacities=None, stream=None):
    return Manager(3).decompress_batch(frames, capacities, stream)


def hybrid_compress(data, level: int = 3) -> bytes:
    return HybridEngine(level).compress(data)


def hybrid_decompress(data) -> bytes:
    return HybridEngine(3).decompress(data)


def validate_compressed_data(data, check_checksum: bool = True) -> bool:
    """Frame-header validation (reference validate_compressed_data_py): True iff the buffer
    starts with (skippable frames and) a parseable zstd frame header."""
    try:
        extract_metadata(data)
        return True
    except ZstdError:
        return False


def estimate_compressed_size(uncompressed_size: int, level: int = 3) -> int:
    return max_compressed_size(uncompressed_size)


def is_cuda_available() -> bool:
    """True when a GPU is visible (the reference's name; here an MI355X through ROCm)."""
    import torch

    return torch.cuda.is_available()


def get_cuda_device_info(device: int = 0) -> dict:
    torch = _torch()
    p = torch.cuda.get_device_properties(device)
    return {"name": p.name, "total_memory": p.total_memory, "multi_processor_count": p.multi_processor_count,
            "gcn_arch_name": getattr(p, "gcnArchName", None), "device": device}


def metadata_frame(level: int) -> bytes:
    """The 16-byte skippable metadata frame recording `level` (cuda_zstd_write_metadata_frame)."""
    buf = ctypes.create_string_buffer(16)
    n = ctypes.c_size_t()
    rc = lib().cuda_zstd_write_metadata_frame(buf, 16, level, ctypes.byref(n), None)
    if rc:
        raise ZstdError(rc, "cuda_zstd_write_metadata_frame")
    return buf.raw[: n.value]


def extract_metadata(data) -> dict:
    """Header fields of the first zstd frame after any skippable frames (host bytes or a
    device tensor): level (from a metadata frame, else 3), content size, dictionary ID, checksum."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        b = bytes(data)
        ptr, keep = ctypes.create_string_buffer(b, max(len(b), 1)), None
        n = len(b)
    else:
        keep, ptr, n = data, data.data_ptr(), data.numel()
    lv, us, did, ck = ctypes.c_uint(), ctypes.c_ulonglong(), ctypes.c_uint(), ctypes.c_int()
    rc = lib().cuda_zstd_extract_metadata(ptr, n, ctypes.byref(lv), ctypes.byref(us), ctypes.byref(did), ctypes.byref(ck))
    del keep
    if rc:
        raise ZstdError(rc, "cuda_zstd_extract_metadata")
    return {"level": lv.value, "uncompressed_size": us.value, "dictionary_id": did.value, "checksum": bool(ck.value)}


def profile_enable(on: bool = True) -> None:
    """Record HIP events around each kernel of every launch (on the launch stream)."""
    lib().cuda_zstd_hip_profile_enable(1 if on else 0)


def profile_collect():
    """-> (launches, [ms_lz, ms_entropy, ms_gather] summed over them)."""
    ms = (ctypes.c_double * 3)()
    n = lib().cuda_zstd_hip_profile_collect(ms)
    return n, list(ms)
