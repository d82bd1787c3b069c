"""Run by tests/test_gpu_k1.py::test_ins_check_variant_never_repairs in a child process with
CUDA_ZSTD_HIP_LIB pointing at libcuda_zstd_hip_inscheck.so (K1 built with -DZH_INS_CHECK): the
C3 sample and the corpora batch at levels 1-3 through the batch path; writes the frames and the
number of inserter repairs the variant took to <out>.npz."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cuda_zstd  # noqa: E402
import ins_check_data as D  # noqa: E402


def main():
    out = sys.argv[1]
    L = cuda_zstd.lib()
    assert os.path.basename(cuda_zstd.LIB_PATH) == "libcuda_zstd_hip_inscheck.so", cuda_zstd.LIB_PATH
    L.zh_fixups_host.restype = ctypes.c_uint32
    L.zh_fixups_host()  # reset
    res = {}
    for level in D.LEVELS:
        frames = D.compress(level)
        res[f"sizes{level}"] = np.array([len(f) for f in frames], np.int64)
        res[f"frames{level}"] = np.frombuffer(b"".join(frames), np.uint8)
    torch.cuda.synchronize()
    res["repairs"] = np.array([L.zh_fixups_host()], np.int64)
    np.savez(out, **res)


if __name__ == "__main__":
    main()
