import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "custom-nvcomp-with-zstd_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    # CPU-side test infrastructure is cheap to (re)build; the HIP library is built by build()
    for d, so in (("oracle", "liboracle.so"), ("tools", "libdatagen.so"), ("custom-nvcomp-with-zstd_amd", "libcuda_zstd_hip.so")):
        if not os.path.exists(os.path.join(ROOT, d, so)):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, d)], check=True)


@pytest.fixture(scope="session")
def libzstd():
    import zh_testlib as T

    z = T.zstd()
    if z is None:
        pytest.skip("libzstd not present (parity falls back to committed golden fixtures)")
    return z
