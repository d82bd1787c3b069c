#!/bin/bash
# On the box: full -m gpu suite (in-tree), the deep tests on tools/libC.so (every chain step
# through the out-of-order fix-up path), C5 and the deep-kernel phase stamps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03k_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03k_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03k_gpu_tests.log
CUDA_ZSTD_HIP_LIB=$R/tools/libC.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "deep or c5 or dictionary_tables or streaming" > gpurun_out/r03k_fixup_tests.log 2>&1 || { tail -30 gpurun_out/r03k_fixup_tests.log; exit 2; }
tail -2 gpurun_out/r03k_fixup_tests.log
timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/r03k_c5.json 2> gpurun_out/r03k_c5.err || exit 3
tail -c 500 gpurun_out/r03k_c5.json
timeout -k 10 200 python3 tools/deep_stamps.py > gpurun_out/r03k_deep_stamps.log 2>&1 || exit 4
grep -v amdgpu.ids gpurun_out/r03k_deep_stamps.log
