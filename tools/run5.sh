#!/bin/bash
# On the box: -m gpu suite (in-tree), deep-kernel phase stamps, C5
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/r5_tests.log 2>&1 || { tail -30 $R/gpurun_out/r5_tests.log; exit 1; }
tail -2 $R/gpurun_out/r5_tests.log
timeout -k 10 200 python3 $R/tools/deep_stamps.py > $R/gpurun_out/deep_stamps5.log 2>&1 || { tail -20 $R/gpurun_out/deep_stamps5.log; exit 1; }
grep -v amdgpu.ids $R/gpurun_out/deep_stamps5.log
timeout -k 10 300 python3 $R/tools/c5_dict.py > $R/gpurun_out/c5_r5.json 2> $R/gpurun_out/c5_r5.err || { tail -5 $R/gpurun_out/c5_r5.err; exit 1; }
tail -c 700 $R/gpurun_out/c5_r5.json
