#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03l_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03l_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03l_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03l_smoke.log 2>&1 || { tail -5 gpurun_out/r03l_smoke.log; exit 2; }
tail -1 gpurun_out/r03l_smoke.log
