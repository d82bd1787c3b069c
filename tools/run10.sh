#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r10_tests.log 2>&1 || { tail -30 gpurun_out/r10_tests.log; exit 1; }
tail -2 gpurun_out/r10_tests.log
bash tools/calib/run.sh || exit 2
