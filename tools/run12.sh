#!/bin/bash
# On the box: the round's final set -- -m gpu suite, smoke, profile set (rocprofv3 trace, HBM
# passes, SQ pass, default bench line) under TAG, C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${TAG:-r03j}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
TAG=$TAG bash tools/gpu_prof.sh || exit 3
tail -c 300 gpurun_out/${TAG}_bench.json
timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || exit 4
tail -c 600 gpurun_out/${TAG}_c5.json
