#!/bin/bash
# On the box: run5 (tests, deep stamps, C5), smoke, then the r03i profile set (rocprofv3 trace,
# HBM passes, SQ pass, default bench line) and the C4 per-rank evidence.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/run5.sh || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03i_smoke.log 2>&1 || { tail -5 gpurun_out/r03i_smoke.log; exit 2; }
tail -1 gpurun_out/r03i_smoke.log
TAG=r03i bash tools/gpu_prof.sh || exit 3
tail -c 400 gpurun_out/r03i_bench.json
cd $R && bash tools/c4_evidence.sh r03i || exit 4
