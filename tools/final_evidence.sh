#!/bin/bash
# The round's evidence set on one GPU box (via gpurun), every step under its own time limit and
# chained so a failure stops the run: the -m gpu suite, smoke(), the full bench line (legs, CPU
# baselines, decode), C5 at levels 9 and 5, the rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE
# passes (tools/profile.sh), the SQ instruction mix and the wave-state split, and the C4 per-rank
# evidence (2,048-16,384 chunks).  usage: bash tools/final_evidence.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 3; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'], {k: v['value'] for k, v in d.get('legs', {}).items()}, d['decompress']['value'])"
C5_LEVEL=9 timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/${TAG}_c5_l9.json 2> gpurun_out/${TAG}_c5_l9.err || { tail gpurun_out/${TAG}_c5_l9.err; exit 4; }
C5_LEVEL=5 timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/${TAG}_c5_l5.json 2> gpurun_out/${TAG}_c5_l5.err || { tail gpurun_out/${TAG}_c5_l5.err; exit 5; }
bash tools/profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail gpurun_out/${TAG}_profile.log; exit 6; }
bash tools/profile_sq.sh $TAG > gpurun_out/${TAG}_sq.log 2>&1 || { tail gpurun_out/${TAG}_sq.log; exit 7; }
bash tools/gpu_diag.sh $TAG stall > gpurun_out/${TAG}_stall_run.log 2>&1 || { tail gpurun_out/${TAG}_stall_run.log; exit 8; }
bash tools/c4_evidence.sh $TAG > gpurun_out/${TAG}_c4.log 2>&1 || { tail gpurun_out/${TAG}_c4.log; exit 9; }
cat gpurun_out/${TAG}_c4.log
echo evidence-done
