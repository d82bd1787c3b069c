#!/bin/bash
# On the GPU box (via gpurun): the round's validation + evidence set under TAG -- the whole -m gpu
# suite, smoke(), the default bench line (with legs and the libzstd baseline), C5 at levels 9 and
# 5, the K1/K2/K3 phase stamps and the rocprofv3 kernel trace of the bench workload.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 2; }
cat gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 3; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'], {k: v['value'] for k, v in d.get('legs', {}).items()})"
C5_LEVEL=9 timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/${TAG}_c5_l9.json 2> gpurun_out/${TAG}_c5_l9.err || { tail gpurun_out/${TAG}_c5_l9.err; exit 4; }
tail -c 600 gpurun_out/${TAG}_c5_l9.json
C5_LEVEL=5 timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/${TAG}_c5_l5.json 2> gpurun_out/${TAG}_c5_l5.err || { tail gpurun_out/${TAG}_c5_l5.err; exit 5; }
timeout -k 10 200 python3 tools/stamps.py mix 4096 > gpurun_out/${TAG}_stamps.log 2>&1 || true
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-legs --no-decompress > $R/gpurun_out/${TAG}_trace.log 2>&1) || true
echo full-done
