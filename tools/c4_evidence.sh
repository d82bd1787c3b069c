#!/bin/bash
# C4 per-rank evidence at N=1 (run on the GPU box via gpurun): the bench line for the chunk
# counts one rank of a 1/2/4/8-GPU strong-scaling run compresses (16384 / N), each also under
# rocprofv3 --kernel-trace --stats.  Outputs gpurun_out/c4_<tag>_<chunks>.json and
# gpurun_out/c4_<tag>_prof_<chunks>/.
set -o pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for C in 2048 4096 8192 16384; do
  timeout -k 10 200 python3 $R/bench.py --chunks $C --steps 20 --warmup 3 --no-cpu-baseline --no-verify --no-decompress --no-legs \
    > $R/gpurun_out/c4_${TAG}_$C.json 2> $R/gpurun_out/c4_${TAG}_$C.err || exit 1
  python3 -c "import json; d=json.loads(open('$R/gpurun_out/c4_${TAG}_$C.json').read().strip().splitlines()[-1]); print($C, d['ms_per_step'], 'ms', d['value'], 'GB/s', d['config']['kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for C in 2048 4096 8192; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4_${TAG}_prof_$C -o run --output-format csv -- \
    python3 $R/bench.py --chunks $C --steps 20 --warmup 3 --no-cpu-baseline --no-verify --no-decompress --no-legs \
    > $R/gpurun_out/c4_${TAG}_prof_$C.log 2>&1 || exit 2
done
echo c4-done
