#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun):
#   1. --kernel-trace --stats       per-kernel average durations
#   2. --pmc FETCH_SIZE             HBM read bytes per dispatch   (own pass: TCC slots)
#   3. --pmc WRITE_SIZE             HBM write bytes per dispatch
# Outputs under gpurun_out/prof_<tag>/; tools/prof_summary.py condenses them.
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-legs > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-legs --no-decompress > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-legs --no-decompress > $OUT/write.log 2>&1
echo profile-done
