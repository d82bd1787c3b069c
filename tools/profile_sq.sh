#!/bin/bash
# SQ instruction-mix counters per kernel for the bench workload (one rocprofv3 --pmc pass:
# 8 SQ counters + GRBM_GUI_ACTIVE, within one pass's hardware limits).  Run on the GPU
# box via gpurun; tools/sq_summary.py condenses the output into profiles/<tag>_sq_summary.json.
set -e
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace -d $OUT/a -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-decompress --no-legs > $OUT/a.log 2>&1
echo sq-done
