#!/bin/bash
# LDS pressure counters for K1 (one --pmc pass of SQ counters): run on the GPU box via gpurun.
# Output: gpurun_out/prof_lds_<tag>/
set -e
TAG=${1:-r03}
LIB=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_lds_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export CUDA_ZSTD_HIP_LIB=$R/$LIB
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  --kernel-trace -d $OUT/a -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-decompress --no-legs > $OUT/a.log 2>&1
echo lds-done
