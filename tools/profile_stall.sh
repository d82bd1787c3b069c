# Stall / instruction-cache counters for the bench workload (two --pmc passes, each within one
# pass's block limits); run on the GPU box via gpurun.  Output: gpurun_out/prof_stall_<tag>/
set -e
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_stall_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --kernel-trace -d $OUT/a -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-decompress --no-legs > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES \
  --kernel-trace -d $OUT/b -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-decompress --no-legs > $OUT/b.log 2>&1
echo stall-done
