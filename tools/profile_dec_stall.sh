# Stall counters of the decoder kernels run in isolation (ZH_DEC_SYNC=1); run via gpurun.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/dec_stall
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export ZH_DEC_SYNC=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
  --kernel-trace -d $OUT/a -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-legs > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
  --kernel-trace -d $OUT/b -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-legs > $OUT/b.log 2>&1
echo dec-stall-done
