#!/bin/bash
# On the GPU box (via gpurun): diagnostics of the current build under TAG.
#   stamps   K1/K2/K3 phase stamps (tools/libcuda_zstd_hip_stamps.so, `make stamps` first)
#   stall    K1..K4 wave-cycle split SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
#   sq       instruction mix + LDS bank conflicts (tools/profile_sq.sh)
#   trace    rocprofv3 --kernel-trace --stats of the default bench workload
#   tests    the -m gpu suite
#   bench    default bench line (no CPU baseline)
# usage: bash tools/gpu_diag.sh TAG step...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out
for s in "$@"; do
  case $s in
    stamps) timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${TAG}_stamps.log 2>&1 ;;
    stall)
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
        --kernel-trace -d $R/gpurun_out/${TAG}_stall -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/${TAG}_stall.log 2>&1) ;;
    sq) bash $R/tools/profile_sq.sh $TAG ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-legs --no-decompress > $R/gpurun_out/${TAG}_trace.log 2>&1) ;;
    tests) timeout -k 10 500 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_gpu_tests.log; exit 1; } ;;
    bench) timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}_bench.err ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "$s done"
done
