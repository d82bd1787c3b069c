#!/bin/bash
# On the GPU box (via gpurun): diagnostics of the current build under TAG.
#   stamps   K1/K2/K3 phase stamps (tools/libcuda_zstd_hip_stamps.so, `make stamps` first)
#   stall    K1..K4 wave-cycle split SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
#   sq       instruction mix + LDS bank conflicts (tools/profile_sq.sh)
#   trace    rocprofv3 --kernel-trace --stats of the default bench workload
#   tests    the -m gpu suite
#   bench    default bench line (no CPU baseline)
#   fullbench the default bench line (CPU baseline, legs, decode)
#   dstamps  deep-matcher phase stamps (tools/deep_stamps.py)
#   k1tests  the K1 / parity GPU tests only
#   rstamps  K1/K2 phase stamps on random data
#   c5       tools/c5_dict.py at level 9 (C5_LEVEL overrides)
#   c5var    for B (the in-tree build) and each tools/libV_<X>.so in $VARIANTS: the deep-matcher
#            GPU tests, C5 at level 9 and the deep-matcher stamps
#   c5lds    LDS / wave-state counters of the deep matcher on the C5 workload (one --pmc pass)
#   c5sq     instruction mix / issue counters of the deep matcher on the C5 workload (one --pmc pass)
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
    fullbench) timeout -k 10 400 python3 $R/bench.py > $R/gpurun_out/${TAG}_fullbench.json 2> $R/gpurun_out/${TAG}_fullbench.err ;;
    dstamps) timeout -k 10 200 python3 $R/tools/deep_stamps.py > $R/gpurun_out/${TAG}_deep_stamps.log 2>&1 ;;
    k1tests) timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_k1.py $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/${TAG}_k1_tests.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_k1_tests.log; exit 1; }; tail -1 $R/gpurun_out/${TAG}_k1_tests.log ;;
    rstamps) timeout -k 10 200 python3 $R/tools/stamps.py random 4096 > $R/gpurun_out/${TAG}_rstamps.log 2>&1 ;;
    c5) C5_LEVEL=${C5_LEVEL:-9} timeout -k 10 300 python3 $R/tools/c5_dict.py > $R/gpurun_out/${TAG}_c5.json 2> $R/gpurun_out/${TAG}_c5.err; tail -c 400 $R/gpurun_out/${TAG}_c5.json ;;
    c5lds)
      (cd /tmp && export TMPDIR=/tmp && C5_LEVEL=9 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE \
        --kernel-trace -d $R/gpurun_out/${TAG}_c5lds -o run --output-format csv -- python3 $R/tools/c5_dict.py > $R/gpurun_out/${TAG}_c5lds.log 2>&1) || { echo "c5lds failed"; exit 3; } ;;
    c5sq)
      (cd /tmp && export TMPDIR=/tmp && C5_LEVEL=9 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
        --kernel-trace -d $R/gpurun_out/${TAG}_c5sq -o run --output-format csv -- python3 $R/tools/c5_dict.py > $R/gpurun_out/${TAG}_c5sq.log 2>&1) || { echo "c5sq failed"; exit 3; } ;;
    c5var)
      for v in B $VARIANTS; do
        L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; LS=$R/tools/libcuda_zstd_hip_stamps.so
        [ $v = B ] || { L=$R/tools/libV_$v.so; LS=$R/tools/libVS_$v.so; }
        CUDA_ZSTD_HIP_LIB=$L timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_dict.py -x -q --timeout 120 --timeout-method thread -k "deep or level9 or c5 or levels" > $R/gpurun_out/${TAG}_c5var_tests$v.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_c5var_tests$v.log; exit 1; }
        echo "tests $v: $(tail -1 $R/gpurun_out/${TAG}_c5var_tests$v.log)"
        CUDA_ZSTD_HIP_LIB=$L C5_LEVEL=9 timeout -k 10 300 python3 $R/tools/c5_dict.py > $R/gpurun_out/${TAG}_c5var_$v.json 2>/dev/null
        python3 -c "import json; d=json.loads(open('$R/gpurun_out/${TAG}_c5var_$v.json').read().strip().splitlines()[-1]); print('$v', d['gpu_GBps'], d['ratio'])"
        STAMPS_LIB=$LS timeout -k 10 200 python3 $R/tools/deep_stamps.py > $R/gpurun_out/${TAG}_c5var_stamps$v.log 2>&1 || true
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "$s done"
done
