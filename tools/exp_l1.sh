#!/bin/bash
# Level-1 stride experiment (round 6): parity of each stride variant against its oracle, the
# level-1 leg per variant, level 3 beside it, and K1 stamps at levels 1 and 3.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-l1}
mkdir -p $R/gpurun_out
for v in s1 s2 s4; do
  O=$R/oracle/liboracle.so; [ $v = s1 ] || O=$R/tools/liboracle_$v.so
  ZH_ORACLE_SO=$O CUDA_ZSTD_HIP_LIB=$R/tools/libV_$v.so timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "levels_match_oracle and 1" > $R/gpurun_out/${T}_tests_$v.log 2>&1 || { tail -30 $R/gpurun_out/${T}_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $R/gpurun_out/${T}_tests_$v.log)"
done
for k in 1 2; do
  for v in s1 s2 s4; do
    CUDA_ZSTD_HIP_LIB=$R/tools/libV_$v.so timeout -k 10 200 python3 $R/tools/level_leg.py 1 | sed "s/^/$v /"
  done
  timeout -k 10 200 python3 $R/tools/level_leg.py 3 | sed "s/^/L3 /"
done
for v in s1 s2; do
  STAMPS_LEVEL=1 STAMPS_LIB=$R/tools/libVS_$v.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${T}_stamps_l1_$v.log 2>&1 || true
done
STAMPS_LIB=$R/tools/libVS_s1.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${T}_stamps_l3.log 2>&1 || true
echo exp-done
