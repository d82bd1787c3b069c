#!/bin/bash
# K1 variant experiment (round 6): the K1 parity tests on each variant tools/libV_<v>.so named in
# $1 (space-separated), then the level-3 bench line and the level-1 leg per variant, alternating,
# and the timeline of the variants named in $2 (tools/libV_<tv>.so, -DZH_TIMELINE builds).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
VS=$1; TVS=$2; T=${3:-k1x}; LV=${LEVELS:-"3 1"}
mkdir -p $R/gpurun_out
for v in $VS; do
  CUDA_ZSTD_HIP_LIB=$R/tools/libV_$v.so timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_k1.py $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${TK:-k1 or levels or c3 or corpora or special}" > $R/gpurun_out/${T}_tests_$v.log 2>&1 || { tail -30 $R/gpurun_out/${T}_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $R/gpurun_out/${T}_tests_$v.log)"
done
for k in $(seq 1 ${ROUNDS:-2}); do
  for v in $VS; do
    for lv in $LV; do
      CUDA_ZSTD_HIP_LIB=$R/tools/libV_$v.so timeout -k 10 200 python3 $R/tools/level_leg.py $lv ${CHUNKS:-16384} | sed "s/^/$v /"
    done
  done
done
for v in $TVS; do
  for lv in $LV; do
    CUDA_ZSTD_HIP_LIB=$R/tools/libV_$v.so timeout -k 10 200 python3 $R/tools/timeline.py $lv 4096 > $R/gpurun_out/${T}_tl_${v}_l$lv.txt 2>&1 || true
    grep -v amdgpu $R/gpurun_out/${T}_tl_${v}_l$lv.txt | tail -16 | sed "s/^/$v L$lv /"
  done
done
echo exp-done
