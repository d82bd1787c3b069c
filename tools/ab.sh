#!/bin/bash
# A/B on one GPU box: A = the committed sources (HEAD, built in-tree), B = the working tree
# (tools/libB.so, stamps build tools/libBS.so).
#   here:    bash tools/ab.sh build
#   the box: bash tools/ab.sh run TAG [pytest -k expression]
# run: the K1 / parity GPU tests on B, then alternating A/B bench lines (C3 mix, no CPU baseline)
# and the K1 phase stamps of A and B.  Output under gpurun_out/TAG_*.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/custom-nvcomp-with-zstd_amd
if [ "$1" = build ]; then
  make -s -C $P >/dev/null
  cp $P/libcuda_zstd_hip.so $R/tools/libB.so
  make -s -C $P stamps >/dev/null
  cp $R/tools/libcuda_zstd_hip_stamps.so $R/tools/libBS.so
  cd $R && git stash -q && (make -s -C custom-nvcomp-with-zstd_amd >/dev/null; make -s -C custom-nvcomp-with-zstd_amd stamps >/dev/null; make -s -C oracle >/dev/null); git stash pop -q
  # the oracle must match B (the tests run on B)
  make -s -C $R/oracle >/dev/null
  exit 0
fi
TAG=${2:-ab}
K=${3:-"k1 or levels or c3 or corpora or special"}
mkdir -p $R/gpurun_out
CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_k1.py $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > $R/gpurun_out/${TAG}_testsB.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_testsB.log; exit 1; }
tail -1 $R/gpurun_out/${TAG}_testsB.log
for k in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$P/libcuda_zstd_hip.so; else L=$R/tools/libB.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/${TAG}_${v}${k}.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/${TAG}_${v}${k}.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  done
done
STAMPS_LIB=$R/tools/libcuda_zstd_hip_stamps.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${TAG}_stampsA.log 2>&1
STAMPS_LIB=$R/tools/libBS.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${TAG}_stampsB.log 2>&1
echo ab-done
