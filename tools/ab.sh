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
# extra variants: tools/libV_<X>.so (+ tools/libVS_<X>.so stamps), named in $VARIANTS
VS="A B $VARIANTS"
for v in B $VARIANTS; do
  L=$R/tools/lib$v.so; [ $v = B ] || L=$R/tools/libV_$v.so
  CUDA_ZSTD_HIP_LIB=$L timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_k1.py $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > $R/gpurun_out/${TAG}_tests$v.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_tests$v.log; exit 1; }
  echo "tests $v: $(tail -1 $R/gpurun_out/${TAG}_tests$v.log)"
done
for k in $(seq 1 ${ROUNDS:-3}); do
  for v in $VS; do
    if [ $v = A ]; then L=$P/libcuda_zstd_hip.so; elif [ $v = B ]; then L=$R/tools/libB.so; else L=$R/tools/libV_$v.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --dataset ${DATASET:-mix} --chunks ${CHUNKS:-16384} --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/${TAG}_${v}${k}.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/${TAG}_${v}${k}.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  done
done
STAMPS_LIB=$R/tools/libcuda_zstd_hip_stamps.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${TAG}_stampsA.log 2>&1
STAMPS_LIB=$R/tools/libBS.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${TAG}_stampsB.log 2>&1
for v in $VARIANTS; do
  STAMPS_LIB=$R/tools/libVS_$v.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/${TAG}_stamps$v.log 2>&1
done
echo ab-done
