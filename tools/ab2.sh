#!/bin/bash
# A/B over datasets on one GPU box: A = in-tree (HEAD, from `tools/ab.sh build`), B = tools/libB.so,
# variants tools/libV_<X>.so named in $VARIANTS.  K1 parity tests on B first ($TESTS).  Output under
# gpurun_out/TAG_*.   usage (box): bash tools/ab2.sh TAG "random mix"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/custom-nvcomp-with-zstd_amd
TAG=${1:-ab2}
DS=${2:-"random mix"}
mkdir -p $R/gpurun_out
if [ -n "$TESTS" ]; then
  CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 400 python3 -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/${TAG}_testsB.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_testsB.log; exit 1; }
  echo "tests B: $(tail -1 $R/gpurun_out/${TAG}_testsB.log)"
fi
for ds in $DS; do
  for k in $(seq 1 ${ROUNDS:-2}); do
    for v in A B $VARIANTS; do
      if [ $v = A ]; then L=$P/libcuda_zstd_hip.so; elif [ $v = B ]; then L=$R/tools/libB.so; else L=$R/tools/libV_$v.so; fi
      CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --dataset $ds --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/${TAG}_${ds}_${v}${k}.json 2>/dev/null
      python3 -c "import json; d=json.loads(open('$R/gpurun_out/${TAG}_${ds}_${v}${k}.json').read().strip().splitlines()[-1]); print('$ds $v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
    done
  done
done
for ds in $STAMPS; do
  STAMPS_LIB=$R/tools/libBS.so timeout -k 10 200 python3 $R/tools/stamps.py $ds 4096 > $R/gpurun_out/${TAG}_stampsB_$ds.log 2>&1 || true
done
echo ab2-done
