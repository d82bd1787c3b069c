#!/bin/bash
# A/B timing on one GPU box: A = the committed sources (HEAD), B = the working tree.
# `bash tools/ab.sh build` (here): B -> tools/libB.so, then the in-tree library from HEAD.
# usage on the box: bash tools/ab.sh run [dataset]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" = build ]; then
  make -s -C $R/custom-nvcomp-with-zstd_amd >/dev/null
  cp $R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so $R/tools/libB.so
  cd $R && git stash -q && make -s -C custom-nvcomp-with-zstd_amd >/dev/null; git stash pop -q
  exit 0
fi
DS=${2:-mix}
for k in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libB.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --dataset $DS 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])"
  done
done
