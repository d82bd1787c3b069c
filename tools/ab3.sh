#!/bin/bash
# On the box: the -m gpu suite on tools/libF.so (a variant build), the C5 tool on the in-tree
# library, then alternating bench lines A (in-tree) / F (variant).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
F=$R/tools/libF.so
CUDA_ZSTD_HIP_LIB=$F timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/ab3_tests.log 2>&1 || { tail -30 $R/gpurun_out/ab3_tests.log; exit 1; }
tail -2 $R/gpurun_out/ab3_tests.log
timeout -k 10 300 python3 $R/tools/c5_dict.py > $R/gpurun_out/c5_A.json 2> $R/gpurun_out/c5_A.err || { tail -5 $R/gpurun_out/c5_A.err; exit 1; }
tail -c 800 $R/gpurun_out/c5_A.json
for k in 1 2 3; do
  for v in A F; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$F; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/ab3_$v$k.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/ab3_$v$k.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  done
done
