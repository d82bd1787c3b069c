#!/bin/bash
# On the box: A (in-tree) / B (tools/libB.so) bench lines at 16384 and 2048 chunks.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for C in 16384 2048; do
for k in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libB.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 bench.py --chunks $C --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > gpurun_out/r17_$v$C$k.json 2>/dev/null || exit 2
    python3 -c "import json; d=json.loads(open('gpurun_out/r17_$v$C$k.json').read().strip().splitlines()[-1]); print('$v', $C, d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  done
done
done
