#!/bin/bash
# On the box: -m gpu suite (in-tree), deep-kernel phase stamps, C5, then A/B in-tree vs tools/libF.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/r4_tests.log 2>&1 || { tail -30 $R/gpurun_out/r4_tests.log; exit 1; }
tail -2 $R/gpurun_out/r4_tests.log
timeout -k 10 200 python3 $R/tools/deep_stamps.py > $R/gpurun_out/deep_stamps.log 2>&1 || { tail -20 $R/gpurun_out/deep_stamps.log; exit 1; }
cat $R/gpurun_out/deep_stamps.log | grep -v amdgpu.ids
timeout -k 10 300 python3 $R/tools/c5_dict.py > $R/gpurun_out/c5_r4.json 2> $R/gpurun_out/c5_r4.err || { tail -5 $R/gpurun_out/c5_r4.err; exit 1; }
tail -c 700 $R/gpurun_out/c5_r4.json
for k in 1 2; do
  for v in A F; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libF.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/r4_$v$k.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/r4_$v$k.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  done
done
