#!/bin/bash
# A/B on one box (after `bash tools/ab.sh build` here): the -m gpu suite on B (the working tree),
# then alternating A/B bench lines with the per-stage kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cat /sys/fs/cgroup/cpu.max > $R/gpurun_out/cgroup_cpu_max.txt 2>&1 || true
nproc >> $R/gpurun_out/cgroup_cpu_max.txt
if [ "${AB_TESTS:-1}" = 1 ]; then
  CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/ab_tests.log 2>&1 || { tail -30 $R/gpurun_out/ab_tests.log; exit 1; }
  tail -2 $R/gpurun_out/ab_tests.log
fi
DS=${1:-mix}
for k in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libB.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs --dataset $DS > $R/gpurun_out/ab_$v$k.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/ab_$v$k.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  done
done
if [ "${AB_C5:-0}" = 1 ]; then
  CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 300 python3 $R/tools/c5_dict.py > $R/gpurun_out/c5_B.json 2> $R/gpurun_out/c5_B.err || { tail -5 $R/gpurun_out/c5_B.err; exit 1; }
  tail -c 1500 $R/gpurun_out/c5_B.json
fi
