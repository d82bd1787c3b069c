#!/bin/bash
# On the box: level-9 tests on tools/libB.so (a deep-matcher variant), then C5 on A (in-tree) and B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "deep or c5 or dictionary_tables or streaming" > gpurun_out/r14_tests.log 2>&1 || { tail -30 gpurun_out/r14_tests.log; exit 1; }
tail -2 gpurun_out/r14_tests.log
for v in A B; do
  if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libB.so; fi
  CUDA_ZSTD_HIP_LIB=$L timeout -k 10 300 python3 tools/c5_dict.py > gpurun_out/r14_c5_$v.json 2> gpurun_out/r14_c5_$v.err || exit 2
  python3 -c "import json; d=json.loads(open('gpurun_out/r14_c5_$v.json').read().strip().splitlines()[-1]); print('$v', d['gpu_GBps'], d['ratio']['gpu_none'], d['ratio']['gpu_cover'])"
done
