#!/bin/bash
# GPU check + A/B: -m gpu suite on the in-tree library (A), the parity tests on tools/libB.so
# (B), then alternating bench lines of A and B (C3 mix).  Run on the box via gpurun.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-ab}
mkdir -p $R/gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo A-tests-failed; exit 1; }
  echo A-tests-ok
fi
CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_B_parity.log 2>&1
rc=$?; echo B-parity $rc
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 2
for k in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libB.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-legs --no-decompress --no-verify ${DS:+--dataset $DS} > gpurun_out/${T}_$v$k.json 2>/dev/null || exit 3
    python3 -c "import json; d=json.load(open('gpurun_out/${T}_$v$k.json')); print('$v', d['value'], d['ms_per_step'], d['config'].get('ratio'), d['config'].get('kernel_ms'))"
  done
done
