# decoder variants: the decode GPU tests on the default build, then per library (default and
# tools/var_*.so) the pipelined bench decompress leg and the isolated (ZH_DEC_SYNC=1) kernel trace
set -e
mkdir -p gpurun_out/var
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var/gputests.log 2>&1
for v in default ${VARS:-b16 b8 g16}; do
  if [ $v = default ]; then unset CUDA_ZSTD_HIP_LIB; else export CUDA_ZSTD_HIP_LIB=$GRAFT_REPO_ROOT/tools/var_$v.so; fi
  if [ $v != default ]; then timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dec or frame" > gpurun_out/var/${v}_gputests.log 2>&1; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-verify --no-legs --steps 5 > gpurun_out/var/${v}_bench.json 2>/dev/null
  ZH_DEC_SYNC=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/var/${v}_iso -o run -- python bench.py --no-cpu-baseline --no-verify --no-legs --steps 2 --warmup 1 > gpurun_out/var/${v}_iso.log 2>&1
done
echo var-done
