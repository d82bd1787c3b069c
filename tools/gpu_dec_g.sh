# decoder pipeline group count: bench decompress leg per tools/var_G*.so library
set -e
mkdir -p gpurun_out/varg
for v in ${VARS:-default G1 G2 G3 G8}; do
  if [ $v = default ]; then unset CUDA_ZSTD_HIP_LIB; else export CUDA_ZSTD_HIP_LIB=$GRAFT_REPO_ROOT/tools/var_$v.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-verify --no-legs --steps 5 > gpurun_out/varg/${v}_bench.json 2>/dev/null
done
echo varg-done
