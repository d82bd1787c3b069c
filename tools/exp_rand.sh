# A/B of whole-library variants (run on the GPU box): tools/libV_<name>.so, bench line only
R=${GRAFT_REPO_ROOT:-$(pwd)}
for N in "$@"; do
  CUDA_ZSTD_HIP_LIB=$R/tools/libV_$N.so timeout -k 10 200 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/v_$N.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$R/gpurun_out/v_$N.json').read().strip().splitlines()[-1]); print('$N', d['value'], d['ms_per_step'], d['config']['kernel_ms'])"
done
