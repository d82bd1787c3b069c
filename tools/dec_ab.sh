#!/bin/bash
# On the GPU box: decompression A/B -- A = the in-tree build, then each tools/libV_<X>.so named in
# $VARIANTS (tools/variants.sh builds them), alternating ROUNDS times; prints the bench's
# decompress leg (GB/s of decompressed bytes, ms per step) per run.  usage: bash tools/dec_ab.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-decab}
mkdir -p $R/gpurun_out
for k in $(seq 1 ${ROUNDS:-3}); do
  for v in A $VARIANTS; do
    if [ $v = A ]; then L=$R/custom-nvcomp-with-zstd_amd/libcuda_zstd_hip.so; else L=$R/tools/libV_$v.so; fi
    CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-legs > $R/gpurun_out/${TAG}_${v}${k}.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/${TAG}_${v}${k}.json').read().strip().splitlines()[-1]); x=d['decompress']; print('$v', x['value'], x['ms_per_step'], x['roundtrip_equal'])"
  done
done
echo dec-ab-done
