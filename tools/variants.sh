#!/bin/bash
# Build K1 variants here (`bash tools/variants.sh build NAME "-DFLAG=..." ...`: NAME -> tools/libV_NAME.so,
# stamps build tools/libVS_NAME.so) and time them on the GPU box (`bash tools/variants.sh run NAME...`).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/custom-nvcomp-with-zstd_amd
if [ "$1" = build ]; then
  shift
  while [ $# -ge 2 ]; do
    N=$1; F=$2; shift 2
    mkdir -p /tmp/vb_$N
    # (zh_lz.hip, zh_lz_deep.hip, zh_entropy.hip and zh_decode.hip get the flags; the other objects are the in-tree build's)
    for f in zh_lz zh_lz_deep zh_entropy zh_decode; do
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$P/csrc $F -c $P/csrc/$f.hip -o /tmp/vb_$N/$f.o
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$P/csrc $F -DZH_STAMPS -c $P/csrc/$f.hip -o /tmp/vb_$N/${f}_s.o
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/libV_$N.so /tmp/vb_$N/zh_lz.o /tmp/vb_$N/zh_entropy.o /tmp/vb_$N/zh_lz_deep.o /tmp/vb_$N/zh_decode.o $P/build/zh_plan.o $P/build/zh_host.o $P/build/zh_dict.o -ldl
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/libVS_$N.so /tmp/vb_$N/zh_lz_s.o /tmp/vb_$N/zh_entropy_s.o /tmp/vb_$N/zh_lz_deep_s.o /tmp/vb_$N/zh_decode_s.o $P/build_stamps/zh_plan.o $P/build_stamps/zh_host.o $P/build_stamps/zh_dict.o -ldl
  done
  exit 0
fi
shift
mkdir -p $R/gpurun_out
for N in "$@"; do
  CUDA_ZSTD_HIP_LIB=$R/tools/libV_$N.so timeout -k 10 200 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/v_$N.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('$R/gpurun_out/v_$N.json').read().strip().splitlines()[-1]); print('$N', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
  STAMPS_LIB=$R/tools/libVS_$N.so timeout -k 10 200 python3 $R/tools/stamps.py mix 4096 > $R/gpurun_out/vs_$N.log 2>&1
done
