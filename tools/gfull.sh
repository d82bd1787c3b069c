#!/bin/bash
# GPU round check (run on the box through gpurun): the whole -m gpu suite, then the C3 mix and
# random bench lines (no CPU baseline).  Logs under gpurun_out/.
mkdir -p gpurun_out
T=${1:-full}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > gpurun_out/${T}_mix.json 2> gpurun_out/${T}_mix.err || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs --dataset random > gpurun_out/${T}_rand.json 2> gpurun_out/${T}_rand.err || exit 1
python3 - "$T" <<'PY'
import json, sys
T = sys.argv[1]
for k in ("mix", "rand"):
    d = json.loads(open(f"gpurun_out/{T}_{k}.json").read().strip().splitlines()[-1])
    print(k, d["value"], "GB/s", d["ms_per_step"], "ms ratio", d["config"]["ratio"], "kernels", d["config"]["kernel_ms"])
PY
