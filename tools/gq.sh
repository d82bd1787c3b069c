#!/bin/bash
# quick GPU check: parity tests + mix/random bench lines (extra bench args via $@)
make -s -C "$(dirname "$0")/../custom-nvcomp-with-zstd_amd" >/dev/null 2>/tmp/gq_build.log || { grep -A3 error /tmp/gq_build.log | head -20; exit 1; }
rm -f gpurun_out/p.log gpurun_out/b.log
timeout 1500 /usr/local/graft/bin/gpurun --timeout 600 -- "timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/p.log 2>&1 && timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $* > gpurun_out/b.log 2>&1 && timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dataset random $* >> gpurun_out/b.log 2>&1" 2>&1 | grep -E "status=|retry|refused"
tail -2 gpurun_out/p.log 2>/dev/null
grep "^{" gpurun_out/b.log 2>/dev/null | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], 'GB/s', d['ms_per_step'], 'ms', 'ratio', d['config'].get('ratio', d.get('ratio')))
"
