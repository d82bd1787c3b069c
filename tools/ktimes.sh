#!/bin/bash
# quick per-kernel average durations of the bench workload (rocprofv3 --kernel-trace --stats)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/kt
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/log 2>&1
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:40]:40s} calls {r['Calls']:>4s} avg_ms {float(r['AverageNs'])/1e6:8.3f}\")
"
