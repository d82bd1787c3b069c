"""Condense a tools/profile.sh run into profiles/<tag>_rocprof_summary.json.

Durations: rocprofv3 --kernel-trace --stats (run_kernel_stats.csv).
HBM bytes: FETCH_SIZE / WRITE_SIZE passes (kilobytes per dispatch).  Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM, CDNA4): on gfx950 FETCH_SIZE reports half
the bytes of 16-B-per-lane streaming reads, so it is doubled; WRITE_SIZE is exact for
16-B streaming stores and uncalibrated for the byte/8-byte stores these kernels issue
(an upper bound: partial-line stores count whole requests).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}")
ours = ("zh_lz_kernel", "zh_entropy_kernel", "zh_fse_chain_kernel", "zh_seq_pack_kernel", "zh_plan_kernel", "zh_gather_kernel")

stats = {}
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
    if r["Name"] in ours:
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6, "share_pct": float(r["Percentage"])}


def counter(kind, name):
    agg = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, kind, "run_counter_collection.csv"))):
        if r["Counter_Name"] == name and r["Kernel_Name"] in ours:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


fetch, write = counter("fetch", "FETCH_SIZE"), counter("write", "WRITE_SIZE")
for k in stats:
    f, w = fetch.get(k), write.get(k)
    stats[k]["fetch_bytes_raw"] = f
    stats[k]["fetch_bytes_corrected"] = 2 * f if f is not None else None
    stats[k]["write_bytes"] = w
    stats[k]["hbm_bytes"] = (2 * f + w) if (f is not None and w is not None) else None
out = {"tag": tag, "workload": "bench.py defaults: C3 16384 x 64 KiB mix chunks, 1 MI355X",
       "commands": ["rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline",
                    "rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline",
                    "rocprofv3 --pmc WRITE_SIZE --kernel-trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"],
       "kernels": stats}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(root, "profiles", f"{tag}_rocprof_summary.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(root, "profiles", f"{tag}_kernel_stats.csv"))
print(json.dumps(out, indent=1))
