"""Condense a `tools/gpu_diag.sh TAG stall` run into profiles/<tag>_stall_summary.json.

Per kernel (mean over its dispatches): the SQ wave-state counters and their fractions of
SQ_WAVE_CYCLES -- SQ_WAIT_ANY (parked in s_waitcnt / barrier), SQ_WAIT_INST_ANY (ready but
waiting for an issue slot), SQ_ACTIVE_INST_ANY (issuing); MI355X_MICROARCH.md: the three add up
to SQ_WAVE_CYCLES.  usage: python3 tools/stall_summary.py TAG [workload note]
"""
import csv
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1]
note = sys.argv[2] if len(sys.argv) > 2 else "bench.py C3 16384 x 64 KiB mix chunks, 1 MI355X"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"{tag}_stall", "run_counter_collection.csv")

vals = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(src)):
    k = r["Kernel_Name"]
    if k.startswith("zh_"):
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"tag": tag, "workload": note,
       "command": "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS "
                  "SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify "
                  "--no-decompress --no-legs (tools/gpu_diag.sh stall)",
       "note": "fractions of SQ_WAVE_CYCLES (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES): "
               "parked in s_waitcnt/barrier, waiting for an issue slot, issuing",
       "kernels": {}}
for k, c in vals.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0)
    out["kernels"][k] = {"counters": m,
                         "frac_of_wave_cycles": {n: round(m[n] / wc, 4) for n in m if n.startswith("SQ_") and n != "SQ_WAVE_CYCLES"} if wc else {}}
dst = os.path.join(root, "profiles", f"{tag}_stall_summary.json")
json.dump(out, open(dst, "w"), indent=1)
for k, e in out["kernels"].items():
    f = e["frac_of_wave_cycles"]
    print(k, {n: f.get(n) for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")})
