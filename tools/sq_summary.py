"""Condense a tools/profile_sq.sh run into profiles/<tag>_sq_summary.json.

Per kernel (mean over its dispatches): SQ_INSTS_VALU / SALU / LDS wave-instructions,
LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), and the VALU issue
fraction = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs; MI355X_MICROARCH.md, DVFS notes).
"""
import csv
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_sq_{tag}", "a", "run_counter_collection.csv")
INPUT_BYTES = 16384 * 65536

vals = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(src)):
    k = r["Kernel_Name"]
    if not k.startswith("zh_"):
        continue
    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"tag": tag, "workload": "bench.py C3 16384 x 64 KiB mix chunks, 1 MI355X",
       "command": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES "
                  "SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -- python3 bench.py --steps 2 --warmup 1 ...", "kernels": {}}
for k, c in vals.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    e = {"counters": m, "kernel_cycles": cyc}
    if cyc:
        e["valu_issue_frac"] = round(m.get("SQ_INSTS_VALU", 0) * 4 / (1024 * cyc), 4)
        e["salu_issue_frac_per_cu"] = round(m.get("SQ_INSTS_SALU", 0) / (256 * cyc), 4)
    if m.get("SQ_INSTS_VALU"):
        e["salu_per_valu"] = round(m.get("SQ_INSTS_SALU", 0) / m["SQ_INSTS_VALU"], 4)
        e["valu_insts_per_input_byte"] = round(m["SQ_INSTS_VALU"] / INPUT_BYTES, 3)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
    out["kernels"][k] = e
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(root, "profiles", f"{tag}_sq_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
