"""Condense `tools/gpu_diag.sh TAG c5lds c5sq` into profiles/<tag>_c5_deep_counters.json: per kernel
the per-dispatch means of both --pmc passes (LDS / wave-state; instruction mix / issue) on the C5
workload, with the derived fractions.  usage: python3 tools/deep_counters_summary.py TAG
  lds_active_per_cu_cycle = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs)
  wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES; wait_inst_any_frac, active_inst_any_frac likewise
  valu_issue_frac = SQ_INSTS_VALU x 4 cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) (one wave's rate)
"""
import csv
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vals = defaultdict(lambda: defaultdict(list))
for kind in ("c5lds", "c5sq"):
    src = os.path.join(root, "gpurun_out", f"{tag}_{kind}", "run_counter_collection.csv")
    for r in csv.DictReader(open(src)):
        k = r["Kernel_Name"]
        if k.startswith("zh_"):
            vals[k][(kind, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {"tag": tag, "workload": "tools/c5_dict.py (C5: 4096 x 16 KiB JSON records, level 9; none / ZDICT / COVER dictionaries, 6 timed launches each + warm-up), C5_GPU_ONLY=1",
       "command": "tools/gpu_diag.sh c5lds + c5sq (two rocprofv3 --pmc passes, --kernel-trace)", "kernels": {}}
for k, c in vals.items():
    m = {}
    for (kind, n), v in c.items():
        m.setdefault(n, sum(v) / len(v))
    g = m.get("GRBM_GUI_ACTIVE", 0) / 8
    e = {"counters": {n: round(v) for n, v in sorted(m.items())}}
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in m:
                e[n.lower()[3:] + "_frac"] = round(m[n] / wc, 4)
    if g:
        if "SQ_LDS_IDX_ACTIVE" in m:
            e["lds_active_per_cu_cycle"] = round(m["SQ_LDS_IDX_ACTIVE"] / (g * 256), 4)
        if "SQ_INSTS_VALU" in m:
            e["valu_issue_frac"] = round(m["SQ_INSTS_VALU"] * 4 / (g * 1024), 4)
    if m.get("SQ_INSTS_LDS"):
        e["lds_bank_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_LDS_IDX_ACTIVE", 1), 1), 4)
    if m.get("SQ_INSTS_VALU"):
        e["salu_per_valu"] = round(m.get("SQ_INSTS_SALU", 0) / m["SQ_INSTS_VALU"], 4)
    out["kernels"][k] = e
dst = os.path.join(root, "profiles", f"{tag}_c5_deep_counters.json")
json.dump(out, open(dst, "w"), indent=1)
for k, e in out["kernels"].items():
    print(k, {n: v for n, v in e.items() if n != "counters"})
