"""Condense tools/calib/run.sh output into profiles/<tag>_fetch_write_calibration.json: per access
width, rocprofv3 FETCH_SIZE / WRITE_SIZE (kilobytes per dispatch, x 1024) over the 1 GiB each
calib kernel moves (MI355X_MICROARCH.md, HBM: calibrate uncalibrated widths on a known count)."""
import csv
import json
import os
import re
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r03j"
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
B = float(1 << 30)


def pass_(kind, name):
    agg = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(root, "gpurun_out", f"calib_{kind}", "run_counter_collection.csv"))):
        if r["Counter_Name"] != name:
            continue
        m = re.search(r"void (rd|wr)<([^>]+)>", r["Kernel_Name"])
        if m:
            agg[f"{m.group(1)} {m.group(2)}"].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


f, w = pass_("fetch", "FETCH_SIZE"), pass_("write", "WRITE_SIZE")
rows = {}
for k in sorted(set(f) | set(w)):
    rows[k] = {"fetch_size_bytes": f.get(k), "write_size_bytes": w.get(k),
               "fetch_over_bytes": round(f[k] / B, 4) if k in f else None, "write_over_bytes": round(w[k] / B, 4) if k in w else None}
out = {"tag": tag, "what": "each kernel streams 1 GiB with one access width, coalesced across lanes (tools/calib/calib.hip)",
       "commands": ["rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/calib/calib", "rocprofv3 --pmc WRITE_SIZE --kernel-trace -- tools/calib/calib"],
       "kernels": rows}
json.dump(out, open(os.path.join(root, "profiles", f"{tag}_fetch_write_calibration.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
