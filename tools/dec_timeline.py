"""Decoder kernel timeline of the last profiled step (rocprofv3 kernel trace CSV): usage
python tools/dec_timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith("zh_de")]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
t0 = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = s if t0 is None else t0
    print(f"{r['Kernel_Name']:20s} q{r['Queue_Id']} {(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}")
