"""Print a window of a rocprofv3 CSV kernel + memory-copy trace in start order (queue ids, durations, gaps):
python3 tools/timeline.py <trace dir> [anchor kernel] [first anchor index] [n anchors]"""
import csv
import os
import sys

d = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_pf_count"
a0 = int(sys.argv[3]) if len(sys.argv) > 3 else 200
na = int(sys.argv[4]) if len(sys.argv) > 4 else 3
rows = []
for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("uc::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "q" + r["Queue_Id"], name[:28]))
mc = os.path.join(d, "run_memory_copy_trace.csv")
if os.path.exists(mc):
    for r in csv.DictReader(open(mc)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "cp", r["Direction"][12:30]))
rows.sort()
idx = [i for i, r in enumerate(rows) if anchor in r[3]]
i0, i1 = idx[a0], idx[min(a0 + na, len(idx) - 1)]
t0 = rows[i0][0]
for r in rows[i0:i1]:
    print(f"{(r[0] - t0) / 1000:9.1f} {(r[1] - t0) / 1000:9.1f} {(r[1] - r[0]) / 1000:8.1f} {r[2]:4s} {r[3]}")
