"""Summarise a rocprofv3 kernel trace: per-kernel totals and the launch sequence of the last step."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(path)))
marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
tot = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"][:90]
    tot[n] += d
    cnt[n] += 1
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
s, e = idx[-2] + 1, idx[-1] + 1
step = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[s:e])
print(f"last step: {e - s} launches, {step / 1e3:.2f} ms of kernel time")
for r in rows[s:e]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if d > float(sys.argv[4] if len(sys.argv) > 4 else 50):
        print(f"{d:9.1f}us grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']}) {r['Kernel_Name'][:100]}")
