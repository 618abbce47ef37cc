"""Per-kernel time of the last full step in a rocprofv3 kernel trace (step delimited by adam_kernel)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Dispatch_Id"]))  # the file is in completion order, not dispatch order
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
s, e = idx[-2] + 1, idx[-1] + 1
tot, cnt = defaultdict(float), defaultdict(int)
for r in rows[s:e]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "")
    n = n.split("(")[0][:80]
    tot[n] += d
    cnt[n] += 1
T = sum(tot.values())
print(f"step kernel time {T / 1e3:.2f} ms, {e - s} launches")
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{v / 1e3:8.2f} ms {cnt[n]:4d}x {100 * v / T:5.1f}%  {n}")
if len(sys.argv) > 4:  # individual launches of the kernels whose name contains argv[4]
    for r in rows[s:e]:
        if sys.argv[4] in r["Kernel_Name"]:
            print(f"  {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f} us  {r['Kernel_Name'][:60]}")
