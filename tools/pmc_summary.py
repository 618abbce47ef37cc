"""Condense one tools/profile.sh output directory into a per-kernel HBM-traffic table.

    python tools/pmc_summary.py gpurun_out/prof_envnet profiles/r01_pmc_envnet.json [marker]

For every kernel symbol it reports, per launch: the average duration (from the kernel-trace pass,
whose timings are undisturbed by counter collection), the HBM bytes read and written (FETCH_SIZE
and WRITE_SIZE passes, one counter per pass) and the achieved GB/s.  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE tallies 64 B per 128-B request of a wide coalesced read,
so it is doubled; WRITE_SIZE is taken as is.  Both counters are in KiB.

Only the launches of the last complete step are used (steps delimited by ``marker``, default the
Adam kernel, the last launch of every training step).
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def last_step(rows, marker):
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < 2:
        return rows
    return rows[idx[-2] + 1: idx[-1] + 1]


def counters(path, marker, name):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = defaultdict(list)
    for r in last_step(rows, marker):
        out[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    d = Path(sys.argv[1])
    dst = Path(sys.argv[2])
    marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
    trace = list(csv.DictReader(open(d / "trace" / "run_kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Dispatch_Id"]))  # the file is in completion order, not dispatch order
    dur = defaultdict(list)
    grid = {}
    for r in last_step(trace, marker):
        n = r["Kernel_Name"]
        dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
        grid[n] = [int(r[f"Grid_Size_{a}"]) // int(r[f"Workgroup_Size_{a}"]) for a in "XYZ"]
    fetch = counters(d / "fetch" / "run_counter_collection.csv", marker, "FETCH_SIZE") \
        if (d / "fetch").exists() else {}
    write = counters(d / "write" / "run_counter_collection.csv", marker, "WRITE_SIZE") \
        if (d / "write").exists() else {}
    step_s = sum(sum(v) for v in dur.values())
    table = {}
    for n, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        avg = sum(ds) / len(ds)
        e = {"launches_per_step": len(ds), "avg_ms": round(avg * 1e3, 4),
             "step_share": round(sum(ds) / step_s, 4), "last_grid": grid[n]}
        if n in fetch and n in write:
            rd = 2.0 * sum(fetch[n]) / len(fetch[n])
            wr = sum(write[n]) / len(write[n])
            e.update({"hbm_read_bytes": int(rd), "hbm_write_bytes": int(wr),
                      "hbm_bytes": int(rd + wr), "hbm_gbs": round((rd + wr) / avg / 1e9, 1)})
        table[n] = e
    out = {"source": str(d), "step_kernel_ms": round(step_s * 1e3, 3),
           "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE x1; KiB -> B",
           "kernels": table}
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(f"step kernel time {step_s * 1e3:.2f} ms")
    for n, e in list(table.items())[:25]:
        short = n.replace("_ZN12_GLOBAL__N_1", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        hb = f"{e['hbm_bytes'] / 1e6:10.1f} MB {e['hbm_gbs']:8.1f} GB/s" if "hbm_bytes" in e else ""
        print(f"{e['avg_ms']:8.3f} ms x{e['launches_per_step']:3d} {100 * e['step_share']:5.1f}% {hb}  {short}")


if __name__ == "__main__":
    main()
