"""Per-kernel SQ counter summary of one tools/profile.sh 'sq' pass (or the older tools/attn_pmc.sh a/b
directories).

    python tools/sq_summary.py gpurun_out/prof_<tag> [profiles/r03_sq_<tag>.json] [marker]

MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over every SIMD
(MI355X_MICROARCH.md, constants table: 32 per v_mfma_f32_32x32x16_bf16), so
util = MFMA_BUSY / (1024 SIMDs x duration x clock); the duration and the clock are the counter run's own:
clock = GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS give-back: rocprofv3 reports
GRBM_GUI_ACTIVE summed over the 8 XCDs; within 3 % of the in-kernel clock on dispatches of 10 ms or more),
so a kernel's MFMA utilisation is MFMA_BUSY / (1024 x GRBM_GUI_ACTIVE / 8).  Round 3's estimate from
SQ_BUSY_CU_CYCLES read 7.6-9.3 GHz (that counter is not per-CU shader cycles) and is not used.  SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles per wave; they are reported as fractions of SQ_WAVE_CYCLES.
Only the launches of the last complete step (marker: the Adam kernel) are used.
"""
from __future__ import annotations

import collections
import csv
import json
import re
import sys
from pathlib import Path

NSIMD, NCU, NXCD = 1024, 256, 8


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n[-60:]


def last_step(rows, marker):
    ids = sorted({int(r["Dispatch_Id"]) for r in rows if marker in r["Kernel_Name"]})
    if len(ids) < 2:
        return rows
    lo, hi = ids[-2], ids[-1]
    return [r for r in rows if lo < int(r["Dispatch_Id"]) <= hi]


def main():
    root = Path(sys.argv[1])
    out = sys.argv[2] if len(sys.argv) > 2 else None
    marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
    res = collections.defaultdict(lambda: collections.defaultdict(float))
    dur_pmc = collections.defaultdict(float)
    launches = collections.Counter()
    for sub in ("sq", "a", "b"):
        p = root / sub / "run_counter_collection.csv"
        if not p.exists():
            continue
        rows = last_step(list(csv.DictReader(open(p))), marker)
        seen = set()
        for r in rows:
            k = short(r["Kernel_Name"])
            res[k][r["Counter_Name"]] += float(r["Counter_Value"])
            d = r["Dispatch_Id"]
            if (sub, d) not in seen:
                seen.add((sub, d))
                if sub in ("sq", "a"):
                    dur_pmc[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                    launches[k] += 1
    # undisturbed durations from the kernel-trace pass
    dur = collections.defaultdict(float)
    tp = root / "trace" / "run_kernel_trace.csv"
    if tp.exists():
        rows = list(csv.DictReader(open(tp)))
        idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
        if len(idx) >= 2:
            rows = rows[idx[-2] + 1: idx[-1] + 1]
        for r in rows:
            dur[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    table = {}
    for k, v in sorted(res.items(), key=lambda kv: -dur_pmc.get(kv[0], 0.0)):
        wc = v.get("SQ_WAVE_CYCLES") or 1.0
        row = {"launches": launches[k], "ms_pmc_run": round(dur_pmc[k] * 1e3, 4)}
        if dur.get(k):
            row["ms_trace"] = round(dur[k] * 1e3, 4)
        if v.get("GRBM_GUI_ACTIVE") and dur_pmc[k] > 0:
            cycles = v["GRBM_GUI_ACTIVE"] / NXCD  # shader clocks over the kernels' wall time
            row["clock_ghz_pmc_run"] = round(cycles / dur_pmc[k] / 1e9, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
                row["mfma_util"] = round(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (NSIMD * cycles), 4)
                if dur.get(k):  # the same busy cycles over the undisturbed trace duration at the run's clock
                    row["mfma_util_trace_duration"] = round(
                        v["SQ_VALU_MFMA_BUSY_CYCLES"] / (NSIMD * dur[k] * cycles / dur_pmc[k]), 4)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in v:
                row[c[3:].lower() + "_frac"] = round(v[c] / wc, 4)
        if v.get("SQ_ACTIVE_INST_LDS"):
            row["lds_bank_conflict_per_lds_active"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_ACTIVE_INST_LDS"], 4)
        if v.get("SQ_INSTS_MFMA"):
            row["valu_per_mfma"] = round(v.get("SQ_INSTS_VALU", 0) / v["SQ_INSTS_MFMA"], 3)
            row["lds_per_mfma"] = round(v.get("SQ_INSTS_LDS", 0) / v["SQ_INSTS_MFMA"], 3)
        table[k] = row
    for k, row in list(table.items())[:30]:
        print(f"{k:60s} " + " ".join(f"{a}={b}" for a, b in row.items()))
    if out:
        Path(out).write_text(json.dumps({"source": str(root), "marker": marker, "kernels": table}, indent=1) + "\n")


if __name__ == "__main__":
    main()
