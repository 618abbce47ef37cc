"""Per-kernel totals of a rocprofv3 --pmc run directory (every dispatch summed), with the derived
fractions: MFMA busy over GRBM_GUI_ACTIVE / 8 shader clocks x 1024 SIMDs, SQ_WAIT_* / SQ_ACTIVE_* over
SQ_WAVE_CYCLES, LDS bank conflicts per active LDS cycle, instructions per MFMA.
    python tools/pmc_kernels.py gpurun_out/<tag>/a [gpurun_out/<tag>/b ...]"""
import collections
import csv
import sys
from pathlib import Path

tot = collections.defaultdict(lambda: collections.defaultdict(float))
nd = collections.Counter()
for d in sys.argv[1:]:
    for p in Path(d).rglob("*counter_collection.csv"):
        seen = set()
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-50:]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if (p, r["Dispatch_Id"]) not in seen:
                seen.add((p, r["Dispatch_Id"]))
                nd[(k, str(p))] += 1
for k, v in tot.items():
    out = {}
    if v.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        out["mfma_busy"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8)
    wc = v.get("SQ_WAVE_CYCLES")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if wc and c in v:
            out[c[3:].lower()] = v[c] / wc
    if v.get("SQ_ACTIVE_INST_LDS"):
        out["lds_conflict_per_active"] = v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_ACTIVE_INST_LDS"]
    if v.get("SQ_INSTS_MFMA"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if c in v:
                out[c[9:].lower() + "_per_mfma"] = v[c] / v["SQ_INSTS_MFMA"]
    if v.get("SQ_ACTIVE_INST_ANY") and v.get("SQ_WAIT_INST_LDS") is not None:
        out["wait_inst_lds_over_active_any"] = v["SQ_WAIT_INST_LDS"] / v["SQ_ACTIVE_INST_ANY"]
    print(f"{k:50s} " + " ".join(f"{a}={b:.3f}" for a, b in out.items()))
