"""Per-kernel LDS bank-conflict fraction from tools/lds_pmc.sh: SQ_LDS_BANK_CONFLICT (extra LDS-array
cycles) / SQ_LDS_IDX_ACTIVE (all LDS-array cycles), summed over the launches of one step.

    python tools/lds_summary.py gpurun_out/lds_<leg> [out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
rows = []
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = defaultdict(lambda: defaultdict(float))
for r in rows:
    k = r["Kernel_Name"]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = {}
for k, c in acc.items():
    idx = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
    if idx <= 0:
        continue
    out[k[:90]] = {"lds_idx_active": idx, "bank_conflict": c.get("SQ_LDS_BANK_CONFLICT", 0.0),
                   "conflict_frac_of_lds_cycles": round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / idx, 4),
                   "insts_lds": c.get("SQ_INSTS_LDS", 0.0),
                   "lds_cycles_share_of_gui": round(idx / max(c.get("GRBM_GUI_ACTIVE", 1.0), 1.0), 4)}
for k, v in sorted(out.items(), key=lambda kv: -kv[1]["bank_conflict"])[:25]:
    print(f"{k[:60]:60s} conflict/lds-cycles {v['conflict_frac_of_lds_cycles']:.3f}  lds-cycles {v['lds_idx_active']:.3e}")
if len(sys.argv) > 2:
    json.dump({"source": d, "kernels": out}, open(sys.argv[2], "w"), indent=1)
