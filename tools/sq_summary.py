"""Per-kernel SQ counter summary of a tools/attn_pmc.sh output directory: python tools/sq_summary.py gpurun_out/<tag>"""
import collections
import csv
import re
import sys
from pathlib import Path

res = collections.defaultdict(dict)
for sub in ("a", "b"):
    p = Path(sys.argv[1]) / sub / "run_counter_collection.csv"
    if not p.exists():
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(p)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        agg[m.group(1) if m else r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        for c, x in v.items():
            res[k][c] = sum(x) / len(x)
for k, v in res.items():
    wc = v.get("SQ_WAVE_CYCLES") or 1
    line = [k]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if c in v:
            line.append(f"{c[3:]}={v[c] / wc:.3f}")
    if v.get("SQ_INSTS_MFMA"):
        line.append(f"valu/mfma={v['SQ_INSTS_VALU'] / v['SQ_INSTS_MFMA']:.2f} lds/mfma={v['SQ_INSTS_LDS'] / v['SQ_INSTS_MFMA']:.2f} "
                    f"salu/mfma={v['SQ_INSTS_SALU'] / v['SQ_INSTS_MFMA']:.2f}")
    if "SQ_LDS_BANK_CONFLICT" in v and v.get("SQ_ACTIVE_INST_LDS"):
        line.append(f"bankconf/lds_active={v['SQ_LDS_BANK_CONFLICT'] / v['SQ_ACTIVE_INST_LDS']:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        line.append(f"mfma_busy={v['SQ_VALU_MFMA_BUSY_CYCLES']:.3e}")
    print("  ".join(line))
