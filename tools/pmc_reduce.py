"""Reduce profiles/pmc_front.sh passes (p1..p4) for one kernel to per-dispatch
means and the derived figures DESIGN.md quotes:
  valu_issue_frac = SQ_INSTS_VALU x 2 cycles (wave64 VALU issue on gfx950) /
                    (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
  wait_frac       = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  hbm_bytes_per_launch   = FETCH_SIZE x 2 (gfx950 half-count) + WRITE_SIZE, KiB -> B
Usage: python3 tools/pmc_reduce.py PMC_DIR KERNEL_SUBSTR OUT_JSON [note]
FIRST=N keeps the first N dispatches of each counter in each pass (the timed
default-bench encodes; later dispatches of a run with side rows are other
configurations, e.g. the filtered cjxl-defaults row)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, kern, out = sys.argv[1], sys.argv[2], sys.argv[3]
note = sys.argv[4] if len(sys.argv) > 4 else ""
first = int(os.environ.get("FIRST", "0"))
vals = defaultdict(list)
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(list)
    with open(p) as f:
        for r in csv.DictReader(f):
            if kern in r["Kernel_Name"]:
                per[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    for k, v in per.items():
        v.sort()
        vals[k] += [x for _, x in (v[:first] if first else v)]
m = {k: sum(v) / len(v) for k, v in vals.items()}
res = {"kernel": kern, "workload": "8k", "note": note}
res.update({k: m[k] for k in sorted(m)})
if "SQ_INSTS_VALU" in m and "GRBM_GUI_ACTIVE" in m:
    res["valu_issue_frac"] = round(m["SQ_INSTS_VALU"] * 2 / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
    res["wait_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
    res["lds_bank_conflict_frac"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 3)
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    res["fetch_bytes_corrected"] = 2.0 * m["FETCH_SIZE"] * 1024.0
    res["write_bytes"] = m["WRITE_SIZE"] * 1024.0
    res["hbm_bytes_per_launch"] = res["fetch_bytes_corrected"] + res["write_bytes"]
    res["correction"] = "FETCH_SIZE x2 (gfx950 half-count), KiB -> bytes"
res["dispatches"] = {k: len(v) for k, v in vals.items()}
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
