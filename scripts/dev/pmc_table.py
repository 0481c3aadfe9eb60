"""Per-kernel SQ counters from a rocprofv3 --pmc csv (last dispatch of each kernel):
python scripts/dev/pmc_table.py <run_counter_collection.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:]
last = {}
vals = defaultdict(dict)
for r in rows:
    n = r["Kernel_Name"]
    if pats and not any(p in n for p in pats):
        continue
    d = int(r["Dispatch_Id"])
    key = n[:60]
    if last.get(key, -1) <= d:
        if last.get(key, -1) < d:
            vals[key] = {"_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
        last[key] = d
        vals[key][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in vals.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:16.0f}")
    if "SQ_WAVE_CYCLES" in v and "SQ_WAVES" in v:
        w = v["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in v:
                print(f"   {c + '/WAVE_CYCLES':34s} {v[c] / w:6.3f}")
        print(f"   quad-cycles per wave {w / v['SQ_WAVES']:.0f}; VALU insts per wave {v.get('SQ_INSTS_VALU', 0) / v['SQ_WAVES']:.0f}")
