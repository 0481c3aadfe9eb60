"""Print the kernels of the last Prepare in a rocprofv3 kernel trace, in launch
order, with durations and the gap to the previous kernel.

python scripts/dev/prepare_timeline.py <dir> [first-kernel-substring] [last-kernel-substring]
The window is the last run that starts at a kernel whose name contains the
first substring (default k_stencil_flags) and ends at the next kernel whose
name contains the last substring (default k_factor_rb).
"""
import csv
import sys

import glob
rows = list(csv.DictReader(open(glob.glob(f"{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_stencil_flags"
last = sys.argv[3] if len(sys.argv) > 3 else "k_factor_rb"
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
i0 = starts[-1]
i1 = next(i for i in range(i0, len(rows)) if last in rows[i]["Kernel_Name"])
t0 = int(rows[i0]["Start_Timestamp"])
prev_end = t0
tot = 0.0
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    d = (e - s) / 1000
    tot += d
    name = r["Kernel_Name"].split("(")[0].replace("rocprim::ROCPRIM_400200_NS::detail::", "rp::")[:70]
    print(f"{(s - t0) / 1000:9.1f} {d:8.1f} gap {(s - prev_end) / 1000:6.1f}  {name}")
    prev_end = e
print(f"window {(prev_end - t0) / 1000:.1f} us, kernels {tot:.1f} us")
