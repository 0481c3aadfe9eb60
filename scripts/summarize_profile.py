"""Summarize a gpurun_out/<dir> produced by scripts/gpu_round*_full.sh into
profiles/<round>/ (kernel stats CSV + PMC per-kernel means + markdown)."""
import collections, csv, json, os, shutil, sys

src, dst = sys.argv[1], sys.argv[2]
commit = sys.argv[3] if len(sys.argv) > 3 else None  # the commit the profiled tree was at
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
for f in ("bench.json", "bench_trace.json", "smoke.log", "pytest_gpu.log"):
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
pmc = collections.defaultdict(list)
for d in ("pmc_fetch", "pmc_write"):
    p = os.path.join(src, d, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        pmc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
stats = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv")))}
bench = json.load(open(os.path.join(src, "bench.json")))
lines = [f"# Profile summary ({os.path.basename(dst)})", "",
         f"bench.py: value {bench['value']} applies/s, {bench['ms_per_step']} ms/apply, "
         f"workload {bench['config']['workload']}", "",
         "## Apply kernels (rocprofv3 --kernel-trace --stats, same bench command)", "",
         "| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
for name, r in stats.items():
    if int(r["Calls"]) >= 100:
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['MinNs'])/1e3:.2f} | "
                     f"{float(r['MaxNs'])/1e3:.2f} |")
lines += ["", "## HBM traffic per launch (separate --pmc passes; FETCH_SIZE x 2 per the gfx950 wide-read "
          "correction, WRITE_SIZE as reported; KB = 1024 B)", "",
          "| kernel | FETCH_SIZE KB | WRITE_SIZE KB | corrected bytes (2*FETCH + WRITE) |", "|---|---|---|---|"]
out = {"__meta__": {"commit": commit, "workload": bench["config"]["workload"],
                    "passes": "rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE (separate runs)"}}
for name in sorted({k[0] for k in pmc}):
    f = pmc.get((name, "FETCH_SIZE"), [0]); w = pmc.get((name, "WRITE_SIZE"), [0])
    if len(f) < 3:
        continue
    fm, wm = sum(f) / len(f), sum(w) / len(w)
    tb = (2 * fm + wm) * 1024
    out[name] = dict(fetch_kb=fm, write_kb=wm, corrected_bytes=tb)
    lines.append(f"| `{name}` | {fm:.0f} | {wm:.0f} | {tb/1e6:.1f} MB |")
json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
