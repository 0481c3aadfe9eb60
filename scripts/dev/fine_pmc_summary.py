"""Summarize scripts/dev/gpu_fine_pmc.sh output: per config and fine variant,
the fine kernel's average duration (kernel trace) and per-launch counter means
(PMC passes p1..p5), with derived rates.  argv: gpurun_out/<dir> [out.md]."""
import collections, csv, glob, json, os, sys

src = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(src, "summary.md")
rows, data = [], {}
for tdir in sorted(glob.glob(os.path.join(src, "*_v*"))):
    if not os.path.isdir(tdir):
        continue
    t = os.path.basename(tdir)
    d = {}
    st = os.path.join(tdir, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            if r["Name"].split("(")[0].split("<")[0].endswith(("k_solve_fine", "k_solve_fine1")):
                d["fine_us"] = float(r["AverageNs"]) / 1e3
                d["kernel"] = r["Name"].split("(")[0]
    acc = collections.defaultdict(list)
    for p in sorted(glob.glob(os.path.join(tdir, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0]
            if k.endswith(("k_solve_fine", "k_solve_fine1")):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d.update({c: sum(v) / len(v) for c, v in acc.items()})
    data[t] = d
lines = [f"# k_solve_fine PMC ({os.path.basename(src.rstrip('/'))})", "",
         "Per-launch means over the profiled applies; FETCH_SIZE / WRITE_SIZE in KB (FETCH x2 = gfx950 "
         "wide-read correction), durations from the kernel trace of the same command.", ""]
keys = sorted({k for d in data.values() for k in d if k not in ("kernel",)})
lines.append("| counter | " + " | ".join(data) + " |")
lines.append("|---|" + "---|" * len(data))
for k in keys:
    vals = []
    for d in data.values():
        v = d.get(k)
        vals.append("" if v is None else (f"{v:.4g}" if abs(v) < 1e6 else f"{v:.4e}"))
    lines.append(f"| {k} | " + " | ".join(vals) + " |")
lines += ["", "Derived:", ""]
for t, d in data.items():
    der = []
    if "fine_us" in d and "FETCH_SIZE" in d:
        tb = (2 * d["FETCH_SIZE"] + d.get("WRITE_SIZE", 0)) * 1024
        der.append(f"HBM {tb / 1e6:.1f} MB/launch = {tb / d['fine_us'] / 1e6:.2f} TB/s")
    if "TCP_UTCL1_TRANSLATION_MISS_sum" in d and "TCP_UTCL1_REQUEST_sum" in d and d["TCP_UTCL1_REQUEST_sum"]:
        der.append(f"UTCL1 miss {100 * d['TCP_UTCL1_TRANSLATION_MISS_sum'] / d['TCP_UTCL1_REQUEST_sum']:.2f} %")
    if "GRBM_UTCL2_BUSY" in d and d.get("GRBM_GUI_ACTIVE"):
        der.append(f"UTCL2 busy {100 * d['GRBM_UTCL2_BUSY'] / d['GRBM_GUI_ACTIVE']:.1f} % of GUI_ACTIVE")
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and (d["TCC_HIT_sum"] + d["TCC_MISS_sum"]):
        der.append(f"L2 hit {100 * d['TCC_HIT_sum'] / (d['TCC_HIT_sum'] + d['TCC_MISS_sum']):.1f} %")
    if "TCC_EA0_RDREQ_LEVEL_sum" in d and d.get("TCC_EA0_RDREQ_sum"):
        der.append(f"mean EA read latency {d['TCC_EA0_RDREQ_LEVEL_sum'] / d['TCC_EA0_RDREQ_sum']:.0f} cycles")
    if "TCP_TCC_READ_REQ_LATENCY_sum" in d and d.get("TCP_UTCL1_REQUEST_sum"):
        der.append(f"TCP->TCC read latency sum {d['TCP_TCC_READ_REQ_LATENCY_sum']:.3e}")
    if "SQ_WAVE_CYCLES" in d and d.get("SQ_BUSY_CYCLES"):
        der.append(f"waves in flight (avg) {d['SQ_WAVE_CYCLES'] / d['SQ_BUSY_CYCLES']:.0f}")
    if "SQ_WAIT_ANY" in d and d.get("SQ_WAVE_CYCLES"):
        der.append(f"wait-any {100 * d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES']:.1f} % of wave-cycles")
    lines.append(f"- `{t}` ({d.get('fine_us', float('nan')):.1f} us): " + "; ".join(der))
open(out, "w").write("\n".join(lines) + "\n")
json.dump(data, open(os.path.splitext(out)[0] + ".json", "w"), indent=1)
print("\n".join(lines))
