"""Condense a tools/profile_round.sh output directory into the committed profiles/ files:
<tag>_<workload>_kernel_trace_stats.json (rocprofv3 --kernel-trace --stats), <tag>_bench_<wl>_n1.log,
<tag>_pmc_{FETCH,WRITE}_SIZE.json and traffic_<workload>.json (HBM bytes per k_paths launch,
FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note)."""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

src, tag = Path(sys.argv[1]), sys.argv[2]
dst = Path(__file__).resolve().parents[1] / "profiles"
for wl in ("burgers", "hjb", "gbm", "gbm_hess"):
    f = src / f"trace_{wl}" / "trace_kernel_stats.csv"
    if f.exists():
        rows = list(csv.DictReader(open(f)))
        out = {"command": f"rocprofv3 --kernel-trace --stats -- python bench.py --workload {wl} --steps 10 --warmup 2 "
                          "--no-cpu-baseline",
               "kernels": [{"name": r["Name"][:160], "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                            "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
                            "pct": float(r["Percentage"])} for r in rows]}
        (dst / f"{tag}_{wl}_kernel_trace_stats.json").write_text(json.dumps(out, indent=1))
    b = src / f"bench_{wl}.log"
    if b.exists():
        shutil.copy(b, dst / f"{tag}_bench_{wl}_n1.log")
pmc = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = src / f"pmc_{c}" / "pmc_counter_collection.csv"
    if not f.exists():
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    pmc[c] = {k: {"dispatches": len(v), "avg_kb_per_dispatch": sum(v) / len(v)} for k, v in agg.items()}
    (dst / f"{tag}_pmc_{c}.json").write_text(json.dumps(
        {"command": f"rocprofv3 --pmc {c} --kernel-include-regex 'k_paths|k_pis|k_gemm' -- python bench.py "
                    "--steps 10 --warmup 2 --no-cpu-baseline", "kernels": pmc[c]}, indent=1))
if pmc:
    k = next(k for k in pmc["FETCH_SIZE"] if k.startswith("dpi::k_paths"))
    fe, wr = pmc["FETCH_SIZE"][k]["avg_kb_per_dispatch"], pmc["WRITE_SIZE"][k]["avg_kb_per_dispatch"]
    t = {"kernel": k, "workload": "Burgers cfg2 16 x 4096 K=50 (bench.py default)", "FETCH_SIZE_KB": fe,
         "WRITE_SIZE_KB": wr, "hbm_bytes_per_launch": (2 * fe + wr) * 1024,
         "note": "separate --pmc passes; FETCH_SIZE doubled per the gfx950 correction (an upper bound for the "
                 "non-16-B loads); Infinity-Cache hits are counted by these fabric-side counters",
         "source": f"profiles/{tag}_pmc_FETCH_SIZE.json, profiles/{tag}_pmc_WRITE_SIZE.json"}
    (dst / "traffic_burgers.json").write_text(json.dumps(t, indent=1))
    print(json.dumps(t, indent=1))
