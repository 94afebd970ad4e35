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
for wl in ("burgers", "burgers_cfg3", "hjb", "gbm", "gbm_hess", "hjb_onestream"):
    f = src / f"trace_{wl}" / "trace_kernel_stats.csv"
    if f.exists():
        rows = list(csv.DictReader(open(f)))
        out = {"command": f"rocprofv3 --kernel-trace --stats -- python bench.py --workload {wl.split('_one')[0]} "
                          f"--steps 10 --warmup 2 --no-cpu-baseline{' --no-prepare' if 'onestream' in wl else ''}",
               "kernels": [{"name": r["Name"][:160], "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                            "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
                            "pct": float(r["Percentage"])} for r in rows]}
        (dst / f"{tag}_{wl}_kernel_trace_stats.json").write_text(json.dumps(out, indent=1))
    b = src / f"bench_{wl}.log"
    if b.exists():
        shutil.copy(b, dst / f"{tag}_bench_{wl}_n1.log")
# HBM traffic per label_moments call, per workload: separate --pmc passes (FETCH_SIZE, WRITE_SIZE) over
# the bench; FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction.  A call is one launch
# of the anchor kernel (k_paths, or k_pis_final for the PISGradNet chain, whose prepare-stream rollout
# runs as several grids per call); the bytes of every
# kernel of the call (rollout, GEMM chain, final, reduce) are summed.
ANCHOR = {"burgers": "dpi::k_paths", "burgers_cfg3": "dpi::k_paths", "gbm": "dpi::k_paths", "gbm_hess": "dpi::k_paths", "hjb": "dpi::k_pis_final"}
for wl, anchor in ANCHOR.items():
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = src / f"pmc_{wl}_{c}" / "pmc_counter_collection.csv"
        if not f.exists():
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
        pmc[c] = {k: {"dispatches": len(v), "total_kb": sum(v)} for k, v in agg.items()}
        (dst / f"{tag}_pmc_{wl}_{c}.json").write_text(json.dumps(
            {"command": f"rocprofv3 --pmc {c} --kernel-include-regex 'k_paths|k_pis|k_gemm|k_reduce|k_noise' -- python "
                        f"bench.py --workload {wl} --steps 10 --warmup 2 --no-cpu-baseline", "kernels": pmc[c]},
            indent=1))
    if len(pmc) < 2:
        continue
    # each pass is its own bench run (the prewarm is timed, so the passes hold different numbers of
    # calls): every counter's total is divided by the anchor launches of its own pass
    ncalls = {c: sum(v["dispatches"] for k, v in pmc[c].items() if k.startswith(anchor)) for c in pmc}
    calls = ncalls["FETCH_SIZE"]
    fe = sum(v["total_kb"] for v in pmc["FETCH_SIZE"].values()) / ncalls["FETCH_SIZE"]
    wr = sum(v["total_kb"] for v in pmc["WRITE_SIZE"].values()) / ncalls["WRITE_SIZE"]
    t = {"workload": wl, "anchor_kernel": anchor, "calls": calls, "calls_write_pass": ncalls["WRITE_SIZE"], "FETCH_SIZE_KB_per_call": fe,
         "WRITE_SIZE_KB_per_call": wr, "hbm_bytes_per_launch": (2 * fe + wr) * 1024,
         "note": "separate --pmc passes; FETCH_SIZE doubled per the gfx950 correction (an upper bound for the "
                 "non-16-B loads); Infinity-Cache hits are counted by these fabric-side counters; all kernels of "
                 "one label_moments call summed",
         "source": f"profiles/{tag}_pmc_{wl}_FETCH_SIZE.json, profiles/{tag}_pmc_{wl}_WRITE_SIZE.json"}
    (dst / f"traffic_{wl}.json").write_text(json.dumps(t, indent=1))
    print(json.dumps(t, indent=1))
# VALU issue per launch (pmc_valu_<wl>: SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU, SQ_INSTS_MFMA, SQ_INSTS_SALU,
# SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE on k_paths): per kernel variant (the network launch
# and the bench's u = 0 noise-floor launch), averaged over dispatches.  SQ_ACTIVE_INST_VALU is in
# quad-cycles summed over all SIMDs (1024); GRBM_GUI_ACTIVE is summed over the 8 XCDs.
N_SIMD, N_XCD = 1024, 8
for wl in ("burgers", "burgers_cfg3", "gbm", "gbm_hess"):
    f = src / f"pmc_valu_{wl}" / "pmc_counter_collection.csv"
    if not f.exists() and wl == "burgers":
        f = src / "pmc_valu" / "pmc_counter_collection.csv"
    if not f.exists():
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    kinds = collections.defaultdict(list)
    for (name, _), c in per.items():
        kinds[name].append(c)
    out = {"command": f"rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES "
                      f"SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex 'k_paths|k_noise' -- python bench.py --workload {wl} "
                      "--steps 10 --warmup 2 --no-cpu-baseline",
           "units": "per launch; valu_busy_cycles_per_simd = SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs; kernel_cycles = "
                    "GRBM_GUI_ACTIVE / 8 XCDs; valu_busy = their ratio (the rocprofv3 VALUBusy expression)",
           "kernels": {}}
    for name, lst in kinds.items():
        avg = {k: sum(c[k] for c in lst) / len(lst) for k in lst[0]}
        busy = avg["SQ_ACTIVE_INST_VALU"] * 4 / N_SIMD
        cyc = avg["GRBM_GUI_ACTIVE"] / N_XCD
        out["kernels"][name] = {"dispatches": len(lst), **{k: round(v) for k, v in avg.items()},
                                "valu_busy_cycles_per_simd": busy, "kernel_cycles": cyc, "valu_busy": busy / cyc,
                                "valu_insts_per_simd": avg["SQ_INSTS_VALU"] / N_SIMD}
    (dst / f"valu_{wl}.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))
