"""Per-call timeline of the HJB prepare-stream schedule from a rocprofv3 kernel trace: for each label
call, the chain's span (k_pis_time .. k_reduce), the gap before it, and how much of the next batch's
rollout (k_pis_rollout grids) ran inside the chain's span."""
import csv
import glob
import sys

f = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void dpi::", ""))
      for r in rows if "dpi::" in r["Kernel_Name"]]
starts = [i for i, e in enumerate(ev) if e[2].startswith("k_pis_time")]
roll = [e for e in ev if e[2].startswith("k_pis_rollout")]
prev_end = None
for a, b in zip(starts, starts[1:] + [len(ev)]):
    chain = [e for e in ev[a:b] if not e[2].startswith("k_pis_rollout") and not e[2].startswith("k_sample")
             and not e[2].startswith("k_baseline") and not e[2].startswith("k_pis_points")]
    t0, t1 = chain[0][0], max(e[1] for e in chain)
    inside = sum(max(0, min(e[1], t1) - max(e[0], t0)) for e in roll)
    gemm = sum(e[1] - e[0] for e in chain if e[2].startswith("k_gemm"))
    gap = (t0 - prev_end) / 1e3 if prev_end else float("nan")
    last_roll_end = max((e[1] for e in roll if e[0] < t1), default=0)
    print(f"chain {(t1 - t0) / 1e3:8.1f} us  gemm {gemm / 1e3:8.1f}  gap-before {gap:7.1f}  rollout-inside {inside / 1e3:8.1f}")
    prev_end = t1
