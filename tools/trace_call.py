"""Kernels of the last full label call in a rocprofv3 kernel trace (one-stream run): name, grid,
duration.  usage: python tools/trace_call.py <trace_kernel_trace.csv> [first-kernel-substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2] if len(sys.argv) > 2 else "k_sample_points"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
tot = 0.0
for r in rows[i0:i1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{r['Kernel_Name'][:48]:48s} grid {r['Grid_Size_X']:>8s} x {r['Workgroup_Size_X']:>4s}  {d:9.1f} us")
span = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3
print(f"kernels {tot:.1f} us, call span {span:.1f} us")
