"""Per-kernel-dispatch PMC summary of rocprofv3 counter_collection CSVs (per wave / per SIMD units)."""
import collections
import csv
import sys

rows = []
for f in sys.argv[1:]:
    rows += list(csv.DictReader(open(f)))
agg = collections.OrderedDict()
for r in rows:
    key = (r["Kernel_Name"].split("(")[0].replace("void dpi::", ""), r["Grid_Size"], r["Dispatch_Id"], r["Correlation_Id"])
    agg.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in agg.items():
    print(k[0], k[2], " ".join(f"{a}={b:.3e}" for a, b in sorted(v.items())))
