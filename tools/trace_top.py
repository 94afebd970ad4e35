"""Top kernels of a rocprofv3 --stats run directory (kernel_stats.csv): name, calls, avg us, %."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))
    if not f:
        print(d, "no kernel_stats.csv")
        continue
    print("==", d)
    for r in list(csv.DictReader(open(f[0])))[:10]:
        print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} {float(r['Percentage']):6.2f}")
