"""Print a compact per-kernel summary of rocprofv3 *_kernel_stats.csv files under a directory."""
import csv
import glob
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_stats.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Name"].replace("void (anonymous namespace)::", "").split("(")[0]
        print(f"  {name[:48]:48s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs']) / 1e3:9.3f} us  "
              f"{float(r['Percentage']):6.2f} %")
