"""Generic per-kernel sums of a rocprofv3 --pmc CSV (run_counter_collection.csv): per-dispatch
averages of every counter collected. Usage: python tools/pmc_sum.py <dir>"""
import collections
import csv
import glob
import sys

files = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in files:
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mtb::", "")
        vals[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
for k in sorted(vals, key=lambda k: -vals[k].get("SQ_WAVE_CYCLES", 0)):
    d = max(1, len(disp[k]))
    print(f"{k[:40]:40s} x{d:3d} " + " ".join(f"{c}={v / d:.4g}" for c, v in sorted(vals[k].items())))
