"""Shrink a rocprofv3 counter-collection directory to the library's kernels (mtb::*), so a pass over a
bench run that also launches thousands of torch kernels stays small enough to copy back."""
import csv
import os
import sys

d = sys.argv[1]
src = os.path.join(d, "run_counter_collection.csv")
rows = list(csv.DictReader(open(src)))
keep = [r for r in rows if "mtb::" in r["Kernel_Name"]]
with open(src, "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else ["Kernel_Name"])
    w.writeheader()
    w.writerows(keep)
for extra in ("run_kernel_trace.csv",):
    p = os.path.join(d, extra)
    if os.path.exists(p):
        os.remove(p)
