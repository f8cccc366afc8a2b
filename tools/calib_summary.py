"""Per-dispatch counters of tools/calib_random_fetch.sh, averaged per kernel and buffer argument, with
the access counts they are checked against. Usage: python3 tools/calib_summary.py gpurun_out/r05/calib"""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
timing = [json.loads(l) for l in open(os.path.join(d, "timing.jsonl")) if l.strip()]
out = {"timing": timing, "passes": {}}
for name in ("fetch", "req", "req2", "write", "wreq"):
    path = os.path.join(d, name, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    kern = {}
    for r in csv.DictReader(open(path)):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] += float(r["Counter_Value"])
        kern[i] = r["Kernel_Name"].split("(")[0]
    # the tool's dispatches: per argument one warm-up + 5 timed launches (fill kernels in between)
    groups, cur, last = [], [], None
    for i in sorted(per):
        if not kern[i].startswith("k_"):
            if cur:
                groups.append(cur)
            cur = []
            continue
        cur.append(i)
    if cur:
        groups.append(cur)
    rows = []
    for g, t in zip(groups, timing):
        timed = g[1:]
        avg = {c: sum(per[i][c] for i in timed) / len(timed) for c in per[timed[0]]}
        rows.append({"kind": t["kind"], "buffer_gb": t["buffer_gb"], "kernel": kern[timed[0]],
                     "accesses_per_launch": t["random_loads"] / 5, "counters_per_launch": avg})
    out["passes"][name] = rows
print(json.dumps(out, indent=1))
