"""Per-kernel time and HBM bytes of one A/B variant (tools/ab_r03.sh): from a rocprofv3 --stats
kernel summary and separate FETCH_SIZE / WRITE_SIZE counter passes (KiB; FETCH_SIZE doubled per
MI355X_MICROARCH.md), the averages per launch of the timed batch's kernels that match the given
name fragments. Prints one JSON object."""
import csv
import json
import os
import sys
from collections import defaultdict

d, frags = sys.argv[1], sys.argv[2].split(",")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mtb::", "")


def pick(name):
    s = short(name)
    return next((f for f in frags if f in s), None)


out = {"variant": os.path.basename(d.rstrip("/")), "kernels": {}}
stats = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        if pick(r["Name"]):
            out["kernels"].setdefault(k, {})["avg_ms"] = round(float(r["AverageNs"]) / 1e6, 4)
            out["kernels"][k]["calls"] = int(r["Calls"])
for sub, counter, scale in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    per = defaultdict(list)
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == counter and pick(r["Kernel_Name"]):
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024 * scale)
    for k, v in per.items():
        # the last launch: the timed batch (the first is the warm-up)
        out["kernels"].setdefault(k, {})[counter.lower() + "_bytes"] = int(v[-1])
bench = os.path.join(d, "bench.json")
if os.path.exists(bench):
    lines = [l for l in open(bench).read().splitlines() if l.startswith("{")]
    if lines:
        b = json.loads(lines[-1])
        out["bench"] = {"value": b["value"], "kernel_ms": b.get("kernel_ms"), "parity_sample": b.get("parity_sample")}
print(json.dumps(out, indent=1))
