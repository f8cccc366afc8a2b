"""Per-kernel bytes and time of the last classify batch in tools/kernel_bytes.sh's counter passes: the
dispatches from the last k_read_meta (a batch's first kernel) to the end, grouped by kernel name.
FETCH_SIZE is doubled (profiles/r05/random_fetch_calibration.json: random and streaming reads alike)."""
import collections
import csv
import json
import os
import sys


def last_batch(path, counter):
    rows = list(csv.DictReader(open(path)))
    per = collections.OrderedDict()
    for r in rows:
        d = int(r["Dispatch_Id"])
        e = per.setdefault(d, {"name": r["Kernel_Name"].split("(")[0].replace("void ", ""), "v": 0.0,
                                "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        if r["Counter_Name"] == counter:
            e["v"] += float(r["Counter_Value"])
    ids = list(per)
    starts = [i for i in ids if per[i]["name"].endswith("k_read_meta")]
    first = starts[-1] if starts else ids[0]
    out = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for i in ids[ids.index(first):]:
        o = out[per[i]["name"]]
        o[0] += per[i]["v"] * 1024
        o[1] += per[i]["ns"] * 1e-6
        o[2] += 1
    return out


d = sys.argv[1]
f = last_batch(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
w = last_batch(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
rows = []
for k in f:
    fb, ms, n = 2 * f[k][0], f[k][1], f[k][2]
    wb = w[k][0] if k in w else 0.0
    rows.append({"kernel": k, "launches": n, "ms": round(ms, 3), "fetch_gb": round(fb / 1e9, 3), "write_gb": round(wb / 1e9, 3),
                 "tb_per_s": round((fb + wb) / (ms * 1e-3) / 1e12, 2) if ms > 0 else None})
rows.sort(key=lambda r: -r["ms"])
print(json.dumps({"source": "tools/kernel_bytes.sh (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, last batch)", "kernels": rows}, indent=1))
