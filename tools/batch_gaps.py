"""Idle time between the kernels of each classify batch in a rocprofv3 kernel trace (no PMC: counter
collection stretches every gap). A batch starts at k_read_meta. Prints per batch its span, the kernels'
busy time and the largest gaps with the kernels around them.
Usage: python tools/batch_gaps.py <run_kernel_trace.csv> [batches]"""
import csv
import json
import sys


def main(path, last=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_read_meta" in r["Kernel_Name"]]
    out = []
    for a, b in zip(starts[-last - 1:], starts[-last:] + [len(rows)]):
        batch = rows[a:b]
        t0, t1 = int(batch[0]["Start_Timestamp"]), int(batch[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in batch)
        gaps = sorted(((int(y["Start_Timestamp"]) - int(x["End_Timestamp"]),
                        x["Kernel_Name"].split("(")[0].replace("void ", "")[-48:],
                        y["Kernel_Name"].split("(")[0].replace("void ", "")[-48:])
                       for x, y in zip(batch, batch[1:])), reverse=True)
        out.append({"span_ms": round((t1 - t0) / 1e6, 3), "busy_ms": round(busy / 1e6, 3),
                    "idle_ms": round((t1 - t0 - busy) / 1e6, 3), "dispatches": len(batch),
                    "gaps_over_20us": sum(1 for g in gaps if g[0] > 20000),
                    "largest_gaps_us": [[round(g / 1e3, 1), x, y] for g, x, y in gaps[:12]]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
