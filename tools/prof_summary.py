"""Summarise rocprofv3 CSV output (kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes)
into a committed markdown file under profiles/.

Usage: python tools/prof_summary.py <trace_kernel_stats.csv> <fetch_counter_collection.csv>
       <write_counter_collection.csv> <out.md> [label]

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half
the bytes of a wide coalesced streaming read, so HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
for such streams (other access widths are uncalibrated; both raw and corrected are listed).
"""
import collections
import csv
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("mtb::", "")


def main():
    stats, fetch, write, out = sys.argv[1:5]
    label = sys.argv[5] if len(sys.argv) > 5 else ""
    rows = list(csv.DictReader(open(stats)))
    pmc = collections.defaultdict(lambda: {"n": 0, "fetch": 0.0, "write": 0.0})
    for f, key in ((fetch, "fetch"), (write, "write")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            pmc[k][key] += float(r["Counter_Value"])
            if key == "fetch":
                pmc[k]["n"] += 1
    lines = [f"# rocprofv3 summary {label}", "",
             "Kernel trace (`rocprofv3 --kernel-trace --stats`), whole process (DB build + warmup + timed steps):", "",
             "| kernel | calls | total ms | avg ms | % |", "|---|---|---|---|---|"]
    for r in rows[:30]:
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    lines += ["", "PMC (separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes; per dispatch averages, GB):", "",
              "| kernel | dispatches | FETCH_SIZE GB | WRITE_SIZE GB | HBM GB (2*FETCH+WRITE) |", "|---|---|---|---|---|"]
    for k, v in sorted(pmc.items(), key=lambda kv: -(kv[1]["fetch"] + kv[1]["write"]))[:25]:
        n = max(1, v["n"])
        fe, wr = v["fetch"] * 1024 / n / 1e9, v["write"] * 1024 / n / 1e9
        lines.append(f"| {k} | {v['n']} | {fe:.3f} | {wr:.3f} | {2 * fe + wr:.3f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
