"""Per-kernel table from tools/pmc_passes.sh output (per-dispatch averages).

Usage: python tools/pmc_table.py gpurun_out/pmc [kernel-substring ...]
FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 reports half the bytes of a wide streaming read).
"""
import collections
import csv
import os
import sys


def load(path):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mtb::", "")
        vals[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
    return vals, {k: len(v) for k, v in disp.items()}


def main():
    root = sys.argv[1]
    filt = sys.argv[2:]
    data = {}
    for p in ("sq", "mix", "fetch", "write"):
        f = os.path.join(root, p, "run_counter_collection.csv")
        if os.path.exists(f):
            data[p] = load(f)
    sq, nsq = data["sq"]
    names = sorted(sq, key=lambda k: -sq[k].get("SQ_WAVE_CYCLES", 0))
    for k in names:
        if filt and not any(f in k for f in filt):
            continue
        n = max(1, nsq[k])
        s = sq[k]
        wc = max(1.0, s.get("SQ_WAVE_CYCLES", 1))
        line = [f"{k[:38]:38s} x{n}", f"waves {s['SQ_WAVES'] / n:9.0f}",
                f"wait {s['SQ_WAIT_ANY'] / wc:.2f} winst {s['SQ_WAIT_INST_ANY'] / wc:.2f} act {s['SQ_ACTIVE_INST_ANY'] / wc:.2f}"
                f" valu {s['SQ_ACTIVE_INST_VALU'] / wc:.2f} vmem {s['SQ_ACTIVE_INST_VMEM'] / wc:.2f}"]
        if "mix" in data:
            m, nm = data["mix"]
            mm = m.get(k, {})
            c = max(1, nm.get(k, 1))
            line.append(f"VALU/wave {mm.get('SQ_INSTS_VALU', 0) / c / max(1, s['SQ_WAVES'] / n):7.0f}"
                        f" LDS/wave {mm.get('SQ_INSTS_LDS', 0) / c / max(1, s['SQ_WAVES'] / n):6.0f}"
                        f" VMRD/wave {mm.get('SQ_INSTS_VMEM_RD', 0) / c / max(1, s['SQ_WAVES'] / n):5.0f}"
                        f" bankc {mm.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, mm.get('SQ_ACTIVE_INST_LDS', 1)):.2f}")
        if "fetch" in data:
            f, nf = data["fetch"]
            line.append(f"fetchGB {2 * f.get(k, {}).get('FETCH_SIZE', 0) * 1024 / 1e9 / max(1, nf.get(k, 1)):.2f}")
        if "write" in data:
            w, nw = data["write"]
            line.append(f"writeGB {w.get(k, {}).get('WRITE_SIZE', 0) * 1024 / 1e9 / max(1, nw.get(k, 1)):.2f}")
        print(" | ".join(line))


if __name__ == "__main__":
    main()
