#!/bin/bash
# SQ counters of the config-3 batch's K5 / K6 kernels (one warm-up + one timed 3.33M-pair batch): where
# their waves wait (SQ_WAIT_ANY: parked on s_waitcnt / barriers; SQ_WAIT_INST_ANY: issue stalls) and
# what they issue (VALU / LDS), plus LDS bank conflicts. One pass (8 SQ counters), kernels by regex.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/sq
mkdir -p $O
GB=3333334
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
CMD="bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 --variants= --gtdb-pairs $GB --gtdb-batch $GB --cold-pairs 0 $Q"
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "k_segsort_regs|k_match_paths|k_choose_taxon_group|k_match<|k_radix_scatter|k_pack_live" \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
  -f csv -d $O/p1 -o run -- python3 $CMD > /dev/null 2> $O/p1.log
python3 - <<'PY'
import csv, collections, json
rows = list(csv.DictReader(open("gpurun_out/r05/sq/p1/run_counter_collection.csv")))
last = {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    d = int(r["Dispatch_Id"])
    last.setdefault(k, {}).setdefault(d, {})[r["Counter_Name"]] = last.get(k, {}).get(d, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {}
for k, ds in last.items():
    d = max(ds)  # the timed batch's dispatch (the last one of the name)
    c = ds[d]
    w = c.get("SQ_WAVE_CYCLES", 1.0) or 1.0
    out[k] = {n: round(v / w, 3) for n, v in c.items() if n != "SQ_WAVE_CYCLES"}
    out[k]["SQ_WAVE_CYCLES"] = c.get("SQ_WAVE_CYCLES")
json.dump(out, open("gpurun_out/r05/sq/sq_summary.json", "w"), indent=1)
for k, v in out.items(): print(k, v)
PY
