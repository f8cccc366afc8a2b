#!/bin/bash
# The headline line alone (config 3, default steps / warmup / batches), N fresh processes on one box:
# its run-to-run spread. Output: gpurun_out/r05/repeats/run<k>.json
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/repeats
mkdir -p $O
Q="--skip-config2 --long-reads 0 --variants= --cold-pairs 0 --cpu-sample 0 --gtdb-cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --skewed-pairs 0 --cold-gtdb 0"
for k in $(seq 1 ${N:-4}); do
  timeout -k 10 300 python3 bench.py $Q --detail $O/run${k}_detail.json > $O/run$k.json 2> $O/run$k.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/run$k.json').read().strip().splitlines()[-1]); print($k, d['value'], d['ms_per_step'], d['kernel_ms'])"
done
