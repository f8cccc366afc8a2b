#!/bin/bash
# Same-box A/B of the config-3 headline line alone (3 timed steps after 1 warm-up, no CPU baseline,
# no side lines) under alternating environments. Usage: tools/ab_headline.sh NAME=ENV[,ENV...] ...
# (each spec runs AB_RUNS times (2), interleaved A B A B). Output: gpurun_out/r04/ab_head/<name>_<i>.json
set -e
O=gpurun_out/r04/ab_head
mkdir -p $O
Q="--skip-config2 --long-reads 0 --variants= --cold-pairs 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
for i in $(seq 1 ${AB_RUNS:-2}); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//,/ } timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 $Q --detail $O/${name}_$i.detail.json \
        > $O/${name}_$i.json 2> $O/${name}_$i.err
    python3 -c "import json; d=json.load(open('$O/${name}_$i.json')); print('$name', $i, d['value'], d['kernel_ms'])"
  done
done
