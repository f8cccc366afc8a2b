#!/bin/bash
# Long-read line alone (config 4: 62.5k ONT-like reads vs the GTDB-scale DB) under A/B environments.
# Usage: [LONG_READS=n LONG_BATCH=b] tools/long_ab.sh NAME=ENV[,ENV...] ...   e.g. base= bitonic=MTB_PRUNE_AFTER=4
# Output: gpurun_out/r04/long_ab/<name>.json (the bench line) and .err
set -e
O=gpurun_out/r04/long_ab
mkdir -p $O
Q="--cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --cold-pairs 0"
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env ${envs//,/ } timeout -k 10 300 python3 bench.py --skip-config2 --steps 3 --warmup 1 --gtdb-pairs 2000 \
      --gtdb-batch 1000 --variants= --long-reads ${LONG_READS:-62500} --long-batch ${LONG_BATCH:-62500} $Q --detail $O/$name.detail.json \
      > $O/$name.json 2> $O/$name.err
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); l=d['long_reads']; print('$name', l['value'], l['ms_per_step'])"
done
