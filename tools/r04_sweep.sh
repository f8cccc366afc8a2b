#!/bin/bash
# Round 4: the headline at larger QuerySplits now that K6 scratch lives in dead buffers, and the
# "related" variant at 2M-pair batches. One JSON line per run in gpurun_out/.
set -o pipefail
common="--skip-config2 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --long-reads 0 --cpu-sample 0 --cold-pairs 0 --steps 3 --warmup 1"
for b in ${BATCHES:-3000000 4000000}; do
  timeout -k 10 300 python -u bench.py $common --variants "" --gtdb-batch $b --detail gpurun_out/sweep_${b}_detail.json \
    > gpurun_out/sweep_${b}.json 2> gpurun_out/sweep_${b}.log || exit $?
done
for b in ${VBATCHES:-2000000}; do
  timeout -k 10 300 python -u bench.py $common --variant-only related --variant-batch $b \
    > gpurun_out/vb_related_${b}.json 2> gpurun_out/vb_related_${b}.log || exit $?
done
