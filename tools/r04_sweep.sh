#!/bin/bash
# Round 4: the headline at larger QuerySplits (K6 scratch now lives in dead buffers) for the
# random-access join and the DB-sweep join (MTB_JOIN=sweep), and the "related" variant at 2M-pair
# batches. One JSON line per run in gpurun_out/.
set -o pipefail
common="--skip-config2 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --long-reads 0 --cpu-sample 0 --cold-pairs 0 --steps 3 --warmup 1"
for j in ${JOINS:-default sweep sweepnf}; do
  for b in ${BATCHES:-2000000 3000000}; do
    tag=${j}_${b}
    MTB_JOIN=$([ $j = default ] && echo "" || echo sweep) MTB_FILTER=$([ $j = sweepnf ] && echo 0 || echo 1) \
      timeout -k 10 300 python -u bench.py $common --variants "" \
      --gtdb-batch $b --detail gpurun_out/sw_${tag}_detail.json > gpurun_out/sw_${tag}.json 2> gpurun_out/sw_${tag}.log || exit $?
  done
done
for b in ${VBATCHES:-}; do
  MTB_JOIN=${VJOIN:-} timeout -k 10 300 python -u bench.py $common --variant-only related --variant-batch $b \
    > gpurun_out/vb_related_${b}.json 2> gpurun_out/vb_related_${b}.log || exit $?
done
