#!/bin/bash
# Same-box A/B of the file -> TSV pipeline's contexts per GPU (bench end_to_end lines: 10M pairs plain +
# BGZF, three runs each): --e2e-contexts 1 (one context, batches from its whole HBM share) against 2,
# alternated twice. Output: gpurun_out/r05/e2e_ctx/ctx<n>_<k>.json (+ MTB_PIPE_TRACE timelines)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/e2e_ctx
mkdir -p $O
B="python -u bench.py --skip-config2 --steps 1 --warmup 0 --variants= --em-pairs 0 --c5-kmers 0 --long-reads 0 --cpu-sample 0 --gtdb-cpu-sample 0 --cold-gtdb 0 --skewed-pairs 0 --cold-pairs 0 --e2e-gzip-pairs 0 --e2e-repeat 3"
for k in 1 2; do
  for n in 2 1; do
    MTB_PIPE_TRACE=$O/trace_ctx${n}_$k.txt timeout -k 10 400 $B --e2e-contexts $n > $O/ctx${n}_$k.json 2> $O/ctx${n}_$k.log || exit 1
    grep "end to end" $O/ctx${n}_$k.log | cut -c1-90
  done
done
