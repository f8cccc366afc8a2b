#!/bin/bash
# Same-box A/B of the file -> TSV pipeline (bench end_to_end lines only, 10M pairs plain / BGZF /
# single-member gzip), three runs per format: default (8 TSV format threads) vs 16
# (MTB_FORMAT_THREADS). Output: gpurun_out/r03/e2e_ab/<variant>.json
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03/e2e_ab
mkdir -p $O
B="python -u bench.py --skip-config2 --steps 1 --warmup 1 --variants= --em-pairs 0 --c5-kmers 0 --long-reads 0 --cpu-sample 0 --e2e-repeat 3"
timeout -k 10 500 env $B > $O/default.json 2> $O/default.log &&
timeout -k 10 500 env MTB_FORMAT_THREADS=16 $B > $O/fmt16.json 2> $O/fmt16.log
