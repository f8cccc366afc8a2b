#!/bin/bash
# Same-box A/B of the file -> TSV pipeline (bench end_to_end lines only, 10M pairs plain / BGZF /
# single-member gzip), three runs per format: default (two contexts sharing the DB, mtb_clone) vs one
# context. Output: gpurun_out/r03/e2e_ab/<variant>.json
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03/e2e_ab
mkdir -p $O
B="python -u bench.py --skip-config2 --steps 1 --warmup 1 --variants= --em-pairs 0 --c5-kmers 0 --long-reads 0 --cpu-sample 0 --e2e-repeat 3"
timeout -k 10 500 env $B > $O/default.json 2> $O/default.log &&
timeout -k 10 500 env $B --e2e-contexts 1 > $O/one_ctx.json 2> $O/one_ctx.log
