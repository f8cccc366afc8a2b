#!/bin/bash
# Same-box A/B of head-first lines (MTB_PERMUTE) on the config-3 short-read line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="python -u bench.py --skip-config2 --cpu-sample 0 --steps 3 --warmup 1 --long-reads 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --variants="
MTB_PERMUTE=0 timeout -k 10 400 $B > gpurun_out/ab_perm0.json 2> gpurun_out/ab_perm0.log || exit 1
MTB_PERMUTE=1 timeout -k 10 400 $B > gpurun_out/ab_perm1.json 2> gpurun_out/ab_perm1.log
