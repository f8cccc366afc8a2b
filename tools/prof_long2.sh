#!/bin/bash
# Kernel statistics of the config-3 long-read line (2 x 25k ONT-like reads, warm-up included) on a
# small GTDB-scale DB build: gpurun_out/r02/long2/run_kernel_stats.csv (the DB build's kernels are
# listed too, under their own names).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
rm -rf $O/long2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/long2 -o run -- python3 bench.py --skip-config2 \
  --gtdb-pairs 2000 --gtdb-batch 1000 --steps 1 --warmup 1 --cpu-sample 0 --long-reads 50000 --e2e-pairs 0 \
  --e2e-gzip-pairs 0 --em-pairs 0 --variants "" > $O/long2.log 2>&1
rm -f $O/long2/run_kernel_trace.csv
