#!/bin/bash
# Round 6: K1F's diagnostic passes (MTB_AB_FILTER=1: after each batch's real pass, the same pass with
# probes and no output, then with neither) on one headline batch, link lines on and off.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
for L in 1 0; do
  MTB_AB_FILTER=1 MTB_LINK_LINES=$L timeout -k 10 300 python3 bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 \
      --variants= --gtdb-pairs 3333334 --gtdb-batch 3333334 --cold-pairs 0 $Q > gpurun_out/r06/filter_diag_link$L.json \
      2> gpurun_out/r06/filter_diag_link$L.log
  grep "mtb ab filter" gpurun_out/r06/filter_diag_link$L.log | tail -2
done
