#!/bin/bash
# Round 6 same-box A/B of the headline (config 3, 3 x 3.33M-pair batches per step): the GTDB-scale DB
# built once, a fresh context per spec under its environment, specs interleaved (bench.py --ab).
# Usage: ab_r06.sh NAME 'specA=K=V,K=V;specB=K=V' [repeats]  ->  gpurun_out/r06/ab_NAME.{json,log}
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
timeout -k 10 420 python3 bench.py --skip-config2 --long-reads 0 --variants= --cold-pairs 0 $Q --steps 3 \
    --ab-repeat ${3:-3} --ab "$2" > gpurun_out/r06/ab_$1.json 2> gpurun_out/r06/ab_$1.log
grep "bench ab" gpurun_out/r06/ab_$1.log
