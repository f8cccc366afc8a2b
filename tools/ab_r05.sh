#!/bin/bash
# Round-5 same-box A/Bs on the config-3 headline (bench.py --ab: the GTDB-scale DB built once, one
# fresh context per spec, specs interleaved). Usage: tools/ab_r05.sh NAME 'spec;spec;...' [repeat]
# AB_EXTRA: more bench flags (e.g. --ab-skewed). Output: gpurun_out/r05/ab_<NAME>.json (+ .err)
set -e
O=gpurun_out/r05
mkdir -p $O
Q="--skip-config2 --long-reads 0 --variants= --cold-pairs 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --skewed-pairs 0"
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 $Q --ab "$2" --ab-repeat ${3:-2} $AB_EXTRA > $O/ab_$1.json 2> $O/ab_$1.err
grep "bench ab" $O/ab_$1.err
