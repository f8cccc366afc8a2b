#!/bin/bash
# Round 6: K4's unit-record read, A/B on one box. MTB_UNIFORM_UNITS=1 gives every
# read 6 K1 units per mate, so the join rebuilds a matched query's info and segment bounds from its
# slot and a 4-B read-length word instead of a 16-B record of the 640-MB unit array; =0 is round 5.
# 1) same-box headline A/B through bench.py --ab (the GTDB-scale DB built once, specs interleaved);
# 2) per-kernel HBM bytes of the last 3.33M-pair batch for each side (separate FETCH_SIZE / WRITE_SIZE
#    passes, tools/kernel_bytes.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/uniform
mkdir -p $O
GB=3333334
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
timeout -k 10 420 python3 bench.py --skip-config2 --long-reads 0 --variants= --cold-pairs 0 $Q --steps 3 --ab-repeat 3 \
    --ab 'round5=MTB_UNIFORM_UNITS=0;uniform=MTB_UNIFORM_UNITS=1' > $O/ab.json 2> $O/ab.log
CMD="bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 --variants= --gtdb-pairs $GB --gtdb-batch $GB --cold-pairs 0 $Q"
for U in 0 1; do
    mkdir -p $O/u$U
    MTB_UNIFORM_UNITS=$U timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/u$U/fetch -o run -- python3 $CMD > /dev/null 2> $O/u$U/fetch.log
    MTB_UNIFORM_UNITS=$U timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/u$U/write -o run -- python3 $CMD > /dev/null 2> $O/u$U/write.log
    python3 tools/kernel_bytes.py $O/u$U > $O/u$U/kernel_bytes.json
    rm -f $O/u$U/fetch/run_counter_collection.csv $O/u$U/write/run_counter_collection.csv
done
