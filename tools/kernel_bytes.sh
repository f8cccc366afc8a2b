#!/bin/bash
# Per-kernel HBM bytes of the config-3 headline batch (FETCH_SIZE doubled + WRITE_SIZE, separate passes),
# with the kernel trace's per-kernel time, for the K5 / K6 kernels' bandwidth: one warm-up + one timed
# 3.33M-pair batch; tools/kernel_bytes.py sums the counters per kernel over the timed batch.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/kbytes
mkdir -p $O
GB=3333334
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
CMD="bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 --variants= --gtdb-pairs $GB --gtdb-batch $GB --cold-pairs 0 $Q"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 $CMD > /dev/null 2> $O/fetch.log
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 $CMD > /dev/null 2> $O/write.log
python3 tools/kernel_bytes.py $O > $O/kernel_bytes.json
rm -f $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv
