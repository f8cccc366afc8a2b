#!/bin/bash
# Round-2 measurement: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (each its own run) of
# one config-3 1M-pair batch, and a kernel trace of the config-3 long-read line (25k ONT-like reads).
# Output under gpurun_out/r02/; summarise with tools/stage_profile.py and copy to profiles/r02/.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
B="python3 bench.py --skip-config2 --steps 1 --warmup 0 --cpu-sample 0 --long-reads 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --variants= --gtdb-pairs 1000000"
if [ "$SKIP_TRACE" != 1 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $B > $O/trace.log 2>&1
python3 tools/stage_profile.py time $O/trace/run_kernel_trace.csv 0 > $O/stage_time_gtdb.json
rm -f $O/trace/run_kernel_trace.csv
fi
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1
python3 tools/pmc_filter.py $O/fetch
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/write -o run -- $B > $O/write.log 2>&1
python3 tools/pmc_filter.py $O/write
python3 tools/stage_profile.py bytes $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv 0 > $O/stage_bytes_gtdb.json
L="python3 bench.py --skip-config2 --gtdb-pairs 2000 --gtdb-batch 1000 --steps 1 --warmup 1 --cpu-sample 0 --long-reads 50000 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --variants="
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/long -o run -- $L > $O/long.log 2>&1
rm -f $O/long/run_kernel_trace.csv
