#!/bin/bash
# Kernel trace of one config-3 batch and one batch of the "related" DB variant (sister species in
# genera): step 0 = config 3, step 1 = related. Summaries under gpurun_out/r02/.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
B="python3 bench.py --skip-config2 --steps 1 --warmup 0 --cpu-sample 0 --long-reads 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --gtdb-pairs 1000000 --variants related"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rel -o run -- $B > $O/rel.log 2>&1
python3 tools/stage_profile.py time $O/rel/run_kernel_trace.csv 1 > $O/stage_time_related.json
rm -f $O/rel/run_kernel_trace.csv
