#!/bin/bash
# Round 6: kernel trace (no counters) of the headline workload, per-batch idle time between kernels
# (tools/batch_gaps.py), and the rocprofv3 --stats summary; then a rehearsal of `bench.py --gpus 2`
# through its own launcher on this one-GPU box (two ranks on cuda:0 over gloo; the values are not
# measurements, the path is: the launcher, the ranks' process group, the C1 gathers).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/trace
mkdir -p $O
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O -o run -- python3 bench.py --skip-config2 --steps 2 \
    --warmup 1 --long-reads 0 --variants= --cold-pairs 0 $Q > $O/bench.json 2> $O/bench.log
python3 tools/batch_gaps.py $O/run_kernel_trace.csv 3 > $O/gaps.json
rm -f $O/run_kernel_trace.csv
if [ "${REHEARSE:-1}" = 1 ]; then
  MTB_BENCH_ONE_DEVICE=1 MTB_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --gtdb-kmers 2e9 \
      --gtdb-pairs 1000000 --gtdb-batch 500000 --long-reads 20000 --long-batch 10000 --c5-kmers 0 --steps 2 --warmup 1 \
      --detail gpurun_out/r06/rehearsal_n2_detail.json > gpurun_out/r06/rehearsal_n2.json 2> gpurun_out/r06/rehearsal_n2.log
fi
