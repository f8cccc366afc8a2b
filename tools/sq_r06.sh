#!/bin/bash
# Round 6: SQ wave-state counters of the headline's kernels on the final build (one config-3 batch after
# a warm-up batch, measure_r06.sh's gtdb command), each pass its own run, no tracing domains; per-kernel
# per-dispatch averages by tools/pmc_sum.py -> gpurun_out/r06/sq/summary.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/sq
mkdir -p $O
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
GB=3333334
CMD="bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 --variants= --gtdb-pairs $GB --gtdb-batch $GB --cold-pairs 0 $Q"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM -f csv -d $O/sq -o run -- python3 $CMD > $O/sq.log 2>&1
python3 tools/pmc_filter.py $O/sq
python3 tools/pmc_sum.py $O/sq > $O/summary.txt
rm -f $O/sq/run_counter_collection.csv
