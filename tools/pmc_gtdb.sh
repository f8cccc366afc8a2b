#!/bin/bash
# rocprofv3 for one config-3 batch (1M pairs vs the 12G-k-mer GTDB-scale DB): a kernel trace and
# FETCH_SIZE / WRITE_SIZE passes, each its own run (no tracing domains combined with --pmc).
# Output under gpurun_out/pmc_gtdb/ (counter files cut to the library's kernels by
# tools/pmc_filter.py); summarise with tools/stage_profile.py (step 0).
set -e
mkdir -p gpurun_out/pmc_gtdb
export TMPDIR=/tmp
B="python bench.py --skip-config2 --steps 1 --warmup 0 --cpu-sample 0 --long-reads 0 --gtdb-pairs 1000000"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pmc_gtdb/trace -o run -- $B > gpurun_out/pmc_gtdb/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_gtdb/fetch -o run -- $B > gpurun_out/pmc_gtdb/fetch.log 2>&1
python tools/pmc_filter.py gpurun_out/pmc_gtdb/fetch
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_gtdb/write -o run -- $B > gpurun_out/pmc_gtdb/write.log 2>&1
python tools/pmc_filter.py gpurun_out/pmc_gtdb/write
