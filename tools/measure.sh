#!/bin/bash
# One measurement round on the GPU box: the default bench line, a rocprofv3 kernel trace of the
# same command, and FETCH_SIZE / WRITE_SIZE passes (separately, no tracing domains) of one step.
# Output under gpurun_out/meas/; summarise with tools/stage_profile.py and copy to profiles/.
set -e
mkdir -p gpurun_out/meas
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/meas/bench.json 2> gpurun_out/meas/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/meas/trace -o run -- python bench.py \
    > gpurun_out/meas/bench_traced.json 2> gpurun_out/meas/bench_traced.err
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d gpurun_out/meas/fetch -o run -- \
    python bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/meas/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d gpurun_out/meas/write -o run -- \
    python bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/meas/write.log 2>&1
