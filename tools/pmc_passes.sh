set -e
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --cpu-sample 0"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -f csv -d gpurun_out/pmc/sq -o run -- $B > gpurun_out/pmc/sq.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d gpurun_out/pmc/fetch -o run -- $B > gpurun_out/pmc/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d gpurun_out/pmc/write -o run -- $B > gpurun_out/pmc/write.log 2>&1
