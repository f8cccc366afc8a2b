#!/bin/bash
# SQ / instruction-mix counters for one config-3 batch, each pass its own run (no tracing domains).
set -e
mkdir -p gpurun_out/pmc_gtdb
export TMPDIR=/tmp
B="python bench.py --skip-config2 --steps 1 --warmup 0 --cpu-sample 0 --gtdb-pairs 1000000"
pass() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -f csv -d gpurun_out/pmc_gtdb/$name -o run -- $B > gpurun_out/pmc_gtdb/$name.log 2>&1
    python tools/pmc_filter.py gpurun_out/pmc_gtdb/$name
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
pass mix SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
pass fetch FETCH_SIZE
pass write WRITE_SIZE
