#!/bin/bash
# SQ counters of K5/K6 kernels on one batch of the "related" config-3 variant, one pass per
# MTB_PRUNE_AFTER mode given (e.g. pmc_k5.sh 0 2); summaries in gpurun_out/pmc_k5_<mode>.txt.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
for m in "$@"; do
  rm -rf gpurun_out/pmc_k5_$m
  MTB_PRUNE_AFTER=$m timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "k_segsort|k_match_paths|k_combine|k_choose|k_pack_live|k_compact_segments" \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    -f csv -d gpurun_out/pmc_k5_$m -o run -- python3 bench.py --variant-only related --gtdb-pairs 1000000 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/pmc_k5_$m.log 2>&1
  python3 tools/pmc_sum.py gpurun_out/pmc_k5_$m > gpurun_out/pmc_k5_$m.txt 2>&1
  find gpurun_out/pmc_k5_$m -name "*.csv" -size +1M -delete
done
