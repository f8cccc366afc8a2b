# SQ counters of the long-read line's K5/K6 kernels (one pass; kernel trace only), summarised on the
# box (the raw per-dispatch CSV is deleted).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_long
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "k_combine|k_choose|k_match_paths|k_thin|k_segsort|k_merge|k_chunk|k_run_|k_group" \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  -f csv -d gpurun_out/pmc_long -o run -- python3 bench.py --skip-config2 --gtdb-pairs 2000 --gtdb-batch 1000 --steps 1 --warmup 0 --cpu-sample 0 --long-reads 25000 > gpurun_out/pmc_long.log 2>&1
python3 tools/pmc_sum.py gpurun_out/pmc_long > gpurun_out/pmc_long_summary.txt 2>&1
find gpurun_out/pmc_long -name "*.csv" -size +1M -delete
