# A/B of the config-3 join: the unstaged run-index join vs the LDS-window (DB-streaming) join, at
# 1M- and 2M-pair batches. Short-read line only.
cd $GRAFT_REPO_ROOT
B="python -u bench.py --skip-config2 --cpu-sample 0 --long-reads 0 --steps 2 --warmup 1"
timeout -k 10 400 env $B --gtdb-batch 1000000 > gpurun_out/ab_unstaged_1m.json 2> gpurun_out/ab_unstaged_1m.log &&
timeout -k 10 400 env MTB_STAGE_FREE_RATIO=1000000 MTB_RUN_INDEX=0 $B --gtdb-batch 1000000 > gpurun_out/ab_windows_1m.json 2> gpurun_out/ab_windows_1m.log &&
timeout -k 10 400 env $B --gtdb-batch 2000000 > gpurun_out/ab_unstaged_2m.json 2> gpurun_out/ab_unstaged_2m.log &&
timeout -k 10 400 env MTB_STAGE_FREE_RATIO=1000000 MTB_RUN_INDEX=0 $B --gtdb-batch 2000000 > gpurun_out/ab_windows_2m.json 2> gpurun_out/ab_windows_2m.log
