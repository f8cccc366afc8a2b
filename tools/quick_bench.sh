# Config-3 kernel timing without the CPU baseline (experiments): short-read line + long-read line.
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u bench.py --skip-config2 --cpu-sample 0 --steps 3 --warmup 1 "$@" > gpurun_out/qb.json 2> gpurun_out/qb.log
