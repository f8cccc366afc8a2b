cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_long -o run -- python3 bench.py --skip-config2 --gtdb-pairs 2000 --gtdb-batch 1000 --steps 1 --warmup 1 --cpu-sample 0 --long-reads 50000 > gpurun_out/prof_long.json 2> gpurun_out/prof_long.log
