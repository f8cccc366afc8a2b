# File -> TSV pipeline timeline (experiments): the e2e lines only, one trace line per batch (MTB_PIPE_TRACE).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/pipe_trace.txt
MTB_PIPE_TRACE=gpurun_out/pipe_trace.txt timeout -k 10 500 python -u bench.py --skip-config2 --cpu-sample 0 --long-reads 0 \
  --variants "" --em-pairs 0 --steps 1 --warmup 0 --e2e-repeat 2 "$@" > gpurun_out/e2e_trace.json 2> gpurun_out/e2e_trace.log
