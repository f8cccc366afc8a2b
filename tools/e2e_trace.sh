# File -> TSV pipeline timeline (experiments): the e2e lines only, one trace line per batch (MTB_PIPE_TRACE).
# Usage: [E2E_ARGS=...] tools/e2e_trace.sh [tag]   (env knobs such as MTB_NO_MMAP pass through; outputs
# gpurun_out/e2e_trace<tag>.*)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-}
rm -f gpurun_out/pipe_trace$T.txt
MTB_PIPE_TRACE=gpurun_out/pipe_trace$T.txt timeout -k 10 500 python -u bench.py --skip-config2 --cpu-sample 0 --long-reads 0 \
  --variants "" --em-pairs 0 --c5-kmers 0 --steps 1 --warmup 0 --e2e-repeat 2 $E2E_ARGS > gpurun_out/e2e_trace$T.json 2> gpurun_out/e2e_trace$T.log
