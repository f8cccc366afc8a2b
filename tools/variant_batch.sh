# DB variants at a given QuerySplit size (experiments): tools/variant_batch.sh <batch> <variant>...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$1; shift
for v in "$@"; do
  timeout -k 10 400 python -u bench.py --variant-only $v --cpu-sample 0 --steps 3 --warmup 1 --variant-batch $B \
    > gpurun_out/vb_${v}_$B.json 2> gpurun_out/vb_${v}_$B.log || exit $?
done
