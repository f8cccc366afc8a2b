# Config-3 device rate vs QuerySplit size (experiments): the headline line alone at several batch sizes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in "$@"; do
  timeout -k 10 400 python -u bench.py --skip-config2 --cpu-sample 0 --long-reads 0 --variants "" --e2e-pairs 0 \
    --e2e-gzip-pairs 0 --em-pairs 0 --steps 3 --warmup 1 --gtdb-batch $b > gpurun_out/sweep_$b.json 2> gpurun_out/sweep_$b.log || exit $?
done
