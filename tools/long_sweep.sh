# Config-4 long-read line vs its batch size (experiments): the long-read line alone per batch size.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in "$@"; do
  timeout -k 10 400 python -u bench.py --skip-config2 --cpu-sample 0 --variants "" --e2e-pairs 0 --e2e-gzip-pairs 0 \
    --em-pairs 0 --c5-kmers 0 --gtdb-pairs 2000 --gtdb-batch 1000 --steps 3 --warmup 1 --long-batch $b \
    > gpurun_out/lsweep_$b.json 2> gpurun_out/lsweep_$b.log || exit $?
done
