# Config 3 with batches spread over two contexts on the GPU (experiments): 1M-pair batches, 1 vs 2 contexts.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 400 python -u bench.py --skip-config2 --cpu-sample 0 --long-reads 0 --variants "" --e2e-pairs 0 \
    --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --steps 3 --warmup 1 --gtdb-batch 1000000 --gtdb-contexts $k \
    > gpurun_out/dual_$k.json 2> gpurun_out/dual_$k.log || exit $?
done
