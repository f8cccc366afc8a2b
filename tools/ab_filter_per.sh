# Same-box A/B of the fused filter's probes per group (MTB_FILTER_PER 16 vs 8), config 3 at 2M-pair batches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ab_fp.log
for per in 16 8 16 8; do
  MTB_FILTER_PER=$per timeout -k 10 400 python -u bench.py --skip-config2 --cpu-sample 0 --long-reads 0 --variants "" \
    --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0 --steps 3 --warmup 1 > /dev/null 2> gpurun_out/ab_fp_run.log || exit $?
  echo "per $per: $(grep 'config 3:' gpurun_out/ab_fp_run.log | cut -c1-200)" >> gpurun_out/ab_fp.log
done
