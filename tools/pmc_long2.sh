#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the long-read line's kernels (2 x 25k
# ONT-like reads after a warm-up pair, small GTDB-scale DB build), summarised on the box per
# kernel: gpurun_out/r02/pmc_long_<counter>.txt (the raw per-dispatch CSVs are deleted).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
O=gpurun_out/r02
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/pmc_long_$c
  timeout -s KILL 400 rocprofv3 --kernel-trace --kernel-include-regex "mtb::k_(extract_filter|match<|radix|segsort|thin|compact|pack_live|run_|group|match_paths|combine|choose|compact_taxcnt|taxcnt|scan)" \
    --pmc $c -f csv -d $O/pmc_long_$c -o run -- python3 bench.py --skip-config2 --gtdb-pairs 2000 --gtdb-batch 1000 \
    --steps 1 --warmup 1 --cpu-sample 0 --long-reads 50000 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --variants "" \
    > $O/pmc_long_$c.log 2>&1
  python3 tools/pmc_sum.py $O/pmc_long_$c > $O/pmc_long_$c.txt 2>&1
  find $O/pmc_long_$c -name "*.csv" -size +1M -delete
done
