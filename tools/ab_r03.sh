#!/bin/bash
# Round-3 A/Bs on config 3 (1M-pair batch vs the 12G-k-mer GTDB-scale DB), same box, each variant a
# kernel-trace --stats run plus separate FETCH_SIZE / WRITE_SIZE passes (tools/ab_summary.py):
#   base      the default path
#   k6group   K6 chooseBestTaxon on a 16-lane group per read (MTB_WAVE_TAXON=2) instead of a thread
#   rankfree  K4 without the per-read rank atomic (MTB_AB_RANK_FREE=1: ranks are wrong and the results
#             invalid; an upper bound of what removing the atomic can save in the join)
#   dirfree   nor the read's stretch bounds (MTB_AB_RANK_FREE=2: no dirOff reads; invalid results)
# Usage: tools/ab_r03.sh [variant ...]. Output: gpurun_out/r03/ab/<variant>/ab.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03/ab
mkdir -p $O
CMD="bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 --variants= --gtdb-pairs 1000000 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
declare -A ENVS
ENVS[base]="MTB_AB_NONE=1"
ENVS[k6group]="MTB_WAVE_TAXON=2"
ENVS[rankfree]="MTB_AB_RANK_FREE=1"
ENVS[dirfree]="MTB_AB_RANK_FREE=2"
for v in ${@:-base k6group rankfree}; do
  D=$O/$v
  mkdir -p $D
  export ${ENVS[$v]}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python3 $CMD > $D/bench.json 2> $D/trace.log
  rm -f $D/trace/run_kernel_trace.csv
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $D/fetch -o run -- python3 $CMD > /dev/null 2> $D/fetch.log
  python3 tools/pmc_filter.py $D/fetch
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $D/write -o run -- python3 $CMD > /dev/null 2> $D/write.log
  python3 tools/pmc_filter.py $D/write
  python3 tools/ab_summary.py $D "k_match<,k_choose_taxon,k_match_paths,k_combine_paths,k_segsort" > $D/ab.json
  rm -f $D/fetch/run_counter_collection.csv $D/write/run_counter_collection.csv
  unset ${ENVS[$v]%%=*}
  echo "measured $v"
done
