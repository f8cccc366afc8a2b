#!/bin/bash
# Round-6 measurement (the recipe of rounds 4-5): per workload, a rocprofv3 kernel trace and separate FETCH_SIZE / WRITE_SIZE
# passes (each its own run; no tracing domains with --pmc) of one timed batch after one warm-up
# batch; summarised into profiles-ready JSON by tools/traffic_json.py.
#   gtdb     config 3: one GTDB_BATCH-pair batch (the bench's QuerySplit, 3333334) vs the 12G-k-mer GTDB-scale DB
#   long     config 4: one 62.5k-read batch of ONT-like reads vs the same DB
#   related  config 3's "related" DB variant
#   syncmer  config 3's syncmer DB variant
#   conserved config 3's heavy-tailed "conserved" DB variant
#   config2  config 2: 1M pairs vs the 0.98G-k-mer DB
# Usage: tools/measure_r06.sh [workload ...]   (default: all). Output: gpurun_out/r06/prof/<workload>/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/prof${TAG:+_$TAG}  # TAG: a variant run (e.g. TAG=sweep MTB_JOIN=sweep) in its own directory
mkdir -p $O
Q="--skewed-pairs 0 --cold-gtdb 0 --cpu-sample 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --em-pairs 0 --c5-kmers 0"
declare -A CMD STEP BATCH
GB=${GTDB_BATCH:-3333334}  # the headline's QuerySplit (the join follows MTB_JOIN / MTB_FILTER of the environment)
VB=2000000; VB3=3333334  # the variants' QuerySplits (bench.py VARIANT_BATCH: related 2M, syncmer / conserved 3.33M)
CMD[gtdb]="bench.py --skip-config2 --steps 1 --warmup 1 --long-reads 0 --variants= --gtdb-pairs $GB --gtdb-batch $GB --cold-pairs 0 $Q"
STEP[gtdb]=1; BATCH[gtdb]=$GB
CMD[long]="bench.py --skip-config2 --steps 1 --warmup 0 --gtdb-pairs 2000 --gtdb-batch 1000 --variants= --long-reads 62500 --long-batch 62500 --cold-pairs 0 $Q"
STEP[long]=3; BATCH[long]=62500
CMD[related]="bench.py --variant-only related --steps 1 --warmup 1 --gtdb-pairs $VB $Q"
STEP[related]=1; BATCH[related]=$VB
CMD[syncmer]="bench.py --variant-only syncmer --steps 1 --warmup 1 --gtdb-pairs $VB3 $Q"
STEP[syncmer]=1; BATCH[syncmer]=$VB3
CMD[conserved]="bench.py --variant-only conserved --steps 1 --warmup 1 --gtdb-pairs $VB3 $Q"
STEP[conserved]=1; BATCH[conserved]=$VB3
CMD[config2]="bench.py --gtdb-kmers 0 --steps 1 --warmup 1 --long-reads 0 --cold-pairs 0 $Q"
STEP[config2]=1; BATCH[config2]=1000000
W="${@:-gtdb long related syncmer conserved config2}"
for w in $W; do
  D=$O/$w
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python3 ${CMD[$w]} > $D/bench.json 2> $D/trace.log
  python3 tools/stage_profile.py time $D/trace/run_kernel_trace.csv ${STEP[$w]} > $D/stage_time.json
  rm -f $D/trace/run_kernel_trace.csv
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $D/fetch -o run -- python3 ${CMD[$w]} > /dev/null 2> $D/fetch.log
  python3 tools/pmc_filter.py $D/fetch
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $D/write -o run -- python3 ${CMD[$w]} > /dev/null 2> $D/write.log
  python3 tools/pmc_filter.py $D/write
  python3 tools/stage_profile.py bytes $D/fetch/run_counter_collection.csv $D/write/run_counter_collection.csv ${STEP[$w]} > $D/stage_bytes.json
  python3 tools/traffic_json.py $w $D ${BATCH[$w]} > $D/stage_traffic_$w.json
  rm -f $D/fetch/run_counter_collection.csv $D/write/run_counter_collection.csv
  echo "measured $w"
done
