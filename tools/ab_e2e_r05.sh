#!/bin/bash
# Same-box A/B of the file -> TSV pipeline (bench end_to_end lines only: 10M pairs plain + BGZF, three
# runs each), alternated twice over environment variants: VARIANTS="name:K=V,K=V name2:..." (default:
# the mapped file prefaulted ahead of the splitter or not). Output: gpurun_out/r05/e2e_ab/<name>_<k>.*
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/e2e_ab
mkdir -p $O
B="python -u bench.py --skip-config2 --steps 1 --warmup 0 --variants= --em-pairs 0 --c5-kmers 0 --long-reads 0 --cpu-sample 0 --gtdb-cpu-sample 0 --cold-gtdb 0 --skewed-pairs 0 --cold-pairs 0 --e2e-gzip-pairs 0 --e2e-repeat 3"
for k in 1 2; do
  for spec in ${VARIANTS:-noprefault:MTB_PREFAULT=0 prefault:MTB_PREFAULT=1}; do
    name=${spec%%:*}
    envs=${spec#*:}
    env ${envs//,/ } MTB_PIPE_TRACE=$O/trace_${name}_$k.txt timeout -k 10 400 $B --detail $O/${name}_${k}_detail.json > $O/${name}_$k.json 2> $O/${name}_$k.log || exit 1
    echo "$name #$k"; grep "end to end" $O/${name}_$k.log | cut -c1-70
  done
done
