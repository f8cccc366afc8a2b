#!/bin/bash
# A/B of env knobs on config 3 + the related variant (no CPU baseline): one bench run per setting,
# kernel times under gpurun_out/ab/<name>.json. Usage: ab_env.sh NAME=ENV[,ENV] ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env_args=$(echo "$envs" | tr ',' ' ')
  env $env_args timeout -k 10 300 python -u bench.py --skip-config2 --cpu-sample 0 --steps 3 --warmup 1 \
    --long-reads 0 --e2e-pairs 0 --e2e-gzip-pairs 0 --variants related > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.log
  grep "reads/s" gpurun_out/ab/$name.log
done
