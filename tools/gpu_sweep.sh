#!/bin/bash
# bench one config under several env-var settings: gpu_sweep.sh <env> <envs> "<VAR=x VAR2=y>" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/sw
export PYTHONDONTWRITEBYTECODE=1
ENV=$1; N=$2; shift 2
i=0
for setting in "$@"; do
  i=$((i+1)); log=gpurun_out/sw/$ENV.$i.log
  env $setting timeout -k 10 200 python bench.py --env $ENV --envs $N --steps 20 --warmup 5 --no-cpu-baseline > $log 2>&1 || { echo "FAIL $setting"; tail -5 $log; exit 1; }
  python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$ENV', '$setting', round(d['value']), d['kernel_ms_per_step'], 'errors', d['env_errors'])"
done
