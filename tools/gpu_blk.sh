#!/bin/bash
# envs-per-workgroup sweep of the robot-scene step kernels (MG_STEP_BLK: 16 / 4 / 1 envs per workgroup)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/blk
export PYTHONDONTWRITEBYTECODE=1
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  for b in 16 4 1; do
    log=gpurun_out/blk/$env.$b.log
    MG_STEP_BLK=$b timeout -k 10 200 python bench.py --env $env --envs 4096 --steps 60 --warmup 10 --no-cpu-baseline > $log 2>&1 || { echo "FAIL $env $b"; tail -5 $log; exit 1; }
    python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env', 'MG_STEP_BLK=$b', round(d['value']), d['kernel_ms_per_step'], 'errors', d['env_errors'])"
  done
done
