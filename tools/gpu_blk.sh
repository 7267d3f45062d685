#!/bin/bash
# envs-per-workgroup sweep of the step kernel (MG_STEP_BLK for LDS variants, MG_STEP_BLK0 for the HBM kernel)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/blk
export PYTHONDONTWRITEBYTECODE=1
run() { # env envs var blk
  local log=gpurun_out/blk/$1.$4.$3.log
  env $4=$3 timeout -k 10 200 python bench.py --env $1 --envs $2 --steps 20 --warmup 5 --no-cpu-baseline > $log 2>&1 || { echo "FAIL $1 $4=$3"; tail -5 $log; exit 1; }
  python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$1', '$4=$3', round(d['value']), d['kernel_ms_per_step'], 'errors', d['env_errors'])"
}
for b in 16 4 1; do run MoveToRegion-Demo-LoRes4E-v0 4096 $b MG_STEP_BLK || exit 1; done
for b in 16 4 1; do run MoveToCorner-Demo-LoRes4E-v0 4096 $b MG_STEP_BLK || exit 1; done
for b in 64 8 1; do run ClusterColour-Demo-LoResStack-v0 8192 $b MG_STEP_BLK0 || exit 1; done
for b in 64 8 1; do run MatchRegions-TestAll-LoRes4E-v0 8192 $b MG_STEP_BLK0 || exit 1; done
