#!/bin/bash
# round 4: pipelined chunks x envs per step workgroup (comparison build: MG_STEP_BLK=8 halves the step
# kernel's LDS per workgroup, so render workgroups can share its CUs).
# gpurun -- 'bash tools/gpu_r04_pipeblk.sh <tag>'
set -u
TAG=${1:-pipeblk}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1 MAGICAL_AMD_EXP_LIB=allforms
for env in MoveToRegion-Demo-LoRes4E-v0; do
  for c in 1 2 4; do
    for b in 16 8; do
      log="$OUT/bench.$env.c$c.b$b.log"
      MG_STEP_BLK=$b timeout -k 10 200 python bench.py --env $env --steps 100 --warmup 10 --no-cpu-baseline --chunks $c > "$log" 2>&1 || { echo "bench FAIL $env $c $b"; tail -5 "$log"; exit 1; }
      python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env chunks $c blk $b', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'], d['env_errors'])"
    done
  done
done
