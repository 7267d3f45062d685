#!/bin/bash
# Pipelined pool: per-chunk stream priorities (MAGICAL_AMD_POOL_PRIO) and the capped reset grid.
set -u
TAG=${1:-pp}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  for pp in "0,0" "-1,0"; do
    log="$OUT/bench.$env.p$pp.log"
    MAGICAL_AMD_POOL_PRIO="$pp" timeout -k 10 200 python bench.py --env $env --steps 100 --warmup 10 --no-cpu-baseline > "$log" 2>&1 || { echo "bench FAIL"; tail -5 "$log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env prio $pp', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'])"
  done
done
