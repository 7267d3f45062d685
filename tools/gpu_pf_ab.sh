#!/bin/bash
# Robot scenes: next-layout shadow (MG_RESET_PREFETCH) x pipelined chunks.
set -u
TAG=${1:-pf}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  for pf in 1 0; do
    for c in 2 1; do
      log="$OUT/bench.$env.pf$pf.c$c.log"
      MG_RESET_PREFETCH=$pf timeout -k 10 200 python bench.py --env $env --steps 100 --warmup 10 --no-cpu-baseline --chunks $c > "$log" 2>&1 || { echo "bench FAIL"; tail -5 "$log"; exit 1; }
      python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env pf $pf chunks $c', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'])"
    done
  done
done
