#!/bin/bash
# round 4: pipelined pool with 2 / 3 chunks (robot scenes), parity of the pool.
set -u
TAG=${1:-pipe3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "pipelined_pool" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  for c in 2 3; do
    log="$OUT/bench.$env.c$c.log"
    timeout -k 10 200 python bench.py --env $env --steps 100 --warmup 10 --no-cpu-baseline --chunks $c > "$log" 2>&1 || { echo "bench FAIL $env $c"; tail -5 "$log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env chunks $c', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'], d['env_errors'])"
  done
done
