#!/bin/bash
# Render-class changes: the render parity tests (forced class hand-overs, full-resolution frames, rollouts of
# the many-block configs, every registered name), then the many-block bench lines.
set -u
TAG=${1:-rcheck}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "step_kernel_forms or full_resolution or rollout_parity or every_registered or reset_paths" > "$OUT/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
for cfg in ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  log="$OUT/bench.$env.$rep.log"
  timeout -k 10 200 python bench.py --env $env --envs $n --steps 100 --warmup 10 --no-cpu-baseline > "$log" 2>&1 || { echo "bench FAIL"; tail -5 "$log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$env', round(d['value']), d['ms_per_step'], 'step', k['step_kernel'], 'render', k['render_kernel'])"
done
done
