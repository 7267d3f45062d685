#!/bin/bash
# Robot-scene auto-reset launch: one wavefront per env vs a capped grid scanning the mask (MG_RESET_WAVES).
set -u
TAG=${1:-rw}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
MG_RESET_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "(rollout_parity or reset_paths or masked_reset) and (MoveTo)" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  for w in 0 128 512; do
    log="$OUT/bench.$env.w$w.log"
    MG_RESET_WAVES=$w timeout -k 10 200 python bench.py --env $env --steps 100 --warmup 10 --no-cpu-baseline > "$log" 2>&1 || { echo "bench FAIL"; tail -5 "$log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env waves $w', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'])"
  done
done
MG_RESET_WAVES_SHADOW=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "(rollout_parity or reset_paths or layout_retry) and (Cluster or MatchRegions or FindDupe)" \
    --timeout 120 --timeout-method thread > "$OUT/pytest_shadow.log" 2>&1 || { echo "pytest shadow FAIL"; tail -30 "$OUT/pytest_shadow.log"; exit 1; }
tail -1 "$OUT/pytest_shadow.log"
for cfg in ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  for w in 512 0; do
    log="$OUT/bench.$env.sw$w.log"
    MG_RESET_WAVES_SHADOW=$w timeout -k 10 200 python bench.py --env $env --envs $n --steps 100 --warmup 10 --no-cpu-baseline > "$log" 2>&1 || { echo "bench FAIL"; tail -5 "$log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$env shadow waves $w', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'])"
  done
done
