#!/bin/bash
# Step-kernel envs-per-workgroup A/B (MG_STEP_BLK) on the robot scenes + phase profiles of the step kernel.
# gpurun -- 'bash tools/gpu_blk_ab.sh <tag> "16 8 4"'
set -u
TAG=${1:-blk}; BLKS=${2:-"16 8 4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "step_kernel_forms" \
    --timeout 120 --timeout-method thread > "$OUT/pytest_forms.log" 2>&1
rc=$?; echo "forms rc=$rc"; tail -3 "$OUT/pytest_forms.log"; [ $rc -eq 0 ] || exit $rc
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  blks=$BLKS; [ $env = MoveToCorner-Demo-LoRes4E-v0 ] && blks=16
  for b in $blks; do
    log="$OUT/bench.$env.$b.log"
    MG_STEP_BLK=$b timeout -k 10 200 python bench.py --env $env --envs 4096 --steps 60 --warmup 10 --no-cpu-baseline > "$log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench FAIL $env $b rc=$rc"; tail -5 "$log"; exit $rc; }
    python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$env BLK=$b', round(d['value']), 'step', k['step_kernel'], 'render', k['render_kernel'])"
  done
  MG_STEP_BLK=16 timeout -k 10 200 python tools/gpu_phase.py $env 4096 20 > "$OUT/phase.$env.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "phase FAIL rc=$rc"; tail -5 "$OUT/phase.$env.log"; exit $rc; }
  grep -A14 "^physics" "$OUT/phase.$env.log"
done
for env in ClusterColour-Demo-LoResStack-v0 MatchRegions-TestAll-LoRes4E-v0; do
  timeout -k 10 200 python tools/gpu_phase.py $env 8192 10 > "$OUT/phase.$env.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "phase FAIL rc=$rc"; tail -5 "$OUT/phase.$env.log"; exit $rc; }
  grep -A14 "^physics" "$OUT/phase.$env.log"
done
