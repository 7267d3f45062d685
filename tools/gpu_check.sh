#!/bin/bash
# Round-end check on one box: the full GPU parity suite, smoke(), then the bench line of every BASELINE
# config (optionally the emulated 8-rank receive side).  gpurun -- 'bash tools/gpu_check.sh <tag> [skip_tests] [emul]'
set -u
TAG=${1:-check}; SKIP=${2:-0}; EMUL=${3:-0}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
run() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { tail -30 "$OUT/$name.log"; exit $rc; }
}
line() { python3 -c "import json; d=json.loads(open('$OUT/$1.log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; g=d.get('gather') or {}; print('$1', round(d['value']), d['ms_per_step'], 'step', k['step_kernel'], 'reset', k['reset_kernel'], 'render', k['render_kernel'], 'chunks', d['config'].get('pipeline_chunks'), 'restack', g.get('restack_ms_per_step'))"; }
if [ "$SKIP" != 1 ]; then
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 MoveToCorner-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  run bench.$env 300 python bench.py --env $env --envs $n --steps 100 --warmup 10 --no-cpu-baseline && line bench.$env
done
if [ "$EMUL" = 1 ]; then
  for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192; do
    env=${cfg%%:*}; n=${cfg##*:}
    run emul8.$env 300 python bench.py --env $env --envs $n --steps 30 --warmup 10 --no-cpu-baseline --emulate-world 8 && line emul8.$env
  done
fi
echo done
