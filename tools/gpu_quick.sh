#!/bin/bash
# quick GPU iteration: parity tests, short bench, phase profile
# gpurun -- 'bash tools/gpu_quick.sh <tag> [env] [envs]'
set -u
TAG=${1:-quick}; ENV=${2:-MoveToRegion-Demo-LoRes4E-v0}; N=${3:-4096}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --env "$ENV" --envs "$N" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gpu_phase.py "$ENV" "$N" 20 > "$OUT/phase.log" 2>&1
rc=$?; echo "phase rc=$rc"; cat "$OUT/phase.log"
exit $rc
