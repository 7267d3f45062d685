#!/bin/bash
# selected GPU tests, then bench lines: gpurun -- 'bash tools/gpu_sel.sh <tag> "<pytest -k expr>" [env ...]'
# (each step under its own time limit; the script stops at the first failure)
set -u
TAG=${1:-sel}; SEL=${2:-}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for ENV in "$@"; do
  N=4096; case $ENV in Cluster*|MatchRegions*) N=8192;; esac
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env "$ENV" --envs $N > "$OUT/bench.$ENV.log" 2>&1
  rc=$?; echo "bench $ENV rc=$rc"; tail -1 "$OUT/bench.$ENV.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], {k: d['kernels'][k]['ms'] for k in ('step_kernel', 'render_kernel')}, d['kernels']['timing'])"; [ $rc -eq 0 ] || exit $rc
done
exit 0
