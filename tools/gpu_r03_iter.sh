#!/bin/bash
# iteration check on one box: the full GPU suite, then a short bench line of every BASELINE config
# (gpurun -- 'bash tools/gpu_r03_iter.sh <tag> [pytest -k expr]')
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/${1:-r03_iter}"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096" "MoveToCorner-Demo-LoRes4E-v0 4096" "ClusterColour-Demo-LoResStack-v0 8192" "MatchRegions-TestAll-LoRes4E-v0 8192"; do
  set -- $spec
  timeout -k 10 200 python bench.py --env $1 --envs $2 --steps 60 --warmup 10 --no-cpu-baseline > "$OUT/bench_$1.log" 2>&1 || { echo "bench FAIL $1"; tail -5 "$OUT/bench_$1.log"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['kernel_ms_per_step'])"
done
