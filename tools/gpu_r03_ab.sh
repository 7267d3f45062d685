#!/bin/bash
# targeted GPU tests (pytest -k expr), then bench lines of one config under each switch setting
# gpurun -- 'bash tools/gpu_r03_ab.sh <tag> "<pytest -k expr>" <env> <envs> "<VAR=val ...>" "<VAR=val ...>" ...'
# (an empty settings string = the defaults)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
TAG=$1; K=$2; ENVN=$3; N=$4; shift 4
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    timeout -k 10 200 env $setting python bench.py --env $ENVN --envs $N --steps 60 --warmup 10 --no-cpu-baseline > "$OUT/bench_$i.log" 2>&1 || { echo "bench FAIL [$setting]"; tail -5 "$OUT/bench_$i.log"; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_$i.log').read().strip().splitlines()[-1]); print($rep, '[$setting]', d['value'], d['kernel_ms_per_step'])"
  done
done
