#!/bin/bash
# physics iteration: parity tests + the two LDS-variant configs (+ optional multi-block)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/pq
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pq/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pq/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "$@"; do
  set -- $spec
  timeout -k 10 200 python bench.py --env $1 --envs $2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pq/$1.log 2>&1 || { echo "FAIL $1"; tail -5 gpurun_out/pq/$1.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/pq/$1.log').read().strip().splitlines()[-1]); print('$1', round(d['value']), d['kernel_ms_per_step'], 'errors', d['env_errors'])"
done
