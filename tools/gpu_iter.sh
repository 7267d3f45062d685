#!/bin/bash
# one iteration on the GPU box: parity tests (optionally a subset), then the four BASELINE configs' bench lines
# gpurun -- 'bash tools/gpu_iter.sh <tag> [test path|none]'
set -u
TAG=${1:-iter}; TESTS=${2:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
if [ "$TESTS" != none ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest -m gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
bash tools/gpu_configs.sh
