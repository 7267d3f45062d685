#!/bin/bash
# round 3: compact-gather / restack / fixture GPU tests, the full GPU suite, default bench, restack cost
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/${1:-r03_gather}"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gather or restack or replay_matches_reference" > "$OUT/pytest_new.log" 2>&1
rc=$?; echo "new gpu tests rc=$rc"; tail -3 "$OUT/pytest_new.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/restack_bench.py MoveToRegion-Demo-LoRes4E-v0 4096 8 > "$OUT/restack.log" 2>&1 || exit 1
timeout -k 10 200 python tools/restack_bench.py ClusterColour-Demo-LoResStack-v0 8192 8 >> "$OUT/restack.log" 2>&1 || exit 1
cat "$OUT/restack.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-600
exit $rc
