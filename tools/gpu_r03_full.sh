#!/bin/bash
# round-end check on one box: pytest -m gpu, smoke(), the default bench line, and the
# rocprofv3 kernel-trace stats of the same default bench command (summarised by prof_summary.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/${1:-r03_full}"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-900; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof/stats" -o run -- python "$R/bench.py" --no-cpu-baseline > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python tools/prof_summary.py "$OUT/prof" --md > "$OUT/kernel_trace_stats.md"; rc=$?
cat "$OUT/kernel_trace_stats.md"; rm -rf "$OUT/prof"
exit $rc
