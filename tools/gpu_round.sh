#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel-trace stats
# and the two PMC passes (FETCH_SIZE / WRITE_SIZE cannot share a pass).
# Usage (from the dev container):
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh <tag> [pytest|nopytest|<test path>] [bench args...]'
set -u
TAG=${1:-r01}
MODE=${2:-pytest}
shift 2 2>/dev/null
BARGS="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1

if [ "$MODE" != "nopytest" ]; then
  TESTS=tests; [ "$MODE" = "pytest" ] || TESTS="$MODE"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest -m gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || exit $rc
fi

timeout -k 10 400 python bench.py $BARGS > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"
[ $rc -eq 0 ] || exit $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
  python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline $BARGS > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/prof.log"; exit $rc; }

timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- \
  python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline $BARGS > "$OUT/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/pmc_fetch.log"; exit $rc; }

timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- \
  python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline $BARGS > "$OUT/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/pmc_write.log"; exit $rc; }

timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/pmc_sq" -o run -- \
  python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline $BARGS > "$OUT/pmc_sq.log" 2>&1
rc=$?; echo "pmc sq rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/pmc_sq.log"; exit $rc; }
find "$OUT" -name "*.csv" | head -20
exit 0
