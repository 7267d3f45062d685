#!/bin/bash
# PMC passes with caller-chosen counter sets (one rocprofv3 run per set):
# gpurun -- 'bash tools/gpu_pmc_sets.sh <tag> "<set1>" "<set2>" ...'   (bench: 3 steps, 1 warmup)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/p$i" -o run -- \
    python "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/p$i.log"; exit $rc; }
done
exit 0
