#!/bin/bash
# round 4: physics/render overlap A/B (tools/overlap_ab.py: C simulators of total/C envs on C streams) with a
# kernel trace of the 2-chunk MoveToRegion run, then the results table (tools/gpu_table.sh).
# gpurun -- 'bash tools/gpu_r04_overlap.sh <tag>'
set -u
TAG=${1:-overlap}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096 1 2 4" "MoveToCorner-Demo-LoRes4E-v0 4096 1 2" "ClusterColour-Demo-LoResStack-v0 8192 1 2"; do
  set -- $spec; env=$1; n=$2; shift 2
  timeout -k 10 300 python -u tools/overlap_ab.py $env $n 60 "$@" > "$OUT/ab.$env.log" 2>&1 || { echo "ab FAIL $env"; tail -5 "$OUT/ab.$env.log"; exit 1; }
  cat "$OUT/ab.$env.log"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python "$R/tools/overlap_ab.py" MoveToRegion-Demo-LoRes4E-v0 4096 20 2 > "$OUT/trace.log" 2>&1 || { echo "trace FAIL"; tail -5 "$OUT/trace.log"; exit 1; }
cd "$R"; python tools/overlap_trace.py "$OUT/trace" | tee "$OUT/trace_summary.txt" || exit 1
rm -rf "$OUT/trace"
[ "${SKIP_TABLE:-0}" = 1 ] || bash tools/gpu_table.sh
