#!/bin/bash
# round 4: FP64 exec-mask micro-benchmark, then phase profiles (profiling build) of the four BASELINE configs.
# gpurun -- 'bash tools/gpu_r04_prof.sh <tag>'
set -u
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for b in 256 1024; do
  timeout -k 10 60 ./tools/ubench/exec_f64 $b > "$OUT/ubench_exec.$b.log" 2>&1 || { echo "ubench FAIL"; cat "$OUT/ubench_exec.$b.log"; exit 1; }
  cat "$OUT/ubench_exec.$b.log"
done
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 MoveToCorner-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 200 python tools/gpu_phase.py $env $n 10 > "$OUT/phase.$env.log" 2>&1 || { echo "phase FAIL $env"; tail -5 "$OUT/phase.$env.log"; exit 1; }
  echo "== $env"; cat "$OUT/phase.$env.log"
done
