#!/bin/bash
# round 4: emulated 8-rank exchange (MoveToRegion, ClusterColour), then phase profiles (profiling build) of the four BASELINE configs.
# gpurun -- 'bash tools/gpu_r04_prof.sh <tag>'
set -u
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 300 python bench.py --env $env --envs $n --steps 30 --warmup 10 --no-cpu-baseline --emulate-world 8 > "$OUT/emul8.$env.log" 2>&1 || { echo "emul FAIL"; tail -5 "$OUT/emul8.$env.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/emul8.$env.log').read().strip().splitlines()[-1]); print('emul8 $env', d['ms_per_step'], d['kernel_ms_per_step'], d['gather']['restack_ms_per_step'])"
done
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 MoveToCorner-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 200 python tools/gpu_phase.py $env $n 10 > "$OUT/phase.$env.log" 2>&1 || { echo "phase FAIL $env"; tail -5 "$OUT/phase.$env.log"; exit 1; }
  echo "== $env"; cat "$OUT/phase.$env.log"
done
