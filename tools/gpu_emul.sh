#!/bin/bash
# the 8-rank receive side on one GPU (bench.py --emulate-world W) for the C2 and C4 configs, plus 1-GPU lines
# gpurun -- 'bash tools/gpu_emul.sh <tag> [W] [extra bench args]'
set -u
TAG=${1:-emul}; W=${2:-8}; shift 2; EXTRA="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096" "ClusterColour-Demo-LoResStack-v0 8192"; do
  set -- $spec
  timeout -k 10 300 python bench.py --env $1 --envs $2 --steps 60 --warmup 8 --no-cpu-baseline --emulate-world $W $EXTRA > "$OUT/emul$W.$1.log" 2>&1
  rc=$?; echo "emul $1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/emul$W.$1.log"; exit $rc; }
  tail -1 "$OUT/emul$W.$1.log" > "$OUT/emul$W.$1.json"
  python -c "import json; d=json.load(open('$OUT/emul$W.$1.json')); g=d['gather']; print('$1', d['value'], d['ms_per_step'], d['config']['pipeline_chunks'], g['restack'], g['restack_ms_per_step'], g['exchange_ms_per_step'], round(g['restack_bytes_per_rank_step']/1e9,2), d['kernel_ms_per_step'])"
done
exit 0
