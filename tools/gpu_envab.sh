#!/bin/bash
# A/B of environment-variable settings on bench lines:
#   gpurun -- 'bash tools/gpu_envab.sh <tag> "<settings>" <env> [env ...]'
# settings: space-separated VAR=value[,VAR=value...] lists ("-" = none); each bench line runs 100 steps, twice
set -u
TAG=$1; SETS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for ENV in "$@"; do
  N=4096; case $ENV in Cluster*|MatchRegions*) N=8192;; esac
  for SET in $SETS; do
    L="$OUT/bench.$ENV.${SET//[^A-Za-z0-9_.-]/_}.$rep.log"
    if [ "$SET" = "-" ]; then EV=(); else IFS=, read -ra EV <<< "$SET"; fi
    timeout -k 10 300 env "${EV[@]}" python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env "$ENV" --envs $N > "$L" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $ENV $SET rc=$rc"; tail -3 "$L"; exit $rc; }
    tail -1 "$L" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ENV', '$SET', $rep, d['value'], d['ms_per_step'], {k: d['kernels'][k]['ms'] for k in ('step_kernel', 'render_kernel')})"
  done
done
done
exit 0
