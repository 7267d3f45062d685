#!/bin/bash
# A/B of in-tree library variants on bench lines: gpurun -- 'bash tools/gpu_libab.sh <tag> "<variants>" <env> [env ...]'
# variants: space-separated MAGICAL_AMD_EXP_LIB tags ("-" = the product library); each bench line runs 100 steps
set -u
TAG=$1; VARS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for ENV in "$@"; do
  N=4096; case $ENV in Cluster*|MatchRegions*) N=8192;; esac
  for V in $VARS; do
    if [ "$V" = "-" ]; then unset MAGICAL_AMD_EXP_LIB; else export MAGICAL_AMD_EXP_LIB=$V; fi
    timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env "$ENV" --envs $N > "$OUT/bench.$ENV.$V.$rep.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $ENV $V rc=$rc"; tail -3 "$OUT/bench.$ENV.$V.$rep.log"; exit $rc; }
    tail -1 "$OUT/bench.$ENV.$V.$rep.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ENV', '$V', $rep, d['value'], d['ms_per_step'], {k: d['kernels'][k]['ms'] for k in ('step_kernel', 'render_kernel')})"
  done
done
done
unset MAGICAL_AMD_EXP_LIB
exit 0
