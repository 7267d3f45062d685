#!/bin/bash
# A/B of in-tree library variants on bench lines: gpurun -- 'bash tools/gpu_libab.sh <tag> "<variants>" <env> [env ...]'
# variants: space-separated MAGICAL_AMD_EXP_LIB tags ("-" = the product library), or "-:<bench args>" / "<tag>:<bench
# args>" (e.g. "-:--stacks=materialize"); each bench line runs 100 steps
set -u
TAG=$1; VARS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for ENV in "$@"; do
  N=4096; case $ENV in Cluster*|MatchRegions*) N=8192;; esac
  for VA in $VARS; do
    V=${VA%%:*}; A=""; [ "$V" != "$VA" ] && A=${VA#*:}
    if [ "$V" = "-" ]; then unset MAGICAL_AMD_EXP_LIB; else export MAGICAL_AMD_EXP_LIB=$V; fi
    L="$OUT/bench.$ENV.${VA//[^A-Za-z0-9_.-]/_}.$rep.log"
    timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env "$ENV" --envs $N $A > "$L" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $ENV $VA rc=$rc"; tail -3 "$L"; exit $rc; }
    tail -1 "$L" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ENV', '$VA', $rep, d['value'], d['ms_per_step'], {k: d['kernels'][k]['ms'] for k in ('step_kernel', 'render_kernel')}, d['kernel_ms_per_step'])"
  done
done
done
unset MAGICAL_AMD_EXP_LIB
exit 0
