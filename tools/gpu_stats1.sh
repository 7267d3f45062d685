#!/bin/bash
# one config's bench line plus a rocprofv3 kernel-trace stats pass of the same command, summarised by
# prof_summary.py (isolated dispatches included):  bash tools/gpu_stats1.sh <tag> <env> <envs> [bench args...]
set -u
TAG=$1; ENV=$2; N=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
T="$R/gpurun_out/$TAG/$ENV"; mkdir -p "$R/gpurun_out/$TAG"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python bench.py --env $ENV --envs $N --steps 100 --warmup 10 --no-cpu-baseline "$@" > $T.log 2>&1 || { echo "FAIL bench"; tail -5 $T.log; exit 1; }
tail -1 $T.log > $T.json
python -c "import json; d=json.load(open('$T.json')); k=d['kernels']; print('$ENV', d['value'], d['ms_per_step'], 'iso', {x: k[x]['ms'] for x in ('step_kernel', 'render_kernel', 'reset_kernel')}, 'timed', d['kernel_ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$T.prof/stats" -o run -- python "$R/bench.py" --env $ENV --envs $N --no-cpu-baseline --steps 20 --warmup 5 "$@" > $T.prof.log 2>&1 || { echo "FAIL stats"; tail -5 $T.prof.log; exit 1; }
cd "$R"
python tools/prof_summary.py "$T.prof" --md > $T.md || exit 1
rm -rf "$T.prof"
grep -A14 "isolated dispatches" $T.md
