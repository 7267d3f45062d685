#!/bin/bash
# Step-kernel counters (issue mix, waits, instruction fetch) for one config, one PMC pass per group.
# gpurun -- 'bash tools/pmc_step.sh <tag> [env] [envs] "<counters pass 1>" "<counters pass 2>" ...'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
TAG=$1; ENV=$2; N=$3; shift 3
T="$R/gpurun_out/$TAG"; mkdir -p "$T"
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "$@"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d "$T/prof/p$i" -o run -- python3 "$R/bench.py" --env $ENV --envs $N --no-cpu-baseline --steps 5 --warmup 2 > "$T/p$i.log" 2>&1 || { echo "FAIL pass $i: $pass"; tail -5 "$T/p$i.log"; exit 1; }
done
cd "$R" && python tools/prof_summary.py "$T/prof" --md > "$T/pmc.md" && rm -rf "$T/prof" && grep -E "step_kernel|render_kernel" "$T/pmc.md"
