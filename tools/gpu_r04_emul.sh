#!/bin/bash
# round 4: the 8-rank receive side on one GPU (bench.py --emulate-world 8) for MoveToRegion 4096 and
# ClusterColour 8192, each beside its plain 1-GPU line, with a kernel trace of the emulated runs (restack
# overlapping step/render); then a PC-sampling pass of the MoveToRegion step kernel.
# gpurun -- 'bash tools/gpu_r04_emul.sh <tag>'
set -u
TAG=${1:-emul}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
run() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
cd /tmp && export TMPDIR=/tmp && cd "$R"
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  run plain.$env 300 python bench.py --env $env --envs $n --steps 40 --warmup 10 --no-cpu-baseline
  run emul8.$env 300 python bench.py --env $env --envs $n --steps 40 --warmup 10 --no-cpu-baseline --emulate-world 8
  run trace.$env 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$env" -o trace -- python3 bench.py --env $env --envs $n --steps 20 --warmup 5 --no-cpu-baseline --emulate-world 8
done
run pcs 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-include-regex step_kernel -d "$OUT/pcs" -o pcs -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline
ls -R "$OUT/pcs" | head -20
