#!/bin/bash
# BASELINE.md results table: every BASELINE config on one GPU with its CPU-restatement baseline
# (1 process, then 16 processes = the job's CPU share), plus the render-kernel PMC traffic / SQ pass of
# each config.  Output: gpurun_out/table/<config>.json + pmc dirs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/table
export PYTHONDONTWRITEBYTECODE=1
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096" "MoveToCorner-Demo-LoRes4E-v0 4096" "ClusterColour-Demo-LoResStack-v0 8192" "MatchRegions-TestAll-LoRes4E-v0 8192"; do
  set -- $spec
  timeout -k 10 400 python bench.py --env $1 --envs $2 --steps 100 --warmup 10 --cpu-steps 600 > gpurun_out/table/$1.log 2>&1 || { echo "FAIL $1"; tail -5 gpurun_out/table/$1.log; exit 1; }
  tail -1 gpurun_out/table/$1.log > gpurun_out/table/$1.json
  python -c "import json; d=json.load(open('gpurun_out/table/$1.json')); print('$1', d['value'], d['kernel_ms_per_step'], d['cpu_baseline']['one_core_env_steps_s'], d['cpu_baseline']['value'])"
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/table/$1.fetch" -o run -- python "$R/bench.py" --env $1 --envs $2 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/table/$1.write" -o run -- python "$R/bench.py" --env $1 --envs $2 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$R/gpurun_out/table/$1.sq" -o run -- python "$R/bench.py" --env $1 --envs $2 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  cd "$R"
done
echo done
