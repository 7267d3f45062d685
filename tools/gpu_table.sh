#!/bin/bash
# BASELINE.md results table: every BASELINE config on one GPU with its CPU-restatement baseline
# (1 process, then 16 processes = the job's CPU share), a kernel-trace stats pass and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ) of each config, summarised on the box.  Every pass runs the bench line's own
# default (pipelined chunks included): rocprofv3's counter collection counts each dispatch on its own, so the
# PMC bytes are those of the chunked launch the bench times (round 5; earlier rounds ran the PMC passes
# unchunked and scaled them).  (The rocpd databases are dropped: gpurun copies back at most 64 MiB.)
# Output: gpurun_out/<tag>/<config>.{json,log,md,traffic.json}.   usage: bash tools/gpu_table.sh [tag]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-table}; mkdir -p gpurun_out/$TAG
export PYTHONDONTWRITEBYTECODE=1
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096" "MoveToCorner-Demo-LoRes4E-v0 4096" "ClusterColour-Demo-LoResStack-v0 8192" "MatchRegions-TestAll-LoRes4E-v0 8192"; do
  set -- $spec
  T="$R/gpurun_out/$TAG/$1"
  timeout -k 10 400 python bench.py --env $1 --envs $2 --steps 100 --warmup 10 --cpu-steps 600 > $T.log 2>&1 || { echo "FAIL $1"; tail -5 $T.log; exit 1; }
  tail -1 $T.log > $T.json
  python -c "import json; d=json.load(open('$T.json')); print('$1', d['value'], d['ms_per_step'], {k: d['kernels'][k]['ms'] for k in ('step_kernel', 'render_kernel')}, d['roofline']['frac'], d['roofline']['step_frac'], d['cpu_baseline']['one_core_env_steps_s'], d['cpu_baseline']['value'])"
  EPL=$(python -c "import json; print(json.load(open('$T.json'))['kernel_ms_per_step']['envs_per_launch'])")
  cd /tmp && export TMPDIR=/tmp
  B="--env $1 --envs $2 --no-cpu-baseline"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$T.prof/stats" -o run -- python "$R/bench.py" $B --steps 20 --warmup 5 > /dev/null 2>&1 || { echo "FAIL stats $1"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$T.prof/fetch" -o run -- python "$R/bench.py" $B --steps 5 --warmup 2 > /dev/null 2>&1 || { echo "FAIL fetch $1"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$T.prof/write" -o run -- python "$R/bench.py" $B --steps 5 --warmup 2 > /dev/null 2>&1 || { echo "FAIL write $1"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$T.prof/sq" -o run -- python "$R/bench.py" $B --steps 5 --warmup 2 > /dev/null 2>&1 || { echo "FAIL sq $1"; exit 1; }
  cd "$R"
  python tools/prof_summary.py "$T.prof" --md > $T.md || exit 1
  for k in render_kernel step_kernel reset_kernel; do
    python tools/prof_summary.py "$T.prof" --traffic-json $T.traffic.json --kernel $k --workload $1 --envs $2 --envs-per-launch $EPL > /dev/null || exit 1
  done
  rm -rf "$T.prof"
done
echo done
