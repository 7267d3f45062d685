#!/bin/bash
# round 4: full GPU parity suite, then bench lines of the four BASELINE configs, then the emulated 8-rank
# receive side with restack grid caps.  gpurun -- 'bash tools/gpu_r04_check.sh <tag> [skip_tests]'
set -u
TAG=${1:-check}; SKIP=${2:-0}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
run() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { tail -30 "$OUT/$name.log"; exit $rc; }
}
line() { python3 -c "import json; d=json.loads(open('$OUT/$1.log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; g=d.get('gather') or {}; print('$1', round(d['value']), d['ms_per_step'], 'step', k['step_kernel'], 'reset', k['reset_kernel'], 'render', k['render_kernel'], 'restack', g.get('restack_ms_per_step'), g.get('emulated_copy'))"; }
if [ "$SKIP" != 1 ]; then
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
if [ -x tools/ubench/exec_f64 ]; then
  timeout -k 10 60 ./tools/ubench/exec_f64 256 > "$OUT/ubench_exec.log" 2>&1 && cat "$OUT/ubench_exec.log"
fi
if [ -f magical-1_amd/magical_amd/libmagical_sim_packed.so ]; then   # A/B: packed quad lane layout
  MAGICAL_AMD_EXP_LIB=packed run pytest_packed 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "step_kernel_forms and (MoveTo)" --timeout 120 --timeout-method thread
  for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
    MAGICAL_AMD_EXP_LIB=packed run packed.$env 300 python bench.py --env $env --envs 4096 --steps 60 --warmup 10 --no-cpu-baseline && line packed.$env
  done
fi
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 MoveToCorner-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  run bench.$env 300 python bench.py --env $env --envs $n --steps 60 --warmup 10 --no-cpu-baseline && line bench.$env
done
for cap in 0; do
  MG_RESTACK_WGS=$cap run emul8.cap$cap 300 python bench.py --envs 4096 --steps 40 --warmup 10 --no-cpu-baseline --emulate-world 8 && line emul8.cap$cap
done
