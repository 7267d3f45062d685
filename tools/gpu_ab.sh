#!/bin/bash
# A/B of library variants (tools/build_variants.sh): bench lines per variant and config, interleaved twice
# gpurun -- 'bash tools/gpu_ab.sh "base nodash ..." "MoveToRegion-Demo-LoRes4E-v0:4096 ..."'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/ab
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for cfg in $2; do
  env=${cfg%%:*}; n=${cfg##*:}
  for v in $1; do
    log=gpurun_out/ab/$v.$env.$rep.log
    if [ "$v" = base ]; then unset MAGICAL_AMD_EXP_LIB; else export MAGICAL_AMD_EXP_LIB=$v; fi
    timeout -k 10 200 python bench.py --env $env --envs $n --steps 60 --warmup 10 --no-cpu-baseline > $log 2>&1 || { echo "FAIL $v $env"; tail -5 $log; exit 1; }
    python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$rep $v $env', round(d['value']), 'step', k['step_kernel'], 'render', k['render_kernel'])"
  done
done
done
