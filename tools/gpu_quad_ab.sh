R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/quad
export PYTHONDONTWRITEBYTECODE=1
python -c "import torch; p=torch.cuda.get_device_properties(0); print(p)" && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "test_step_kernel_forms and (VARIANT5 or VARIANT6 or VARIANT1 or VARIANT2)" > gpurun_out/quad/parity.log 2>&1 || { tail -30 gpurun_out/quad/parity.log; exit 1; }
tail -3 gpurun_out/quad/parity.log
for rep in 1 2; do
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096:5 MoveToCorner-Demo-LoRes4E-v0:4096:6; do
  IFS=: read env n q <<< "$cfg"
  for v in base $q; do
    log=gpurun_out/quad/$v.$env.$rep.log
    if [ $v = base ]; then unset MG_STEP_VARIANT; else export MG_STEP_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --env $env --envs $n --steps 60 --warmup 10 --no-cpu-baseline > $log 2>&1 || { echo "FAIL $v $env"; tail -5 $log; exit 1; }
    python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$rep $v $env', round(d['value']), 'step', k['step_kernel'], 'render', k['render_kernel'], 'err', d['env_errors'])"
  done
done
done
