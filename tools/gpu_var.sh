# step-kernel form comparison on MoveToRegion / MoveToCorner 4096
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/var
export PYTHONDONTWRITEBYTECODE=1
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
for v in 1 4 3; do
  MG_STEP_VARIANT=$v timeout -k 10 120 python bench.py --env $env --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/var/$env.v$v.log 2>&1 || { tail -3 gpurun_out/var/$env.v$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/var/$env.v$v.log').read().strip().splitlines()[-1]); print('$env var $v', d['kernel_ms_per_step'], d['env_errors'])"
done; done
