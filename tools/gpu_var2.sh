# step-kernel form comparison on the many-block configs at 8192 envs
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/var
export PYTHONDONTWRITEBYTECODE=1
for env in ClusterColour-Demo-LoResStack-v0 MatchRegions-TestAll-LoRes4E-v0; do
for v in "4 x" "0 64" "0 32" "3 1"; do
  set -- $v
  if [ $1 = 0 ]; then X="MG_STEP_BLK0=$2"; elif [ $1 = 3 ]; then X="MG_STEP_BLK=$2"; else X=""; fi
  env MG_STEP_VARIANT=$1 $X timeout -k 10 120 python bench.py --env $env --envs 8192 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/var/$env.v$1.$2.log 2>&1 || { tail -3 gpurun_out/var/$env.v$1.$2.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/var/$env.v$1.$2.log').read().strip().splitlines()[-1]); print('$env var $1 blk $2', d['kernel_ms_per_step'], d['env_errors'])"
done; done
