R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/r03_start
export PYTHONDONTWRITEBYTECODE=1
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096" "MoveToCorner-Demo-LoRes4E-v0 4096" "ClusterColour-Demo-LoResStack-v0 8192" "MatchRegions-TestAll-LoRes4E-v0 8192"; do
  set -- $spec
  timeout -k 10 200 python bench.py --env $1 --envs $2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r03_start/$1.log 2>&1 || { echo FAIL $1; tail -5 gpurun_out/r03_start/$1.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03_start/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['kernel_ms_per_step'])"
done
