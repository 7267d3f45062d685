cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in "" "MG_DEBUG_WIN=1" "MG_DEBUG_WIN=2"; do
  env $v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env MoveToRegion-Demo-LoRes4E-v0 > gpurun_out/wexp.log 2>&1 || exit 1
  tail -1 gpurun_out/wexp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['kernels']['render_kernel']['ms'], d['kernels']['step_kernel']['ms'])"
done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env MoveToRegion-Demo-LoRes4E-v0 --stacks materialize > gpurun_out/wexp.log 2>&1 || exit 1
tail -1 gpurun_out/wexp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('materialize', d['value'], d['kernels']['render_kernel']['ms'], d['kernels']['step_kernel']['ms'])"
done
