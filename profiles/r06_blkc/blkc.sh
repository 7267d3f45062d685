set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r06_blkc; export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for E in MoveToCorner-Demo-LoRes4E-v0 MoveToRegion-Demo-LoRes4E-v0; do
for B in 8 16; do for C in 2 3; do
  L=gpurun_out/r06_blkc/$E.b$B.c$C.$rep.log
  MG_STEP_BLK=$B timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --env $E --envs 4096 --chunks $C > $L 2>&1 || { echo fail $E $B $C; tail -3 $L; exit 1; }
  tail -1 $L | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$E', 'blk$B', 'c$C', $rep, d['value'], d['ms_per_step'], d['config']['step_form'], {k: d['kernels'][k]['ms'] for k in ('step_kernel', 'render_kernel')})"
done; done; done; done
