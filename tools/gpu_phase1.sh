# phase profile of one config (profiling build): bash tools/gpu_phase1.sh <env> <envs>
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/phase
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 180 python tools/gpu_phase.py ${1:-MoveToRegion-Demo-LoRes4E-v0} ${2:-4096} 10 > gpurun_out/phase/one.log 2>&1
rc=$?; cat gpurun_out/phase/one.log; exit $rc
