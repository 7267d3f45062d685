# physics/render phase profiles (profiling build) of two configs
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/phase
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 180 python tools/gpu_phase.py MoveToRegion-Demo-LoRes4E-v0 4096 10 > gpurun_out/phase/mtr.log 2>&1 || exit 1
timeout -k 10 180 python tools/gpu_phase.py MatchRegions-TestAll-LoRes4E-v0 8192 10 > gpurun_out/phase/mr.log 2>&1 || exit 1
grep -A9 physics gpurun_out/phase/mtr.log; grep -A9 physics gpurun_out/phase/mr.log
