# render scene-size statistics of the many-block configs (profiling build, every (env, view) through the
# large class): bash tools/gpu_sizes.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/phase
export PYTHONDONTWRITEBYTECODE=1
for cfg in "ClusterColour-Demo-LoResStack-v0 8192" "MatchRegions-TestAll-LoRes4E-v0 8192" "ClusterColour-TestAll-LoResStack-v0 8192" "FindDupe-TestAll-LoRes4E-v0 4096" "MakeLine-TestAll-LoRes4E-v0 4096"; do
  set -- $cfg
  MG_DEBUG_RENDER_RETRY=2 timeout -k 10 180 python tools/gpu_phase.py $1 $2 10 > gpurun_out/phase/sizes_$1.log 2>&1 || { echo "fail $1"; tail -5 gpurun_out/phase/sizes_$1.log; exit 1; }
  echo "== $1"; grep "scene sizes" gpurun_out/phase/sizes_$1.log
done
