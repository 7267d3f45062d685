set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/phase
export PYTHONDONTWRITEBYTECODE=1
for cfg in "MoveToRegion-Demo-LoRes4E-v0 4096" "MoveToCorner-Demo-LoRes4E-v0 4096" "ClusterColour-Demo-LoResStack-v0 8192" "MatchRegions-TestAll-LoRes4E-v0 8192"; do
  set -- $cfg
  timeout -k 10 180 python tools/gpu_phase.py $1 $2 10 > gpurun_out/phase/$1.log 2>&1 || { echo "fail $1"; tail -5 gpurun_out/phase/$1.log; exit 1; }
  echo "== $1"; cat gpurun_out/phase/$1.log
done
bash tools/gpu_skip.sh
