#!/bin/bash
# mg_restack variants (MG_RESTACK_LDS=0/1/2): restack parity tests under the default, then the emulated 8-rank
# receive side per variant.  gpurun -- 'bash tools/gpu_restack_ab.sh <tag> "2 1"'
set -u
TAG=${1:-restack}; VARS=${2:-"2 1"}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "restack or packed_gather" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  for v in $VARS; do
    log="$OUT/emul8.$env.$v.log"
    MG_RESTACK_LDS=$v timeout -k 10 300 python bench.py --env $env --envs $n --steps 30 --warmup 10 --no-cpu-baseline --emulate-world 8 > "$log" 2>&1 || { echo "emul FAIL"; tail -5 "$log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('emul8 $env lds=$v', d['ms_per_step'], d['kernel_ms_per_step'], d['gather']['restack_ms_per_step'])"
  done
done
