#!/bin/bash
# round 4: pipelined env pool (magical_amd.pipeline) -- parity, bench lines chunked / unchunked, kernel trace
# of the default bench line with its overlap summary.
# gpurun -- 'bash tools/gpu_r04_pipe.sh <tag>'
set -u
TAG=${1:-pipe}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "pipelined_pool or packed_gather or restack" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for env in MoveToRegion-Demo-LoRes4E-v0 MoveToCorner-Demo-LoRes4E-v0; do
  for c in auto 1; do
    timeout -k 10 200 python bench.py --env $env --steps 100 --warmup 10 --no-cpu-baseline --chunks $c > "$OUT/bench.$env.$c.log" 2>&1 || { echo "bench FAIL $env $c"; tail -5 "$OUT/bench.$env.$c.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench.$env.$c.log').read().strip().splitlines()[-1]); print('$env chunks $c', round(d['value']), d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
  done
done
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke FAIL"; tail -5 "$OUT/smoke.log"; exit 1; }
echo smoke ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python "$R/bench.py" --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { echo "trace FAIL"; tail -5 "$OUT/trace.log"; exit 1; }
cd "$R"; python tools/overlap_trace.py "$OUT/trace" | tee "$OUT/trace_summary.txt" || exit 1
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/trace"
for spec in "MoveToRegion-Demo-LoRes4E-v0 4096 1" "MoveToRegion-Demo-LoRes4E-v0 4096 0" "ClusterColour-Demo-LoResStack-v0 8192 1"; do
  set -- $spec
  MG_RESTACK_LDS=$3 timeout -k 10 300 python bench.py --env $1 --envs $2 --steps 30 --warmup 10 --no-cpu-baseline --emulate-world 8 > "$OUT/emul8.$1.$3.log" 2>&1 || { echo "emul FAIL"; tail -5 "$OUT/emul8.$1.$3.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/emul8.$1.$3.log').read().strip().splitlines()[-1]); print('emul8 $1 lds=$3', d['ms_per_step'], d['kernel_ms_per_step'], d['gather']['restack_ms_per_step'])"
done
