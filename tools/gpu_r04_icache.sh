#!/bin/bash
# round 4: parity of the step-kernel forms, bench lines of the robot scenes, the emulated 8-rank exchange
# (MoveToRegion, ClusterColour), then instruction-fetch counters of the step kernel (MoveToRegion,
# ClusterColour): which SQ/SQC counters exist is read from `rocprofv3 -L` first.
# gpurun -- 'bash tools/gpu_r04_icache.sh <tag>'
set -u
TAG=${1:-icache}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "step_kernel_forms or parity" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 MoveToCorner-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192 MatchRegions-TestAll-LoRes4E-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 200 python bench.py --env $env --envs $n --steps 60 --warmup 10 --no-cpu-baseline > "$OUT/bench.$env.log" 2>&1 || { echo "bench FAIL $env"; tail -5 "$OUT/bench.$env.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench.$env.log').read().strip().splitlines()[-1]); print('$env', round(d['value']), d['kernel_ms_per_step'])"
done
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 300 python bench.py --env $env --envs $n --steps 30 --warmup 10 --no-cpu-baseline --emulate-world 8 > "$OUT/emul8.$env.log" 2>&1 || { echo "emul FAIL"; tail -5 "$OUT/emul8.$env.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/emul8.$env.log').read().strip().splitlines()[-1]); print('emul8 $env', d['ms_per_step'], d['kernel_ms_per_step'], d['gather']['restack_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || { echo "list FAIL"; exit 1; }
pick() { local o=""; for c in "$@"; do grep -qw "$c" "$OUT/counters.txt" && o="$o $c"; done; echo $o; }
A=$(pick SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES)
B=$(pick SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE)
C=$(pick SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_LEVEL_SMEM)
echo "pass A: $A"; echo "pass B: $B"; echo "pass C: $C"
for cfg in MoveToRegion-Demo-LoRes4E-v0:4096 ClusterColour-Demo-LoResStack-v0:8192; do
  env=${cfg%%:*}; n=${cfg##*:}
  P="$OUT/prof.$env"
  for pass in A B C; do
    cs=${!pass}; [ -n "$cs" ] || continue
    timeout -s KILL 90 rocprofv3 --pmc $cs -d "$P/$pass" -o run -- python "$R/bench.py" --env $env --envs $n --no-cpu-baseline --steps 5 --warmup 2 > "$P.$pass.log" 2>&1 || { echo "pmc $pass FAIL $env"; tail -5 "$P.$pass.log"; exit 1; }
  done
  cd "$R"; python tools/prof_summary.py "$P" --md > "$OUT/pmc.$env.md" || exit 1
  grep -E "step_kernel|render_kernel" "$OUT/pmc.$env.md"; rm -rf "$P"; cd /tmp
done
echo done
