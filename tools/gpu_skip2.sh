#!/bin/bash
# render kernel time under the profiling build's debug skips (1 outlines, 2 fill, 4 HBM stores, 8 spans, 16 setup only)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/skip
export PYTHONDONTWRITEBYTECODE=1 MAGICAL_AMD_PROFILE=1
for sk in ${SKIPS:-0 16 1 2 4 8 15}; do
  MG_DEBUG_SKIP=$sk timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/skip/s$sk.log 2>&1 || { echo "FAIL $sk"; tail -3 gpurun_out/skip/s$sk.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/skip/s$sk.log').read().strip().splitlines()[-1]); print('skip $sk', d['kernel_ms_per_step'])"
done
