#!/bin/bash
# attribution by elimination (profiling build): render kernel time with phases skipped
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for m in 0 16 1 8 2 4 15; do
  MG_DEBUG_SKIP=$m MAGICAL_AMD_PROFILE=1 timeout -k 10 120 python tools/bench_prof.py > gpurun_out/skip_$m.log 2>&1 || exit 1
  echo "skip=$m $(tail -1 gpurun_out/skip_$m.log)"
done
