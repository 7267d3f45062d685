#!/bin/bash
# full GPU test suite, then an A/B of library variants (tools/gpu_ab.sh arguments)
# gpurun -- 'bash tools/gpu_suite_ab.sh "base v1 ..." "Env:N ..."'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -30 gpurun_out/suite.log; exit 1; }
tail -2 gpurun_out/suite.log
[ -n "$1" ] && bash tools/gpu_ab.sh "$1" "$2"
