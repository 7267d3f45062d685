#!/bin/bash
# SQ counter passes for the step / render kernels (each pass its own run).
# gpurun -- 'bash tools/gpu_pmc.sh <tag> [bench args...]'
set -u
TAG=${1:-pmc}
shift 1 2>/dev/null
BARGS="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "rocprofv3 -L rc=$?"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d "$OUT/p$i" -o run -- \
    python "$R/bench.py" --no-cpu-baseline $BARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/p$i.log"; exit $rc; }
done
exit 0
