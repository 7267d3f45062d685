# step-kernel diagnostics: envs-per-workgroup sweep and SQ counters (MoveToRegion 4096)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/physq
export PYTHONDONTWRITEBYTECODE=1
for b in 16 8 4 2 1; do
  MG_STEP_BLK=$b timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/physq/blk$b.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/physq/blk$b.log').read().strip().splitlines()[-1]); print('blk $b', d['kernel_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM -d "$R/gpurun_out/physq/pmc1" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/physq/pmc1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d "$R/gpurun_out/physq/pmc2" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/physq/pmc2.log" 2>&1 || exit 1
echo done
