R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('base', d['kernel_ms_per_step'])"
MAGICAL_AMD_PROFILE=1 timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('exp', d['kernel_ms_per_step'])"
