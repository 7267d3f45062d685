"""Throughput benchmark: env-steps/s of the batched MAGICAL hot path on MI355X.

python bench.py --gpus N --steps K --warmup W [--envs 4096] [--env MoveToRegion-Demo-LoRes4E-v0]

One env-step = one step() of every env: action decode, 10 physics substeps
(Chipmunk-7 semantics), episode bookkeeping + score, the in-place reset of the
envs whose episode ended, allocentric + egocentric 384^2 render, 96^2 area
downsample and LoRes4E frame stack.  Episode phases are staggered (env i starts
at episode step i mod max_episode_steps; --no-phase-spread starts them in
phase), so every timed step resets ~N / max_episode_steps envs, as a steady
training stream does.  Actions come from device Philox (key 42, counter =
(step, env)).  Multi-GPU: one process per GPU, envs sharded contiguously
(global env id = rank * envs + i, seed 1000 + id), no data-path collective
(instances are independent) -> weak scaling; the timed region is bracketed by
barrier + synchronize and the max over ranks is reported.  --gather adds the north
star's exchange: each step's results (obs, reward, done, eval_score) of every rank
all-gathered to every rank as one packed buffer over RCCL, on its own stream,
overlapping the next step (magical_amd.dist).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "magical-1_amd"), os.path.join(ROOT, "oracle")]

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s peak


def obs_bytes(preproc):
    return {"LoRes4E": 165888, "LoRes4A": 165888, "LoRes3EA": 165888, "LoResCHW4E": 165888, "LoResCHW4A": 165888,
            "LoResStack": 221184}.get(preproc, 2 * 384 * 384 * 3)


def _cpu_worker(args):
    """CPU oracle (test infrastructure restatement) on one core: env-steps in wall seconds."""
    name, steps, seed = args
    import numpy as np
    import pyoracle as po
    from magical_amd import registry
    spec = registry.lookup(name)
    env = po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=seed)
    acts = np.random.RandomState(seed).randint(0, 18, steps)
    env.reset()
    t0 = time.perf_counter()
    for a in acts:
        _, _, d, _ = env.step(int(a))
        if d:
            env.reset()
    return steps, time.perf_counter() - t0


def _pool_run(name, workers, steps):
    ctx = mp.get_context("fork")  # before any GPU initialisation in this process
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(name, steps, 1000 + i) for i in range(workers)])
    wall = time.perf_counter() - t0
    return sum(r[0] for r in res) / wall, sum(r[0] / r[1] for r in res) / workers, wall


def cpu_baseline(name, workers, steps):
    """The C oracle restatement (1 env per process, resets included) on 1 core and on `workers`
    cores of this host.  On the GPU box `workers` is the job's CPU share (16 of the host's CPUs);
    the whole-host figure is the per-core rate times the host's CPU count, labelled as scaled."""
    one, _, wall1 = _pool_run(name, 1, 2 * steps)
    many, per_core, wall = _pool_run(name, workers, steps)
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu_model)
    except OSError:
        pass
    host = os.cpu_count() or workers
    return {"value": round(many, 1), "unit": "env-steps/s", "cores": workers, "kind": "port",
            "cpu_model": cpu_model, "host_cpus": host,
            "sample": f"C oracle restatement of {name}, 1 env per process incl. resets: 1 process x {2 * steps} "
                      f"steps (wall {wall1:.1f}s), then {workers} processes x {steps} steps (wall {wall:.1f}s)",
            "one_core_env_steps_s": round(one, 1),
            "per_core_env_steps_s": round(per_core, 1),
            "host_scaled_env_steps_s": round(per_core * host, 1),
            "host_scaled_note": f"per-core rate x {host} host CPUs (linear scaling assumed, not measured: "
                                f"the job may use {workers} of them)"}


def load_pmc(kernel, workload, envs):
    """PMC record of `kernel` (HBM bytes per launch, VALU issue fraction) from the committed passes, newest
    first: profiles/r02_final/<workload>.traffic.json (tools/gpu_table.sh at the round's final build), then
    profiles/r02_table/, then profiles/pmc_traffic.json -- only when collected on this workload and env count."""
    for path in (os.path.join(ROOT, "profiles", "r02_final", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "r02_table", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "pmc_traffic.json")):
        if not os.path.exists(path):
            continue
        with open(path) as f:
            rec = json.load(f).get(kernel)
        if rec and rec.get("workload") == workload and rec.get("envs") == envs:
            return rec
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=4096, help="env instances per GPU")
    ap.add_argument("--env", default="MoveToRegion-Demo-LoRes4E-v0")
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--cpu-steps", type=int, default=1500)  # ~16 x 1 s of CPU work (about 15-25 s)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="N > 1: all-gather every step's packed results (obs, reward, done, score) to every rank "
                         "(the north star's exchange; magical_amd.dist.ShardedVecEnv), pipelined with the next step")
    ap.add_argument("--no-phase-spread", action="store_true",
                    help="start every env at episode step 0 (resets then happen on the same step for all envs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
        cpu = cpu_baseline(args.env, workers, args.cpu_steps)

    import torch
    import torch.distributed as dist
    import magical_amd
    from magical_amd import native, registry

    spec = registry.lookup(args.env)
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    n = args.envs
    seeds = [1000 + rank * n + i for i in range(n)]
    gather = args.gather and world > 1
    if gather:
        from magical_amd import dist as mdist
        shard = mdist.ShardedVecEnv(args.env, n, rank=rank, device=str(device), gather=True)
        vec = shard.vec
        step = shard.step_async
    else:
        vec = magical_amd.make_vec(args.env, n, device=str(device), seeds=seeds)
        step = vec.step
    lib = vec.lib
    actions = torch.empty(n, dtype=torch.uint8, device=device)
    if gather:
        shard.reset_async()
    else:
        vec.reset()
    phase_spread = not args.no_phase_spread and spec.max_episode_steps > 1
    if phase_spread:  # env i starts at episode step (global id) mod max_episode_steps
        L = spec.max_episode_steps
        vec.set_episode_steps(torch.tensor([(rank * n + i) % L for i in range(n)], dtype=torch.int32))
    for s in range(args.warmup):
        vec.random_actions(s, out=actions)
        step(actions)
    if gather:
        for h in shard.pending:
            if h is not None:
                h.wait()
    torch.cuda.synchronize(device)
    native.check(lib.mg_enable_timing(vec.handle, args.steps))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s in range(args.steps):
        vec.random_actions(args.warmup + s, out=actions)
        step(actions)
    if gather:   # the timed region ends after the last step's gather
        for h in shard.pending:
            if h is not None:
                h.wait()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    import ctypes
    tm = (ctypes.c_double * 4)()
    native.check(lib.mg_read_timing(vec.handle, tm))
    t_step_ms, t_render_ms, n_timed = tm[0] / args.steps, tm[1] / args.steps, int(tm[2])
    t_reset_ms = tm[3] / args.steps
    errors = int((vec.errors() != 0).sum().item())
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([errors], dtype=torch.int64, device=device)
        dist.all_reduce(e)
        errors = int(e.item())
    value = world * n * args.steps / elapsed
    if rank == 0:
        per_env = obs_bytes(spec.preproc) + 2048  # obs bytes + ~2 KB state per env-step
        dom = "render_kernel" if t_render_ms >= t_step_ms else "step_kernel"
        dom_ms = max(t_render_ms, t_step_ms)
        achieved = per_env * n / (dom_ms * 1e-3) / 1e9
        pmc = load_pmc(dom, args.env, n)
        out = {
            "metric": "env-steps/sec (whole node) at N instances/GPU, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device Philox uniform actions over the 18 discrete actions; env i seeded 1000+i)",
            "config": {"workload": args.env, "envs_per_gpu": n, "episode_steps": spec.max_episode_steps,
                       "physics_substeps": 10, "solver_iterations": 10, "render": "2 x 384^2 -> 96^2",
                       "phase_spread": phase_spread,
                       "parallelism": (f"dp{world} (envs sharded; one packed all-gather of every step's results, "
                                       f"pipelined with the next step)" if gather else
                                       f"dp{world} (envs sharded, no data-path collective)")},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": pmc and pmc["bytes_per_launch"], "bytes_per_env_step": per_env,
                         "units_per_launch": n, "kernel_avg_ms": round(dom_ms, 4),
                         # the binding resource is VALU issue, not HBM: SQ_INSTS_VALU x 2 cycles over
                         # 1024 SIMDs x GRBM_GUI_ACTIVE / 8 of the committed SQ pass (profiles/)
                         "valu_issue_frac": pmc and pmc.get("valu_issue_frac"),
                         "wait_any_frac": pmc and pmc.get("wait_any_frac")},
            "kernel_ms_per_step": {"step_kernel": round(t_step_ms, 4), "reset_kernel": round(t_reset_ms, 4),
                                   "render_kernel": round(t_render_ms, 4), "timed_launches": n_timed},
            "env_errors": errors,
            "gather": ({"bytes_per_rank_step": shard.layout.nbytes, "ranks": world,
                        "received_bytes_per_rank_step": (world - 1) * shard.layout.nbytes} if gather else None),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    (shard if gather else vec).close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
