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
barrier + synchronize and the max over ranks is reported.  `--gpus N` with N > 1
(and no WORLD_SIZE in the environment) launches the N ranks itself through
torch.distributed.run, before anything touches a GPU.  For N > 1 the north star's
exchange is on by default (--no-gather turns it off): each step's results of every
rank reach every rank through one packed RCCL all-gather on a side stream,
overlapping the next step; by default only the current LoRes frames plus
reward/done/eval_score are gathered and every receiver rebuilds the frame stacks
(mg_restack), --gather-mode stacked gathers the whole observations
(magical_amd.dist).  --dry-run checks the launcher and the process group (gloo, no
GPU): rank 0 prints {"ranks_seen": N}.
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "magical-1_amd"), os.path.join(ROOT, "oracle")]

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s peak


FR = 96 * 96 * 3            # one LoRes RGB frame
STATE_BYTES = 2048          # per-env state read + written once per env-step (~2 KB)


def survey_bytes(preproc):
    """SURVEY.md 8(d) algorithmic bytes of one env-step: the observation outputs + ~2 KB of state
    (LoRes4E family 167 936 B, LoResStack 223 232 B).  roofline.frac uses these for every kernel."""
    return obs_bytes(preproc) + STATE_BYTES


def kernel_survey_bytes(kernel, preproc):
    """The share of survey_bytes a kernel is charged in roofline.traffic_ratio: the render kernel writes the
    observations (+ the nominal state, as 8(d) counts the env-step), the step kernel reads + writes the state."""
    return survey_bytes(preproc) if kernel == "render_kernel" else STATE_BYTES


AC_NUM = 10                 # contact fields per arbiter contact (csrc/mg_state.h)


def step_state_bytes(form, caps, live_arbiters):
    """Bytes per env-step the step kernel's HBM state transfer moves by its design (csrc/mg_stepk.h): the
    substeps run on an LDS copy of the env's state, loaded once (xfer_state_quad, or the cooperative form's
    xfer_state, `in`) and written back once (xfer_state `out`), every [slot][N] row up to the form's slot caps
    (bodies nb, shapes ns, constraints nc, arbiter slots na); arbiter slots carry contact data only while live.
      in:  bodies 12 x nb f64 (p, v, angle, w, bias velocities, rotation cache) + 1/m, 1/I (2 x nb f64);
           constraint slots MAXF..JACC2 and parameters 8-11 (9 x nc f64); arbiter keys (na i32), per live slot
           n, u (3 f64), stamp (u32), state / count / bodies (4 i8), 2 contacts x 10 f64, 2 hashes (u64), its
           active-list entry (i8); nactive, stamp, overflow (3 x 4), curr_dt, target_speed, rel_turn,
           target_finger (4 x f64), nbodies / nshapes / ncons / robot_body0 / robot_cons0 (5 x i32); per shape
           radius, friction (2 f64), group, hashid (2 i16), body, poly (2 i8); the cooperative form also its
           runtime constraint list (3 x nc i8);
      out: bodies 12 x nb f64, warm-start impulses JACC / JACC2 (2 x nc f64), arbiter keys and live slots as
           in, nactive, curr_dt, stamp, overflow;
      io:  action (u8), episode_steps (r/w i32), reward (f32), done (u8), eval_score (f64), reset mask (u8).
    The fused / shadow resets and the library (L2-resident, shared by every env) are not counted."""
    nb, ns, nc, na = caps
    live = float(live_arbiters)
    slot = 3 * 8 + 4 + 4 + 2 * AC_NUM * 8 + 2 * 8 + 1
    arbs = na * 4 + live * slot + 4
    rd = 14 * nb * 8 + 9 * nc * 8 + arbs + 3 * 4 + 4 * 8 + 5 * 4 + ns * (2 * 8 + 2 * 2 + 2) + (3 * nc if form == 4 else 0)
    wr = 12 * nb * 8 + 2 * nc * 8 + arbs + 8 + 4 + 4
    io = 1 + 2 * 4 + 4 + 1 + 8 + 1
    return int(round(rd + wr + io))


def env_overrides():
    """Every MG_* / MAGICAL_AMD_* variable set in this process's environment (they select kernel forms, block
    sizes, reset paths or a library variant at mg_create): recorded on the bench line"""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(("MG_", "MAGICAL_AMD_"))}


def obs_bytes(preproc):
    return {"LoRes4E": 165888, "LoRes4A": 165888, "LoRes3EA": 165888, "LoResCHW4E": 165888, "LoResCHW4A": 165888,
            "LoResStack": 221184}.get(preproc, 2 * 384 * 384 * 3)


def render_bytes(preproc, frames_only=False, window=False, K=8):
    """Bytes the render kernel must move per env-step: the observation outputs, plus the frame ring of
    each stacked view (3 earlier frames read, the current one written; the 4 slots are filled at reset).
    frames_only (compact multi-GPU gather): the two current frames only -- the stacks are rebuilt by
    mg_restack on the receivers.  window (mg_bind_window): each stacked view writes its current frame once
    into its window ring (+ 3 / K for the duplicate slots) instead of stack + ring, plus the plain frames."""
    if frames_only:
        return 2 * FR
    stacked_views = {"LoResStack": 2, "LoRes4E": 1, "LoRes4A": 1, "LoResCHW4E": 1, "LoResCHW4A": 1}.get(preproc, 0)
    if window and stacked_views:
        plain = 0 if preproc == "LoResStack" else 2 * FR
        return int(round(plain + stacked_views * (1 + 3 / K) * FR))
    ring = stacked_views * 4 * FR
    if preproc == "LoRes3EA":   # ego ring (1 write) + compose pass (allo + 3 ring frames read, 4 frames written)
        ring = FR + 4 * FR + 4 * FR
    return obs_bytes(preproc) + ring


def restack_bytes(preproc, window=True, K=8):
    """Receiver-side restack per received env-step and stacked view.  Window ring (mg_restack_window, the
    default except LoRes3EA): the current frame read, written once channel-planar plus, on 3 of every K steps,
    once more (the slots that keep the 4-frame window contiguous): FR + (1 + 3 / K) FR.  Materialised stacks
    (mg_restack): current frame read, 3 ring frames read, 1 ring frame written and the 4-frame stack written
    (LoRes3EA: + the allo frame read)."""
    views = 2 if preproc == "LoResStack" else 1
    if window and preproc != "LoRes3EA":
        return int(round(views * (FR + (1 + 3 / K) * FR)))
    return views * (FR + 3 * FR + FR + 4 * FR) + (FR if preproc == "LoRes3EA" else 0)


def step_fraction(preproc, envs, ms_per_step):
    """roofline.step_frac: SURVEY 8(d) bytes of the env-steps one GPU completes per step over the measured
    ms_per_step, against the 8 TB/s HBM peak -- (achieved GB/s, fraction)."""
    ach = survey_bytes(preproc) * envs / (ms_per_step * 1e-3) / 1e9
    return ach, ach / HBM_PEAK_GBS


def cpu_share():
    """CPUs this job may use: the affinity mask, capped by a cgroup v2 quota when one is set."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


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


def cpu_baseline(name, workers, steps, affinity, quota):
    """The C oracle restatement (1 env per process, resets included) on 1 core and on `workers`
    processes = every CPU this job may use (affinity mask, capped by the cgroup quota), measured.
    The whole-host figure is the per-core rate times the host's CPU count, labelled as scaled."""
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
            "affinity_cpus": affinity, "cgroup_quota_cpus": quota,
            "one_core_env_steps_s": round(one, 1),
            "per_core_env_steps_s": round(per_core, 1),
            "host_scaled_env_steps_s": round(per_core * host, 1),
            "host_scaled_note": f"per-core rate x {host} host CPUs (linear scaling assumed, not measured: "
                                f"the job may use {workers} of them)"}


def load_pmc(kernel, workload, envs, envs_per_launch=None):
    """PMC record of `kernel` (HBM bytes per launch, VALU issue fraction) from the committed passes, newest
    first: profiles/r06_final/<workload>.traffic.json (tools/gpu_table.sh at the round's final build), then
    the earlier rounds' -- only when collected on this workload, env count and envs per launch (records without
    envs_per_launch were collected unchunked: envs per launch = envs)."""
    epl = envs if envs_per_launch is None else envs_per_launch
    for path in (os.path.join(ROOT, "profiles", "r06_final", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "r05_final", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "r04_final", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "r03_final", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "r02_final", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "r02_table", f"{workload}.traffic.json"),
                 os.path.join(ROOT, "profiles", "pmc_traffic.json")):
        if not os.path.exists(path):
            continue
        with open(path) as f:
            rec = json.load(f).get(kernel)
        if rec and rec.get("workload") == workload and rec.get("envs") == envs and \
                abs(rec.get("envs_per_launch", rec.get("envs")) - epl) < 0.5:   # (recorded to 0.1 env)
            return rec
    return None


CPU_ENV = "MAGICAL_BENCH_CPU_BASELINE"   # launcher parent -> rank 0: the measured cpu_baseline object (JSON)


def measure_cpu_baseline(args):
    share, affinity, quota = cpu_share()
    workers = args.cpu_workers or share
    return cpu_baseline(args.env, workers, args.cpu_steps, affinity, quota)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """One process per GPU: re-run this script under torch.distributed.run with n ranks (rendezvous on
    127.0.0.1) and return its exit code.  Called before anything in this process touches a GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1")))


def kernel_record(name, ms, preproc, n, pmc, frames_only=False, window=False, step_bytes=None):
    """One kernel's roofline figures over its average duration (ms per launch, one launch per step):
    * achieved / hbm_frac: SURVEY 8(d) bytes of the env-steps the launch completes (survey_bytes x n);
    * kernel_bytes_*: the bytes this kernel must move by its design (render: obs + the frame ring's reads
      and writes; step: its state transfer, step_state_bytes, when given -- else the 8(d) nominal 2 KB);
    * traffic_ratio: PMC HBM bytes per launch (committed rocprofv3 FETCH/WRITE passes of the same workload
      and env count) over the render kernel's 8(d) share x n (obs + state), the step kernel's design bytes x n."""
    if ms is None or ms <= 0:
        return None
    sb = survey_bytes(preproc)
    ach = sb * n / (ms * 1e-3) / 1e9
    kb = render_bytes(preproc, frames_only, window) if name == "render_kernel" else (step_bytes or STATE_BYTES)
    kach = kb * n / (ms * 1e-3) / 1e9
    traffic = pmc and pmc.get("bytes_per_launch")
    share = kernel_survey_bytes(name, preproc) if name == "render_kernel" else kb
    return {"ms": round(ms, 4), "bytes_per_env_step": sb, "achieved_gbs": round(ach, 2),
            "hbm_frac": round(ach / HBM_PEAK_GBS, 5),
            "traffic_bytes_per_launch": traffic,
            "traffic_ratio": round(traffic / (share * n), 2) if traffic else None,
            "traffic_ratio_basis_bytes_per_env_step": share,
            "kernel_bytes_per_env_step": kb, "kernel_bytes_achieved_gbs": round(kach, 2),
            "kernel_bytes_hbm_frac": round(kach / HBM_PEAK_GBS, 5),
            "valu_issue_frac": pmc and pmc.get("valu_issue_frac"), "wait_any_frac": pmc and pmc.get("wait_any_frac")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=4096, help="env instances per GPU")
    ap.add_argument("--env", default="MoveToRegion-Demo-LoRes4E-v0")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: every CPU this job may use")
    ap.add_argument("--cpu-steps", type=int, default=1500)  # ~1-2 s of CPU work per process
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", dest="gather", action="store_true", default=None,
                    help="all-gather every step's results to every rank (default for N > 1)")
    ap.add_argument("--no-gather", dest="gather", action="store_false")
    ap.add_argument("--gather-mode", default="frames", choices=("frames", "stacked"),
                    help="frames: current frames + scalars, stacks rebuilt on each receiver; stacked: whole obs")
    ap.add_argument("--no-phase-spread", action="store_true",
                    help="start every env at episode step 0 (resets then happen on the same step for all envs)")
    ap.add_argument("--dry-run", action="store_true", help="launcher / process-group check only (gloo, no GPU)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one GPU runs rank 0 of a W-rank node's exchange: each step's frames-only buffer is copied "
                         "into all W receive blocks (standing in for the all-gather) and restacked for W x envs on "
                         "the restack stream, beside the next step (value stays this rank's env-steps/s x W)")
    ap.add_argument("--chunks", default="auto",
                    help="env chunks pipelined on their own HIP streams (magical_amd.pipeline): an int, or auto = "
                         "2 for the robot scenes (MoveToRegion / MoveToCorner: measured faster), 1 otherwise "
                         "(also under the all-gather: the collective waits for every chunk's stream)")
    ap.add_argument("--iso-steps", type=int, default=20,
                    help="chunked runs: steps of chunk 0 alone after the timed region, for the roofline's isolated "
                         "per-kernel times (0: none)")
    ap.add_argument("--stacks", default="materialize", choices=("window", "materialize"),
                    help="the simulator's frame stacks: materialised [N, 96, 96, 12] tensors (default) or strided "
                         "views of window rings (mg_bind_window; measured slower in the render kernel)")
    ap.add_argument("--restack", default="window", choices=("window", "materialize"),
                    help="frames-mode receivers: window ring views (mg_restack_window) or materialised stacks "
                         "(mg_restack)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the CPU baseline is measured here, in the launcher parent, before any rank (or GPU) exists; rank 0
        # puts it on its line
        if not args.no_cpu_baseline:
            os.environ[CPU_ENV] = json.dumps(measure_cpu_baseline(args))
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:   # an outside launcher decides the world size; --gpus is informational then
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using {world} ranks", file=sys.stderr)

    # rank 0's CPU baseline: from the launcher parent when bench.py launched the ranks, else measured here
    # before this process touches a GPU (an outside torch.distributed.run: the other ranks wait in the
    # process-group rendezvous meanwhile)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = json.loads(os.environ[CPU_ENV]) if os.environ.get(CPU_ENV) else measure_cpu_baseline(args)
        cpu["measured_in"] = "launcher parent" if os.environ.get(CPU_ENV) else "rank 0 before GPU init"

    if args.dry_run:
        import torch
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
        t = torch.ones(1)
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": args.gpus, "ranks_seen": int(t.item()),
                              "gather": args.gather if args.gather is not None else world > 1,
                              "cpu_baseline": cpu}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    import torch
    import torch.distributed as dist
    import magical_amd
    from magical_amd import native, pipeline, registry

    spec = registry.lookup(args.env)
    # rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0 over a gloo group (RCCL refuses two ranks
    # on one device); the variable is recorded in config.env_overrides, and such a line is not a node measurement
    same_gpu = world > 1 and os.environ.get("MAGICAL_AMD_BENCH_SAME_GPU") == "1"
    device = torch.device("cuda", 0 if same_gpu else local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        if same_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
    n = args.envs
    seeds = [1000 + rank * n + i for i in range(n)]
    emulate = args.emulate_world if world == 1 and args.emulate_world > 1 else 0
    gather = (world > 1 or emulate > 0) if args.gather is None else (args.gather and (world > 1 or emulate > 0))
    chunks = int(args.chunks) if args.chunks != "auto" else pipeline.default_chunks(spec, n)
    if gather and args.chunks == "auto":
        # the exchange takes a stream of its own: 2 chunk streams + it + the caller's fit the 4 hardware queues
        chunks = min(chunks, 2)
    if gather:
        from magical_amd import dist as mdist
        shard = mdist.ShardedVecEnv(args.env, n, rank=rank, device=str(device), gather=True,
                                    gather_mode=args.gather_mode, emulate_world=emulate or None,
                                    window=args.restack == "window", chunks=chunks)
        vec = shard.vec
        step = shard.step_async
    window = args.stacks == "window"
    if chunks > 1 and not gather:
        vec = pipeline.PipelinedVecEnv(args.env, n, chunks=chunks, device=str(device), seeds=seeds, window=window)
        step = vec.step
    elif not gather:
        vec = magical_amd.make_vec(args.env, n, device=str(device), seeds=seeds, window=window)
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
        shard.wait_all()
    if chunks > 1:
        vec.wait()
    torch.cuda.synchronize(device)
    if chunks > 1:
        vec.enable_timing(args.steps)
    else:
        native.check(lib.mg_enable_timing(vec.handle, args.steps))
    if gather:
        shard.enable_restack_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s in range(args.steps):
        vec.random_actions(args.warmup + s, out=actions)
        step(actions)
    if gather:   # the timed region ends after the last step's exchange (all-gather + restack)
        shard.wait_all()
    if chunks > 1:   # ... and after every chunk's last step
        vec.wait()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    import ctypes
    if chunks > 1:   # per-launch averages over the chunks' launches (each launch covers n / chunks envs)
        tms = vec.read_timing()
        tm = [sum(t[i] for t in tms) / chunks for i in range(4)]
    else:
        tm = (ctypes.c_double * 4)()
        native.check(lib.mg_read_timing(vec.handle, tm))
    t_step_ms, t_render_ms, n_timed = tm[0] / args.steps, tm[1] / args.steps, int(tm[2])
    t_reset_ms = tm[3] / args.steps
    units = n / chunks   # envs one kernel launch completes (on average over the chunks)
    errors = int((vec.errors() != 0).sum().item())   # the timed run's (before the isolated pass below)
    sim0 = vec.sims[0] if chunks > 1 else vec
    form, blk, caps = sim0.step_form()
    live = float(sim0.bodies()[1][:, 3].double().mean().item())   # active arbiters per env after the timed run
    step_bytes = step_state_bytes(form, caps, live)
    # chunked runs: the timed launches overlap the other chunk's kernels, so their HIP-event times are
    # co-running figures.  The roofline's per-kernel times come from an isolated pass after the timed region:
    # chunk 0 stepped alone (its step, reset and render kernels back to back on one stream, nothing beside
    # them), args.iso_steps steps of the same env count per launch.  Unchunked runs keep the timed launches (one
    # stream; the many-block scenes' next-layout shadow co-runs on the simulator's side stream in every step, as
    # in steady-state use).  Round 6: an isolated pass for them too (the device synchronised before each step)
    # measured the cooperative step kernel 5% LONGER than the timed launches (2.84 vs 2.70 ms, ClusterColour), and
    # under rocprofv3 the same HIP events read 2.47 / 2.58 ms against rocprof's 2.45 / 2.54 ms -- the events
    # agree with the profiler within the same run, and the profiler itself shortens that kernel by ~10%.
    iso = None
    if chunks > 1 and args.iso_steps > 0:
        native.check(lib.mg_enable_timing(sim0.handle, args.iso_steps))
        a0 = torch.empty(sim0.num_envs, dtype=torch.uint8, device=device)
        for s in range(args.iso_steps):
            sim0.random_actions(10 ** 6 + s, out=a0)
            sim0.step(a0)
        torch.cuda.synchronize(device)
        ti = (ctypes.c_double * 4)()
        native.check(lib.mg_read_timing(sim0.handle, ti))
        iso = {"steps": args.iso_steps, "envs_per_launch": sim0.num_envs,
               "step_kernel": ti[0] / args.iso_steps, "render_kernel": ti[1] / args.iso_steps,
               "reset_kernel": ti[3] / args.iso_steps}

    def pmc_for(kernel):
        """The committed PMC record of this workload at this many envs per launch (the passes run the bench's
        own chunking; rocprofv3 counts each dispatch on its own)."""
        return load_pmc(kernel, args.env, n, units)
    ranks_seen = world
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([errors, 1], dtype=torch.int64, device=device)
        dist.all_reduce(e)
        errors, ranks_seen = int(e[0].item()), int(e[1].item())
    value = world * n * args.steps / elapsed   # (--emulate-world: this rank's env-steps/s under the W-rank load)
    restack_ms = shard.restack_ms() / args.steps if gather and shard.restack_timing else None
    exchange_ms = shard.exchange_ms() / args.steps if gather and shard.restack_timing else None
    if rank == 0:
        frames_only = gather and args.gather_mode == "frames"
        stacks_window = bool(getattr(vec, "window_k", 0)) and not gather
        # per-kernel roofline records: from the isolated pass when the timed launches co-ran (chunks > 1)
        k_step, k_render, k_reset = (iso["step_kernel"], iso["render_kernel"], iso["reset_kernel"]) if iso else \
            (t_step_ms, t_render_ms, t_reset_ms)
        kernels = {
            "render_kernel": kernel_record("render_kernel", k_render, spec.preproc, units,
                                           pmc_for("render_kernel"), frames_only, stacks_window),
            "step_kernel": kernel_record("step_kernel", k_step, spec.preproc, units, pmc_for("step_kernel"),
                                         step_bytes=step_bytes),
            "reset_kernel": {"ms": round(k_reset, 4)},
            "timing": "isolated (chunk 0 alone after the timed region)" if iso else "timed launches (one stream)",
            "step_form": {"form": form, "envs_per_workgroup": blk, "caps_bodies_shapes_constraints_arbiters": caps,
                          "live_arbiters_per_env": round(live, 3), "state_bytes_per_env_step": step_bytes},
        }
        dom = "render_kernel" if k_render >= k_step else "step_kernel"
        dk = kernels[dom]
        ms_step = elapsed / args.steps * 1e3
        # whole-step fraction: SURVEY 8(d) bytes of every env-step this GPU completes per timed step
        step_achieved, step_frac = step_fraction(spec.preproc, n, ms_step)
        out = {
            "metric": "env-steps/sec (whole node) at N instances/GPU, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "emulated_world": emulate or None,
            # --emulate-world W: one process stands in for rank 0 of a W-rank node; value is THIS rank's
            # env-steps/s under the emulated exchange, not a whole-node figure
            "value_scope": "per rank (emulated W-rank exchange on one GPU)" if emulate else "whole node",
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device Philox uniform actions over the 18 discrete actions; env i seeded 1000+i)",
            "config": {"workload": args.env, "envs_per_gpu": n, "episode_steps": spec.max_episode_steps,
                       "physics_substeps": 10, "solver_iterations": 10, "render": "2 x 384^2 -> 96^2",
                       "phase_spread": phase_spread,
                       "step_form": f"{form}/{blk}",
                       "env_overrides": env_overrides(),
                       "pipeline_chunks": chunks,
                       "frame_stacks": ("strided views of channel-planar window rings (mg_bind_window)"
                                        if stacks_window else "materialised [N, 96, 96, 12]" if not gather else
                                        "receivers: " + ("window rings" if isinstance(getattr(shard, "restacker", None),
                                                                                   mdist.WindowRestacker) else
                                                         "materialised")),
                       "parallelism": (f"dp{world} (envs sharded; one packed all-gather per step ({args.gather_mode}), "
                                       f"pipelined with the next step)" if gather else
                                       f"dp{world} (envs sharded, no data-path collective)")},
            # dominant kernel against HBM with SURVEY 8(d)'s bytes per env-step x the envs one launch
            # completes; traffic_ratio = its PMC bytes per launch over its own 8(d) share (render: obs + state,
            # step: state); the ring-inclusive bytes of the render kernel's design under "kernel_bytes"; the
            # binding resource of both kernels is VALU issue / latency
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": dk["achieved_gbs"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": dk["hbm_frac"], "traffic": dk["traffic_bytes_per_launch"],
                         "kernel_timing": kernels["timing"],
                         "step_achieved": round(step_achieved, 2), "step_frac": round(step_frac, 5),
                         "traffic_ratio": dk["traffic_ratio"],
                         "traffic_ratio_basis_bytes_per_env_step": dk["traffic_ratio_basis_bytes_per_env_step"],
                         "bytes_per_env_step": dk["bytes_per_env_step"], "units_per_launch": round(units, 1),
                         "kernel_avg_ms": dk["ms"],
                         "kernel_bytes": {"bytes_per_env_step": dk["kernel_bytes_per_env_step"],
                                          "achieved": dk["kernel_bytes_achieved_gbs"],
                                          "frac": dk["kernel_bytes_hbm_frac"]},
                         "binding": "valu_issue_latency",
                         "valu_issue_frac": dk["valu_issue_frac"], "wait_any_frac": dk["wait_any_frac"]},
            "kernels": kernels,
            # the timed launches' HIP-event averages, per launch (one launch per chunk and step: chunks > 1 co-run
            # them with the other chunk's kernels, so these do not add up to ms_per_step)
            "kernel_ms_per_step": {"step_kernel": round(t_step_ms, 4), "reset_kernel": round(t_reset_ms, 4),
                                   "render_kernel": round(t_render_ms, 4), "timed_launches": n_timed,
                                   "envs_per_launch": round(units, 1),
                                   "timing": "co-running (chunks overlap)" if chunks > 1 else "one stream"},
            "env_errors": errors,
            "gather": ({"mode": args.gather_mode, "ranks": shard.world, "bytes_per_rank_step": shard.layout.nbytes,
                        "stacked_bytes_per_rank_step": shard.stacked_nbytes,
                        "received_bytes_per_rank_step": (shard.world - 1) * shard.layout.nbytes,
                        "restack": ("window" if isinstance(shard.restacker, mdist.WindowRestacker) else "materialize")
                                   if frames_only else None,
                        "restack_bytes_per_rank_step": (shard.world * n * restack_bytes(
                            spec.preproc, window=isinstance(shard.restacker, mdist.WindowRestacker))
                                                        if frames_only else 0),
                        "emulated": bool(emulate), "emulated_copy": shard.emulated_copy,
                        "restack_ms_per_step": round(restack_ms, 4) if restack_ms is not None else None,
                        "exchange_ms_per_step": round(exchange_ms, 4) if exchange_ms is not None else None}
                       if gather else None),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    (shard if gather else vec).close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
