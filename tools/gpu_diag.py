"""Diagnostic rollout: GPU vs oracle for each hot-path config (prints, never asserts)."""
import os, sys, time, traceback
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "magical-1_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import torch
import magical_amd
import pyoracle as po
from magical_amd import registry, envs


def split(spec, flat):
    out, off = {}, 0
    for k, s in envs._obs_shapes(spec).items():
        n = int(np.prod(s)); out[k] = flat[off:off + n].reshape(s); off += n
    return out


def run(name, n, steps):
    spec = registry.lookup(name)
    seeds = [1000 + i for i in range(n)]
    t0 = time.time()
    vec = magical_amd.make_vec(name, n, seeds=seeds)
    orc = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=s) for s in seeds]
    obs = vec.reset()
    ref = [split(spec, o.reset()) for o in orc]
    bad = []
    for k in obs:
        g = obs[k].cpu().numpy()
        for i in range(n):
            if not np.array_equal(g[i], ref[i][k]):
                bad.append(("reset", k, i, int((g[i] != ref[i][k]).sum())))
    print(name, "create+reset", round(time.time() - t0, 2), "s; reset mismatches", bad[:4], flush=True)
    if bad:
        full = vec.render_full().cpu().numpy()
        a, gg = orc[0].render_full()
        print("  full-res allo diff px", int((full[0, 0] != a).any(-1).sum()), "ego diff px", int((full[0, 1] != gg).any(-1).sum()))
        ys, xs = np.nonzero((full[0, 1] != gg).any(-1))
        print("  first ego diffs", list(zip(ys[:8], xs[:8])), full[0, 1][ys[:3], xs[:3]], gg[ys[:3], xs[:3]])
    acts = np.random.RandomState(42).randint(0, 18, (steps, n))
    maxd = 0.0
    first_obs_bad = None
    for t in range(steps):
        obs, rew, done, info = vec.step(torch.as_tensor(acts[t], dtype=torch.uint8))
        bodies, counts = vec.bodies()
        bodies = bodies.cpu().numpy(); got = {k: v.cpu().numpy() for k, v in obs.items()}
        dn = done.cpu().numpy(); sc = info["eval_score"].cpu().numpy()
        for i in range(n):
            o, r, d, s = orc[i].step(int(acts[t, i]))
            if bool(dn[i]) != d or sc[i] != s:
                print(f"  step {t} env {i}: done {dn[i]} vs {d}, score {sc[i]} vs {s}")
            if d:
                o = orc[i].reset()
            else:
                b = orc[i].bodies()
                dd = float(np.abs(bodies[i, :len(b)] - b).max())
                if dd > maxd:
                    maxd = dd
                    if dd > 1e-9:
                        print(f"  step {t} env {i}: body diff {dd:.3e} (argmax {np.unravel_index(np.abs(bodies[i,:len(b)]-b).argmax(), b.shape)})")
            rr = split(spec, o)
            for k in got:
                if not np.array_equal(got[k][i], rr[k]) and first_obs_bad is None:
                    first_obs_bad = (t, i, k, int((got[k][i] != rr[k]).sum()))
    err = vec.errors().cpu().numpy()
    print(f"  {steps} steps: max body diff {maxd:.3e}; first obs mismatch {first_obs_bad}; error flags {np.unique(err)}; {time.time()-t0:.1f}s", flush=True)
    vec.close()


if __name__ == "__main__":
    print("device", torch.cuda.get_device_name(0), flush=True)
    cfgs = [("MoveToRegion-Demo-LoRes4E-v0", 4, 90), ("MoveToCorner-Demo-LoRes4E-v0", 4, 90),
            ("ClusterColour-Demo-LoResStack-v0", 2, 50), ("MatchRegions-TestAll-LoRes4E-v0", 3, 130)]
    for name, n, steps in cfgs:
        try:
            run(name, n, steps)
        except Exception:
            traceback.print_exc()
