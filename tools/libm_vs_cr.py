"""How much does the correctly rounded sin/cos choice change the trajectories?  

Runs the BASELINE configs' parity rollouts (env i seeded 1000 + i, actions RandomState(42)) on two builds
of the CPU oracle in lockstep: the correctly rounded trig the product uses (_build/libmg_oracle.so) and this
image's libm sin/cos/tan (make libm -> _build/libmg_oracle_libm.so), the reference's own math.sin /
Chipmunk cpfsin.  Counts the LoRes observation bytes that differ and the body states (p, angle, v, w) that
differ by more than 1e-4.  CPU only.

    python tools/libm_vs_cr.py [--out profiles/r03_libm_vs_cr.json]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "magical-1_amd")]

CONFIGS = [("MoveToRegion-Demo-LoRes4E-v0", 64, 200), ("MoveToCorner-Demo-LoRes4E-v0", 64, 200),
           ("ClusterColour-Demo-LoResStack-v0", 16, 250), ("MatchRegions-TestAll-LoRes4E-v0", 32, 250)]


def _libs():
    import subprocess
    import pyoracle as po
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "libm"], check=True)
    cr = po.lib()
    po._lib, saved = None, po.LIB_PATH
    po.LIB_PATH = os.path.join(ROOT, "oracle", "_build", "libmg_oracle_libm.so")
    libm = po.lib()
    po._lib, po.LIB_PATH = cr, saved
    return cr, libm


def _env(L, spec, seed):
    import pyoracle as po
    e = object.__new__(po.OracleEnv)
    e.L = L
    e.h = L.oenv_create(po.TASKS[spec.task], spec.rand_flags, po.PREPROCS[spec.preproc], spec.max_episode_steps, seed)
    e.nbytes = L.oenv_obs_bytes(e.h)
    return e


def run(args):
    name, lo, hi, steps = args
    import pyoracle as po
    from magical_amd import registry
    spec = registry.lookup(name)
    cr, libm = _libs()
    acts = np.random.RandomState(42).randint(0, 18, (steps, 4096))
    r = {"env_steps": 0, "obs_bytes": 0, "obs_bytes_diff": 0, "obs_env_steps_diff": 0, "body_states": 0,
         "body_states_gt_1e-4": 0, "body_max_abs": 0.0, "score_diff": 0, "placement_diff": 0,
         "first_obs_diff_step": [], "first_body_diff_step": []}
    for i in range(lo, hi):
        a, b = _env(cr, spec, 1000 + i), _env(libm, spec, 1000 + i)
        try:
            oa, ob = a.reset(), b.reset()
        except po.PlacementError:
            r["placement_diff"] += 1
            continue
        first_o = first_b = None
        for t in range(steps + 1):
            if t > 0:
                oa, ra, da, sa = a.step(int(acts[t - 1, i]))
                ob, rb, db, sb = b.step(int(acts[t - 1, i]))
                r["score_diff"] += (sa != sb) or (da != db)
                if da:
                    try:
                        oa = a.reset()
                        ob = b.reset()
                    except po.PlacementError:
                        r["placement_diff"] += 1
                        break
            d = int(np.count_nonzero(oa != ob))
            r["env_steps"] += 1
            r["obs_bytes"] += oa.size
            r["obs_bytes_diff"] += d
            r["obs_env_steps_diff"] += d > 0
            if d and first_o is None:
                first_o = t
            ba, bb = a.bodies(), b.bodies()
            if ba.shape == bb.shape:
                dif = np.abs(ba - bb)
                r["body_states"] += dif.size
                r["body_states_gt_1e-4"] += int(np.count_nonzero(dif > 1e-4))
                r["body_max_abs"] = max(r["body_max_abs"], float(dif.max()))
                if (dif > 1e-4).any() and first_b is None:
                    first_b = t
        r["first_obs_diff_step"].append(first_o)
        r["first_body_diff_step"].append(first_b)
    return name, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_libm_vs_cr.json"))
    ap.add_argument("--workers", type=int, default=8)
    args = ap.parse_args()
    _libs()
    jobs = []
    for name, n, steps in CONFIGS:
        chunk = max(1, n // 8)
        jobs += [(name, lo, min(n, lo + chunk), steps) for lo in range(0, n, chunk)]
    with mp.get_context("fork").Pool(args.workers) as pool:
        res = pool.map(run, jobs)
    out = {}
    for name, n, steps in CONFIGS:
        agg = None
        for nm, r in res:
            if nm != name:
                continue
            if agg is None:
                agg = dict(r, first_obs_diff_step=list(r["first_obs_diff_step"]),
                           first_body_diff_step=list(r["first_body_diff_step"]))
                continue
            for k, v in r.items():
                if isinstance(v, list):
                    agg[k] += v
                elif k == "body_max_abs":
                    agg[k] = max(agg[k], v)
                else:
                    agg[k] += v
        fo = [s for s in agg["first_obs_diff_step"] if s is not None]
        fb = [s for s in agg["first_body_diff_step"] if s is not None]
        agg.update(envs=n, steps=steps, envs_with_obs_diff=len(fo), envs_with_body_diff=len(fb),
                   median_first_obs_diff_step=float(np.median(fo)) if fo else None,
                   median_first_body_diff_step=float(np.median(fb)) if fb else None,
                   obs_byte_diff_frac=agg["obs_bytes_diff"] / max(1, agg["obs_bytes"]))
        del agg["first_obs_diff_step"], agg["first_body_diff_step"]
        out[name] = agg
        print(name, json.dumps(agg), flush=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
