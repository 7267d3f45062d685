"""Build the in-tree HIP library: python -m magical_amd.build [--force] [--profile]

Translation units compiled in parallel for gfx950 (hipcc
--offload-arch=gfx950, -ffp-contract=off: no fused multiply-add except the
explicit __fma_rn that reproduces numpy's BLAS arithmetic), then linked into
magical_amd/libmagical_sim.so.  Objects are rebuilt only when their sources
change.  --profile builds libmagical_sim_prof.so with -DMG_PROFILE phase timers.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "magical_sim.h")
OBJDIR = os.path.join(os.path.dirname(HERE), "build")
OUT = os.path.join(HERE, "libmagical_sim.so")
PROF_OUT = os.path.join(HERE, "libmagical_sim_prof.so")  # -DMG_PROFILE phase timers (tools/gpu_phase.py)
_COMMON = ["mg_common.h", "mg_math.h", "mg_state.h", "mg_launch.h", "mg_prof.h"]
_PHYS = _COMMON + ["mg_phys.h", "mg_step.h"]
_STEP = _PHYS + ["mg_reset.h", "mg_score.h", "mg_stepk.h", "mg_stepq.h"]
UNITS = {  # translation unit -> headers it depends on (one unit per kernel family: they compile in parallel)
    "mg_sim.hip": _COMMON + ["mg_phys.h"],
    "mg_physics.hip": _COMMON + ["mg_phys.h"],
    "mg_reset.hip": _COMMON + ["mg_phys.h", "mg_reset.h"],
    "mg_step_v4.hip": _STEP,
    "mg_step_quad.hip": _STEP,
    "mg_step_hbm.hip": _STEP,
    "mg_raster.hip": _PHYS + ["mg_render.h"],
    "mg_replay.hip": ["mg_common.h"],
}
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-Wno-unused-result"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def build(force=False, verbose=False, profile=False):
    out = PROF_OUT if profile else OUT
    tag = "prof" if profile else "opt"
    units = dict(UNITS)
    os.makedirs(OBJDIR, exist_ok=True)
    procs, objs = [], []
    for unit, headers in units.items():
        obj = os.path.join(OBJDIR, unit.replace(".hip", f".{tag}.o"))
        objs.append(obj)
        deps = [os.path.join(CSRC, unit), INCLUDE] + [os.path.join(CSRC, h) for h in headers]
        if not force and _mtime(obj) > max(_mtime(d) for d in deps):
            continue
        cmd = ["hipcc"] + FLAGS + (["-DMG_PROFILE"] if profile else []) + ["-c", os.path.join(CSRC, unit),
                                                                         "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd, cwd=CSRC), obj))
    for p, obj in procs:
        if p.wait() != 0:
            raise RuntimeError(f"hipcc failed for {obj}")
        os.replace(obj + ".tmp", obj)
    if force or procs or _mtime(out) < max(_mtime(o) for o in objs):
        cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, profile="--profile" in sys.argv))
