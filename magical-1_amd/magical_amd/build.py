"""Build the in-tree HIP library: python -m magical_amd.build

hipcc --offload-arch=gfx950 with -ffp-contract=off (no fused multiply-add
except the explicit __fma_rn that reproduces numpy's BLAS arithmetic).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
OUT = os.path.join(HERE, "libmagical_sim.so")
SOURCES = ["mg_sim.hip"]
HEADERS = ["mg_common.h", "mg_math.h", "mg_state.h", "mg_phys.h", "mg_step.h", "mg_reset.h", "mg_score.h",
           "mg_render.h"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "magical_sim.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    cmd = ["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-shared",
           "-Wno-unused-result", "-o", OUT + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
