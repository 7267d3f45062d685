"""Phase breakdown of the step and render kernels (profiling build).

MAGICAL_AMD_PROFILE=1 python tools/gpu_phase.py [env] [envs] [steps]
Loads libmagical_sim_prof.so (-DMG_PROFILE): one lane per wave (physics) /
thread 0 per workgroup (render) accumulates s_memtime deltas per phase.
Render phases are measured after each barrier, so a phase includes the wait
for the slowest wave of the workgroup.
"""
import ctypes
import os
import sys

os.environ["MAGICAL_AMD_PROFILE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "magical-1_amd")]
import torch  # noqa: E402
import magical_amd  # noqa: E402
from magical_amd import native  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "MoveToRegion-Demo-LoRes4E-v0"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
vec = magical_amd.make_vec(name, n, seeds=[1000 + i for i in range(n)])
lib = native.load()
lib.mg_debug_read_profile.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 64)()
acts = torch.empty(n, dtype=torch.uint8, device="cuda")
vec.reset()
for s in range(5):
    vec.random_actions(s, out=acts)
    vec.step(acts)
torch.cuda.synchronize()
lib.mg_debug_read_profile(buf)
for s in range(steps):
    vec.random_actions(100 + s, out=acts)
    vec.step(acts)
torch.cuda.synchronize()
lib.mg_debug_read_profile(buf)
v = list(buf)
R = ["setup: bin fill", "band clear+prefetch", "band lines", "band fill+resolve", "band output"]
X = ["max-thread lines work", "max-thread fill work", "long segments", "bin items", "band geoms"]
P = ["robot_update", "integrate+bb", "broad+narrow", "arb filter", "prestep", "cached impulses", "iterations",
     "tail(score/reset)", "  (broad: pair tests + collide)", "  (broad: arbiter updates)", "  (collide calls)",
     "  (arbiter updates)"]
for view, base in (("allo", 0), ("ego", 16)):
    tot = sum(v[base:base + 5]) + sum(v[base + 10:base + 16])
    print(f"render {view}: total {tot / 1e6:.1f}M ticks over {steps} steps x {n} WGs")
    for i, nm in enumerate(R):
        print(f"   {nm:22s} {v[base + i] / max(tot, 1) * 100:6.1f}%  {v[base + i] / (steps * n):10.0f} ticks/WG")
    for i, nm in zip(range(10, 16), ["  setup: ents/xforms", "  setup: geom tables", "  setup: matrices",
                                      "  setup: verts+dashes", "  setup: bounds+count", "  setup: ebin count+scan"]):
        print(f"   {nm:22s} {v[base + i] / max(tot, 1) * 100:6.1f}%  {v[base + i] / (steps * n):10.0f} ticks/WG")
    for i, nm in enumerate(X):
        print(f"   {nm:22s} {v[base + 5 + i] / (steps * n):10.1f} per WG (sum over bands)")
if v[63]:
    print(f"render scene sizes over {v[63]} (env, view) renders: max geoms {v[52]}, vertices {v[53]}, dash lines "
          f"{v[54]}, solid edges {v[55]}, bin entries {v[56]}; above caps: geoms>48 {v[57]}, geoms>64 {v[58]}, "
          f"geoms>72 {v[59]}, NV>1168 {v[60]}, bins>2080 {v[61]}, dashes>128 or sedges>712 {v[62]}")
tot = sum(v[32:42])
# one timer per workgroup (its first lane): the robot scenes' quad forms run blk envs per workgroup (16, or 8 below
# 16 envs per CU), the cooperative form one env per workgroup
robot = name.startswith(("MoveToRegion", "MoveToCorner"))
blk = int(os.environ.get("MG_STEP_BLK", 0)) or ((16 if n >= 16 * 256 else 8) if robot else 1)
wgs = (n + blk - 1) // blk
print(f"physics: total {tot / 1e6:.1f}M ticks, {wgs} workgroups of {blk} envs")
for i, nm in enumerate(P):
    print(f"   {nm:32s} {v[32 + i] / max(tot, 1) * 100:6.1f}%  {v[32 + i] / (steps * wgs):10.0f} per workgroup-step")
vec.close()
