"""Kernel times of the profiling build (MAGICAL_AMD_PROFILE=1), e.g. under MG_DEBUG_SKIP."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "magical-1_amd")]
import torch  # noqa: E402
import magical_amd  # noqa: E402
from magical_amd import native  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "MoveToRegion-Demo-LoRes4E-v0"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
vec = magical_amd.make_vec(name, n, seeds=[1000 + i for i in range(n)])
lib = native.load()
acts = torch.empty(n, dtype=torch.uint8, device="cuda")
vec.reset()
for s in range(5):
    vec.random_actions(s, out=acts)
    vec.step(acts)
torch.cuda.synchronize()
native.check(lib.mg_enable_timing(vec.handle, 20))
for s in range(20):
    vec.random_actions(100 + s, out=acts)
    vec.step(acts)
torch.cuda.synchronize()
tm = (ctypes.c_double * 4)()
native.check(lib.mg_read_timing(vec.handle, tm))
print(f"step {tm[0] / 20:.3f} ms render {tm[1] / 20:.3f} ms")
