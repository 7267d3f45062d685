"""Receiver-side restack cost of the compact multi-GPU gather on one MI355X (mg_restack), as an 8-rank
node would run it every step: W = 8 rank blocks of n envs each, synthetic frames, every 40th env done.

    python tools/restack_bench.py [env] [n] [world]
Prints one JSON line: ms per restack (HIP events), algorithmic bytes and the HBM fraction.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "magical-1_amd")]
import torch  # noqa: E402
from magical_amd import dist as mdist, registry  # noqa: E402
import bench  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "MoveToRegion-Demo-LoRes4E-v0"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
W = int(sys.argv[3]) if len(sys.argv) > 3 else 8
spec = registry.lookup(name)
lay = mdist.PackedLayout.for_spec(spec, n, frames_only=True)
dev = torch.device("cuda", 0)
recv = torch.randint(0, 256, (W * lay.nbytes,), dtype=torch.uint8, device=dev)
v = lay.unpack(recv)
v["done"].copy_((torch.arange(W * n, device=dev) % 40 == 0).view(W, n))
rs = mdist.NativeRestacker(lay, W, dev)
outs = [{k: torch.empty((W * n, 96, 96, 12), dtype=torch.uint8, device=dev) for k in mdist.stacked_keys(spec.preproc)}
        for _ in range(2)]
for t in range(3):
    rs(recv, outs[t % 2], t, t == 0)
torch.cuda.synchronize()
K = 20
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for t in range(K):
    rs(recv, outs[t % 2], 3 + t, False)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / K
byt = bench.restack_bytes(spec.preproc) * W * n
print(json.dumps({"kernel": "restack_kernel", "workload": name, "envs_per_rank": n, "world": W, "ms": round(ms, 4),
                  "bytes_per_launch": byt, "achieved_gbs": round(byt / ms / 1e6, 1),
                  "hbm_frac": round(byt / ms / 1e6 / bench.HBM_PEAK_GBS, 4)}), flush=True)
