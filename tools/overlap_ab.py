"""Does physics/render overlap pay?  (measured before building it into mg_step.)

The same workload (env name, total envs) run as C independent simulators of total/C envs each, every
one on its own HIP stream, stepped round-robin: the GPU is then free to run chunk k's render beside chunk
k+1's step kernel -- what splitting mg_step into env chunks on internal streams would do.  Prints the
env-steps/s for C = 1 (one stream, the bench) and each C given.

    python tools/overlap_ab.py MoveToRegion-Demo-LoRes4E-v0 4096 60 1 2 4
"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/magical-1_amd")
import magical_amd  # noqa: E402


def run(name, total, steps, chunks, warmup=10):
    n = total // chunks
    dev = torch.device("cuda:0")
    vecs, streams, acts = [], [], []
    for c in range(chunks):
        v = magical_amd.make_vec(name, n, device="cuda:0", seeds=[1000 + c * n + i for i in range(n)])
        v.reset()
        L = v.max_episode_steps
        if L > 1:
            v.set_episode_steps(torch.tensor([(c * n + i) % L for i in range(n)], dtype=torch.int32))
        vecs.append(v)
        streams.append(torch.cuda.Stream(dev) if chunks > 1 else torch.cuda.current_stream(dev))
        acts.append(torch.empty(n, dtype=torch.uint8, device=dev))

    def one(s):
        for v, st, a in zip(vecs, streams, acts):
            with torch.cuda.stream(st):
                v.random_actions(s, out=a)
                v.step(a)

    for s in range(warmup):
        one(s)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(steps):
        one(warmup + s)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    for v in vecs:
        assert int((v.errors() != 0).sum().item()) == 0
    return total * steps / dt, 1e3 * dt / steps


if __name__ == "__main__":
    name, total, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    for c in [int(x) for x in sys.argv[4:]] or [1, 2]:
        rate, ms = run(name, total, steps, c)
        print(f"{name} envs {total} chunks {c}: {rate:,.0f} env-steps/s, {ms:.3f} ms per step", flush=True)
