"""Find seeds whose reset needs >= 1 failed pm_randomise_all_poses retry and then places
(geom.py:295-341), per TestAll task, by scanning the CPU oracle.  The seeds feed
tests/test_gpu_parity.py::test_layout_retry_parity.
python tools/scan_retry_seeds.py N MAX_TRIES [names...]   (MAX_TRIES lowers geom.py:198's 10000)"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "oracle"),
                os.path.join(os.path.dirname(__file__), "..", "magical-1_amd")]
import pyoracle as po  # noqa: E402
from magical_amd import registry  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
MAX_TRIES = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
for name in sys.argv[3:] or ["MatchRegions-TestAll-v0", "FindDupe-TestAll-v0", "FixColour-TestAll-v0",
                             "ClusterColour-TestAll-v0", "MakeLine-TestAll-v0"]:
    spec = registry.lookup(name)
    hits, fails = [], 0
    for seed in range(N):
        o = po.OracleEnv(spec.task, spec.rand_flags, None, 1, seed=seed)
        o.set_max_tries(MAX_TRIES)
        try:
            o.reset()
        except po.PlacementError:
            fails += 1
            continue
        if o.placement_retries() > 0:
            hits.append((seed, o.placement_retries()))
    print(name, f"{len(hits)} retry-then-place seeds of {N}, {fails} PlacementErrors:", hits[:12], flush=True)
