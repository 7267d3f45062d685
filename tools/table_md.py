"""BASELINE.md results table from a tools/gpu_table.sh run.

python tools/table_md.py gpurun_out/table > profiles/r02_results.md
Per config: the bench line (whole-job env-steps/s, HIP-event kernel times, CPU-restatement baseline at
1 process and 16 processes), and per kernel the PMC traffic (FETCH_SIZE x2 + WRITE_SIZE, per launch),
the VALU issue fraction (SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) and the
fraction of wave-cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES).
"""
import glob
import json
import os
import sys

ORDER = ["MoveToRegion-Demo-LoRes4E-v0", "MoveToCorner-Demo-LoRes4E-v0", "ClusterColour-Demo-LoResStack-v0",
         "MatchRegions-TestAll-LoRes4E-v0"]


def main(d):
    rows, krows = [], []
    names = [n for n in ORDER if os.path.exists(os.path.join(d, n + ".json"))]
    names += sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(d, "*-v0.json"))
                    if os.path.basename(p)[:-5] not in names)
    for n in names:
        b = json.load(open(os.path.join(d, n + ".json")))
        t = json.load(open(os.path.join(d, n + ".traffic.json")))
        km = b["kernel_ms_per_step"]
        cb = b["cpu_baseline"]
        r = t["render_kernel"]
        # the PMC passes run unchunked (envs per launch = the traffic record's envs); a pipelined bench line's
        # launches cover envs_per_launch envs each
        sc = km.get("envs_per_launch", r["envs"]) / r["envs"]
        rg = r["bytes_per_launch"] * sc / (km["render_kernel"] * 1e-3) / 1e9
        rows.append(f"| {n} | {b['config']['envs_per_gpu']} | 1 | {b['value']:,.0f} | {b['ms_per_step']:.3f} | "
                    f"{b['roofline']['bytes_per_env_step']:,} | {b['roofline']['achieved']:.0f} | {rg:.0f} | "
                    f"{b['roofline']['achieved'] / 8000:.3f} | {r.get('valu_issue_frac', float('nan')):.2f} | "
                    f"{cb['one_core_env_steps_s']:,.0f} / {cb['value']:,.0f} ({cb['cores']} proc) |")
        for k in ("step_kernel", "reset_kernel", "render_kernel"):
            if k not in t:
                continue
            v = t[k]
            ms = km.get(k, float("nan"))
            krows.append(f"| {n} | {k} | {ms:.3f} | {v['read_bytes'] * sc / 1e6:.1f} | {v['write_bytes'] * sc / 1e6:.1f} | "
                         f"{v['bytes_per_launch'] * sc / (ms * 1e-3) / 1e9:.0f} | {v.get('valu_issue_frac', float('nan')):.3f} | "
                         f"{v.get('wait_any_frac', float('nan')):.3f} | {v['sq'].get('SQ_INSTS_VALU', 0) / max(v['sq'].get('SQ_WAVES', 1), 1):,.0f} |")
    print("| config | envs/GPU | GPUs | env-steps/s | ms/step | algorithmic B/env-step | render GB/s (algorithmic) | "
          "render GB/s (PMC) | HBM fraction (algorithmic / 8 TB/s) | render VALU issue | CPU restatement env-steps/s "
          "(1 proc / job share) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))
    print()
    print("| config | kernel | ms/launch (HIP events; per chunk when pipelined) | PMC read MB | PMC write MB | PMC GB/s | VALU issue frac | "
          "wait-any frac | VALU instrs/wave |")
    print("|---|---|---|---|---|---|---|---|---|")
    print("\n".join(krows))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/table")
