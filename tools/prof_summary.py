"""Summarise rocprofv3 rocpd databases (kernel-trace stats and PMC passes).

python tools/prof_summary.py gpurun_out/<tag>        -> prints tables
python tools/prof_summary.py gpurun_out/<tag> --md   -> markdown (for profiles/)
python tools/prof_summary.py gpurun_out/<tag> --traffic-json profiles/pmc_traffic.json --kernel render_kernel
"""
import argparse
import glob
import json
import os
import sqlite3


def short(name):
    return name.split("(")[0].replace("void ", "")[:60]


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(short(r[0]), r[1], r[2], r[3], r[4]) for r in rows]


def pmc(db):
    c = sqlite3.connect(db)
    q = ("select kernel_name, counter_name, count(*), avg(value), sum(value) from counters_collection "
         "group by kernel_name, counter_name")
    return [(short(r[0]), r[1], r[2], r[3], r[4]) for r in c.execute(q).fetchall()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--traffic-json")
    ap.add_argument("--kernel", default="render_kernel")
    ap.add_argument("--workload", default="MoveToRegion-Demo-LoRes4E-v0")
    ap.add_argument("--envs", type=int, default=4096)
    a = ap.parse_args()
    out = []
    for db in sorted(glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)):
        sub = os.path.relpath(db, a.dir)
        c = sqlite3.connect(db)
        has_pmc = c.execute("select count(*) from counters_collection").fetchone()[0] > 0
        if has_pmc:
            out.append(f"\n### PMC {sub}\n\n| kernel | counter | dispatches | avg per dispatch |\n|---|---|---|---|")
            for k, cn, n, avg, _ in pmc(db):
                if k.startswith(("at::", "__amd")):
                    continue
                out.append(f"| {k} | {cn} | {n} | {avg:.1f} |")
        else:
            out.append(f"\n### kernel trace {sub}\n\n| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|")
            for k, n, tot, avg, pct in kernel_stats(db):
                out.append(f"| {k} | {n} | {tot:.0f} | {avg:.1f} | {pct:.2f} |")
    print("\n".join(out))
    if a.traffic_json:
        # FETCH_SIZE / WRITE_SIZE are KiB per dispatch; gfx950 FETCH_SIZE counts half of wide
        # coalesced reads (MI355X_MICROARCH.md, HBM section) -> doubled.
        # a kernel with several template instances (the render capacity classes, each launched once per
        # step over the same grid): per-step values are the sums over the instances
        fetch = write = None
        sq = {}
        for db in glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True):
            for k, cn, n, avg, _ in pmc(db):
                if not k.startswith(a.kernel):
                    continue
                if cn == "FETCH_SIZE":
                    fetch = (fetch or 0.0) + avg * 1024 * 2
                if cn == "WRITE_SIZE":
                    write = (write or 0.0) + avg * 1024
                if cn.startswith("SQ_") or cn.startswith("GRBM_"):
                    sq[cn] = sq.get(cn, 0.0) + avg
        data = {}
        if os.path.exists(a.traffic_json):
            data = json.load(open(a.traffic_json))
        if fetch is not None and write is not None:
            data[a.kernel] = {"bytes_per_launch": round(fetch + write), "read_bytes": round(fetch),
                              "write_bytes": round(write), "source": a.dir, "workload": a.workload, "envs": a.envs,
                              "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B"}
            if "SQ_INSTS_VALU" in sq and "GRBM_GUI_ACTIVE" in sq:
                # VALU issue utilisation: a wave64 VALU instruction occupies a SIMD-32 for 2 cycles
                # (MI355X_MICROARCH.md, Wave scheduling); 1024 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs
                cyc = sq["GRBM_GUI_ACTIVE"] / 8
                data[a.kernel]["valu_issue_frac"] = round(sq["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 4)
                data[a.kernel]["sq"] = {k: round(v, 1) for k, v in sorted(sq.items())}
                if "SQ_WAVE_CYCLES" in sq and "SQ_WAIT_ANY" in sq:
                    data[a.kernel]["wait_any_frac"] = round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 4)
            json.dump(data, open(a.traffic_json, "w"), indent=1)
            print("traffic", a.kernel, data[a.kernel])


if __name__ == "__main__":
    main()
