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


def isolated_stats(db):
    """Per kernel: calls and average duration (us) of the dispatches that overlap no other kernel dispatch in
    time (bench.py's isolated pass: chunk 0 stepped alone), next to all dispatches."""
    c = sqlite3.connect(db)
    try:
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
    except sqlite3.Error:
        return {}
    ev = [(short(n), s, e) for n, s, e in rows]
    out = {}
    max_end = -1
    for i, (n, s, e) in enumerate(ev):
        prev_overlap = max_end > s
        nxt_overlap = i + 1 < len(ev) and ev[i + 1][1] < e
        max_end = max(max_end, e)
        d = out.setdefault(n, [0, 0.0, 0, 0.0])
        d[0] += 1; d[1] += (e - s) / 1e3
        if not prev_overlap and not nxt_overlap:
            d[2] += 1; d[3] += (e - s) / 1e3
    return {n: (d[0], d[1] / d[0], d[2], d[3] / d[2] if d[2] else None) for n, d in out.items()}


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
    ap.add_argument("--envs-per-launch", type=float, default=None,
                    help="envs one launch of the kernel covers (chunked bench runs: envs / chunks)")
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
            iso = isolated_stats(db)
            if iso:
                out.append(f"\n#### isolated dispatches {sub} (overlapping no other kernel: bench.py's isolated pass)\n\n"
                           "| kernel | isolated calls | isolated avg us | all calls | all avg us |\n|---|---|---|---|---|")
                for k, (n, avg, ni, iavg) in sorted(iso.items(), key=lambda x: -x[1][0] * x[1][1]):
                    if k.startswith(("at::", "__amd")) or n < 2:
                        continue
                    out.append(f"| {k} | {ni} | {iavg:.1f} | {n} | {avg:.1f} |" if iavg else f"| {k} | 0 | - | {n} | {avg:.1f} |")
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
                              "envs_per_launch": a.envs_per_launch if a.envs_per_launch else a.envs,
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
