"""Summarise a rocprofv3 kernel trace (csv) of tools/overlap_ab.py: how much of the step kernels' time ran
beside a render kernel (the overlap VERDICT r3 item 5 asks for), plus per-kernel average durations.

    python tools/overlap_trace.py <dir with *kernel_trace.csv>
"""
import csv
import glob
import sys


def main(d):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    steps = [(s, e) for n, s, e in rows if n.startswith("step_kernel") or "step_kernel<" in n]
    renders = sorted((s, e) for n, s, e in rows if "render_kernel" in n)
    # union of the render intervals
    merged = []
    for s, e in renders:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot = ov = 0
    for s, e in steps:
        tot += e - s
        for a, b in merged:
            if b <= s:
                continue
            if a >= e:
                break
            ov += min(b, e) - max(a, s)
    by = {}
    for n, s, e in rows:
        k = n.split("(")[0][:60]
        c, t = by.get(k, (0, 0))
        by[k] = (c + 1, t + e - s)
    for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
        print(f"{k:60s} {c:6d} launches  avg {t / c / 1e6:8.4f} ms")
    print(f"step kernels: {len(steps)}, {tot / 1e6:.2f} ms in all; beside a render kernel: {ov / 1e6:.2f} ms "
          f"({100.0 * ov / max(tot, 1):.1f}%)")


if __name__ == "__main__":
    main(sys.argv[1])
