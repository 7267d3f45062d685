"""Rebuild <config>.traffic.json from the PMC tables of a prof_summary --md file (the rocpd databases are
dropped on the box), summing the per-dispatch averages over a kernel's template instances.

python tools/traffic_from_md.py profiles/r02_final   (every <config>.md with a matching .json bench line)
"""
import glob
import json
import os
import sys


def main(d):
    for md in sorted(glob.glob(os.path.join(d, "*-v0.md"))):
        name = os.path.basename(md)[:-3]
        envs = json.load(open(md[:-3] + ".json"))["config"]["envs_per_gpu"]
        acc = {}
        for line in open(md):
            f = [x.strip() for x in line.strip().strip("|").split("|")]
            if len(f) != 4 or not f[2].isdigit():
                continue
            kern, cn, avg = f[0].split("<")[0], f[1], float(f[3])
            acc.setdefault(kern, {})
            acc[kern][cn] = acc[kern].get(cn, 0.0) + avg
        data = {}
        for k in ("render_kernel", "step_kernel", "reset_kernel"):
            c = acc.get(k, {})
            if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
                continue
            fetch, write = c["FETCH_SIZE"] * 1024 * 2, c["WRITE_SIZE"] * 1024
            e = {"bytes_per_launch": round(fetch + write), "read_bytes": round(fetch), "write_bytes": round(write),
                 "source": md, "workload": name, "envs": envs,
                 "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B; summed over template instances"}
            if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
                e["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 2 / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 4)
                e["sq"] = {n: round(v, 1) for n, v in sorted(c.items()) if n.startswith(("SQ_", "GRBM_"))}
                if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
                    e["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
            data[k] = e
        json.dump(data, open(md[:-3] + ".traffic.json", "w"), indent=1)
        print(name, {k: (v["bytes_per_launch"], v.get("valu_issue_frac")) for k, v in data.items()})


if __name__ == "__main__":
    main(sys.argv[1])
