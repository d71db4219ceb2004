#!/usr/bin/env python3
"""Per-step kernel sequence from a rocprofv3 SQLite database (rocpd format).

    python tools/prof_step.py gpurun_out/prof/run_results.db [--anchor env_step_kernel] [--index 60]

Takes the window between two consecutive launches of the anchor kernel (one bench step)
and prints every kernel in it with its start offset and duration, then a per-kernel-family
summary and the busy time. Used to find what a step is made of under HIP-graph replay.
"""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="env_step_kernel")
    ap.add_argument("--index", type=int, default=-10, help="which anchor launch starts the window")
    ap.add_argument("--quiet", action="store_true", help="summary only")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if a.anchor in r[0]]
    i0, i1 = idx[a.index], idx[a.index + 1]
    t0 = rows[i0][1]
    fam = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in rows[i0:i1]:
        name = re.sub(r"\(.*", "", r[0].replace("(anonymous namespace)::", "").replace("void ", ""))
        d = (r[2] - r[1]) / 1e3
        busy += d
        key = name[:70]
        fam[key][0] += 1
        fam[key][1] += d
        if not a.quiet:
            print(f"{(r[1] - t0) / 1e3:8.1f} {d:7.1f}  {r[3] // max(r[4], 1):6d}x{r[4]:4d}  {name[:90]}")
    print(f"window {(rows[i1][1] - t0) / 1e3:.1f} us, {i1 - i0} kernels, busy {busy:.1f} us")
    for k, (n, d) in sorted(fam.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{d:9.1f} us {n:4d}x  {k}")


if __name__ == "__main__":
    main()
