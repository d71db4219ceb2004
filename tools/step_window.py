#!/usr/bin/env python3
"""One graph-replayed training step's kernels from a rocprofv3 rocpd database: the window between two
consecutive launches of the anchor kernel (default the fused critic update) in the middle of the run,
every kernel in it (both streams) with start offset, duration and queue, then a per-family summary.

    python tools/step_window.py gpurun_out/<run>/run_results.db [--anchor critic_fused_kernel] [--at 0.6]
"""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="critic_fused_kernel")
    ap.add_argument("--at", type=float, default=0.6, help="where in the run (fraction of the anchor launches)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else "0")
    rows = list(c.execute(f"select name, start, end, {q} from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if a.anchor in r[0]]
    k = int(len(idx) * a.at)
    i0, i1 = idx[k], idx[k + 1]
    t0 = rows[i0][1]
    fam = collections.defaultdict(lambda: [0, 0.0])
    for r in rows[i0:i1]:
        name = re.sub(r"\(.*", "", r[0].replace("(anonymous namespace)::", "").replace("void ", ""))
        d = (r[2] - r[1]) / 1e3
        fam[name[:70]][0] += 1
        fam[name[:70]][1] += d
        print(f"{(r[1] - t0) / 1e3:8.1f} {d:7.1f}  q{r[3]}  {name[:90]}")
    print(f"window {(rows[i1][1] - t0) / 1e3:.1f} us, {i1 - i0} kernels")
    for n, (cnt, d) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{d:9.1f} us {cnt:3d}x  {n}")


if __name__ == "__main__":
    main()
