#!/usr/bin/env python3
"""Per-kernel average durations side by side from tools/ab_bench.sh's traces:
    python tools/ab_stats.py default v1 ... [--top 20]"""
import csv
import sys

names = [a for a in sys.argv[1:] if not a.startswith("--")]
top = 22
tabs = {}
for n in names:
    rows = list(csv.DictReader(open(f"gpurun_out/ab_{n}/run_kernel_stats.csv")))
    tabs[n] = {r["Name"][:70]: (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"])) for r in rows}
base = tabs[names[0]]
order = sorted(base, key=lambda k: -base[k][2])[:top]
print(" ".join(f"{n:>10s}" for n in names), " kernel (avg us)")
for k in order:
    print(" ".join(f"{tabs[n].get(k, (float('nan'),))[0]:10.1f}" for n in names), "", k)
print(" ".join(f"{sum(v[2] for v in tabs[n].values()) / 1e6:10.2f}" for n in names), " total ms")
