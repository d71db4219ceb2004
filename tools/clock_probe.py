#!/usr/bin/env python3
"""Effective GPU clock per dispatch across a bench run, for the start-up transient of the driver's short timed
region: rocprofv3 --pmc GRBM_GUI_ACTIVE (summed over the 8 XCDs; MI355X_MICROARCH.md 'DVFS
give-back': clock = GRBM_GUI_ACTIVE / 8 / wall, reads high on dispatches shorter than ~0.3 ms, so compare a kernel
with itself over time) with the dispatch's own start / end timestamps. Prints, for the named kernel, its dispatches
in time order in buckets: time since the first dispatch of the process, mean duration, mean effective clock.

    python tools/clock_probe.py gpurun_out/clock/run_counter_collection.csv [--kernel critic_fused_kernel]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="critic_fused_kernel")
    ap.add_argument("--buckets", type=int, default=12)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), float(r["Counter_Value"]))
                 for r in rows if a.kernel in r["Kernel_Name"]), key=lambda x: x[0])
    if not ks:
        raise SystemExit(f"no {a.kernel} dispatches")
    n = len(ks)
    b = max(1, n // a.buckets)
    print(f"{a.kernel}: {n} dispatches; clock = GRBM_GUI_ACTIVE / 8 / duration")
    print(f"{'dispatches':>12s} {'t (ms)':>9s} {'us':>8s} {'GHz':>6s}")
    for i in range(0, n, b):
        g = ks[i:i + b]
        dur = sum(e - s for s, e, _ in g) / len(g)
        ghz = sum(c / 8.0 / (e - s) for s, e, c in g) / len(g)
        print(f"{i:5d}-{i + len(g) - 1:<6d} {(g[0][0] - t0) / 1e6:9.2f} {dur / 1e3:8.2f} {ghz:6.3f}")


if __name__ == "__main__":
    main()
