#!/usr/bin/env python3
"""Per-kernel averages of the PMC passes written by tools/pmc_run.sh.

    python tools/pmc_summary.py gpurun_out/pmc [--match critic_kernel]

FETCH_SIZE is reported raw and doubled (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md 'HBM'); sizes are in KB per dispatch as rocprofv3 reports them."""
import argparse
import collections
import csv
import glob
import os
import re


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default=None, help="also write {kernel: {counter: mean}} here")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("sq", "sq2", "f64", "fetch", "write"):
        for r in load(os.path.join(a.dir, p)):
            name = r.get("Kernel_Name", r.get("Kernel-Name", "")).replace("(anonymous namespace)", "anon")
            name = re.sub(r"\(.*", "", name)
            if a.match and a.match not in name:
                continue
            cn = r.get("Counter_Name", r.get("Counter-Name"))
            agg[name][cn].append(float(r.get("Counter_Value", r.get("Counter-Value"))))
    summary = {}
    for name, cs in sorted(agg.items()):
        out = {k: sum(v) / len(v) for k, v in cs.items()}
        if "FETCH_SIZE" in out:
            out["FETCH_SIZE_x2"] = 2 * out["FETCH_SIZE"]
        summary[re.sub(r"^(void )?asvrl::anon::", "", name)] = out
        print(name[:90])
        for k in sorted(out):
            print(f"    {k:28s} {out[k]:16.1f}  (n={len(cs[k]) if k in cs else len(cs['FETCH_SIZE'])})")
    if a.json:
        import json
        json.dump({"source": "rocprofv3 --pmc, tools/pmc_run.sh (bench.py workload); sizes in KB per dispatch",
                   **summary}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
