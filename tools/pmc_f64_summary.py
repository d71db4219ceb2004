#!/usr/bin/env python3
"""Per-launch FP64 VALU instruction counts of the env kernels from tools/pmc_f64.sh:
    python tools/pmc_f64_summary.py gpurun_out/pmc_f64/f64 profiles/r01_env_f64_pmc.json
FLOP per launch = 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave instructions (an upper bound: every
lane counted active). SQ_WAVES matches the launch's wave count, so the SQ counters are chip totals."""
import collections
import csv
import json
import os
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in ("run_counter_collection.csv",):
    for r in csv.DictReader(open(os.path.join(src, f))):
        n = r["Kernel_Name"]
        if "env_step" not in n and "env_reset" not in n:
            continue
        n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)", "anon"))
        n = re.sub(r"^(void )?asvrl::anon::", "", n)
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"source": "rocprofv3 --pmc SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 (tools/pmc_f64.sh, bench.py workload); "
                 "per-launch means, wave instructions"}
for n, cs in agg.items():
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    m["f64_flop"] = 64 * (m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] + m["SQ_INSTS_VALU_TRANS_F64"]
                          + 2 * m["SQ_INSTS_VALU_FMA_F64"])
    m["launches"] = len(cs["SQ_WAVES"])
    out[n] = m
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
