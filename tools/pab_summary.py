#!/usr/bin/env python3
"""Average duration per critic-kernel instantiation in gpurun_out/pab_<variant>/run_results.db."""
import collections
import re
import sqlite3
import sys

for v in sys.argv[1:]:
    c = sqlite3.connect(f"gpurun_out/pab_{v}/run_results.db")
    d = collections.defaultdict(list)
    for n, s, e in c.execute("select name, start, end from kernels"):
        if "critic" in n:
            d[re.sub(r"\(asvrl.*", "", n).replace("void asvrl::(anonymous namespace)::", "")].append((e - s) / 1e3)
    print("==", v, "  ".join(f"{k}={sum(x) / len(x):.1f}" for k, x in sorted(d.items())))
