#!/usr/bin/env python3
"""profiles/rNN_env_pmc.json from two tools/pmc_env.sh runs (tools/pmc_summary.py --json outputs):
the env step at 4096 envs (bench config 2's shape, env_pairs_kernel<256, 2>) and at 2^18 envs (the
plateau shape, env_pairs_kernel<64, 2>). Per-launch means; f64_flop = 64 lanes x (ADD + MUL + TRANS +
2 FMA) FP64 wave instructions (an upper bound: every lane counted active).

    python tools/env_pmc_json.py /tmp/e4096.json /tmp/e262k.json profiles/r04_env_pmc.json
"""
import json
import sys


def pick(f, name):
    d = json.load(open(f))
    for k, v in d.items():
        if k.endswith(name):
            v = dict(v)
            v["f64_flop"] = 64 * (v["SQ_INSTS_VALU_ADD_F64"] + v["SQ_INSTS_VALU_MUL_F64"] + v["SQ_INSTS_VALU_TRANS_F64"]
                                  + 2 * v["SQ_INSTS_VALU_FMA_F64"])
            return v
    raise KeyError(name)


out = {"source": "rocprofv3 --pmc, tools/pmc_env.sh (tools/bench_env.py, f32 noise, automatic launch shape); "
                 "per-launch means; sizes in KB",
       "env_pairs_kernel<256, 2> @4096": pick(sys.argv[1], "env_pairs_kernel<256, 2>"),
       "env_pairs_kernel<64, 2> @262144": pick(sys.argv[2], "env_pairs_kernel<64, 2>")}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1)[:400])
