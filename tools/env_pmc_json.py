#!/usr/bin/env python3
"""profiles/rNN_env_pmc.json from two tools/pmc_env.sh runs (tools/pmc_summary.py --json outputs):
the env step at 4096 envs (bench config 2's shape) and at 2^18 envs (the plateau shape), each summary's one
env_pairs_kernel instance (the automatic launch shape's). Per-launch means; f64_flop = 64 lanes x (ADD + MUL + TRANS +
2 FMA) FP64 wave instructions (an upper bound: every lane counted active).

    python tools/env_pmc_json.py /tmp/e4096.json /tmp/e262k.json profiles/r04_env_pmc.json
"""
import json
import sys


def pick(f, name):
    """The summary's entry for kernel `name`, or for its only env_pairs_kernel instance when name is None."""
    d = json.load(open(f))
    for k, v in d.items():
        if (name is None and "env_pairs_kernel<" in k) or (name is not None and k.endswith(name)):
            v = dict(v)
            v["f64_flop"] = 64 * (v["SQ_INSTS_VALU_ADD_F64"] + v["SQ_INSTS_VALU_MUL_F64"] + v["SQ_INSTS_VALU_TRANS_F64"]
                                  + 2 * v["SQ_INSTS_VALU_FMA_F64"])
            return k[k.index("env_pairs_kernel<"):], v
    raise KeyError(name)


k4, v4 = pick(sys.argv[1], None)
kp, vp = pick(sys.argv[2], None)
out = {"source": "rocprofv3 --pmc, tools/pmc_env.sh (tools/bench_env.py, f32 noise, automatic launch shape); "
                 "per-launch means; sizes in KB",
       f"{k4} @4096": v4, f"{kp} @262144": vp}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1)[:400])
