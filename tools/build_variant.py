#!/usr/bin/env python3
"""Build an A/B / instrumentation variant of libasvrl.so into variants/libasvrl_<name>.so: every
source compiled as in build.py, plus extra macros for the named sources (never the shipped library).

    python tools/build_variant.py stamps asvrl_critic_fused.hip=-DASVRL_FUSED_STAMPS
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributional_rl_decision_and_control_amd import build as B  # noqa: E402


def main():
    name = sys.argv[1]
    extra = {}
    for a in sys.argv[2:]:
        src, flags = a.split("=", 1)
        extra[src] = flags.split(",")
    out_dir = os.path.join(ROOT, "variants")
    os.makedirs(out_dir, exist_ok=True)
    procs, objs = [], []
    for src in B.SOURCES:
        base = os.path.basename(src)
        o = os.path.join(out_dir, f"{name}.{base}.o")
        objs.append(o)
        cmd = [B.HIPCC] + B.FLAGS[:3] + ["-c"] + B.FLAGS[3:] + B.SOURCE_FLAGS.get(base, []) + extra.get(base, []) + \
            ["-o", o, src]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("compile failed")
    lib = os.path.join(out_dir, f"libasvrl_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
