#!/usr/bin/env python3
"""Instruction mix of kernels in a device assembly file (hipcc --cuda-device-only -S):
    python tools/isa_mix.py file.s critic_kernelILi1ELi32 [--top 40]"""
import collections
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    s = open(path).read()
    for m in re.finditer(r"^(_Z\S+):", s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        ins = collections.Counter()
        for line in body.split("\n"):
            t = line.strip().split()
            if t and re.match(r"^(s|v|ds|global|buffer|flat|scratch)_", t[0]):
                ins[t[0]] += 1
        print(name[:80], "total", sum(ins.values()))
        for k, v in ins.most_common(top):
            print(f"  {v:6d} {k}")


if __name__ == "__main__":
    main()
