#!/usr/bin/env python3
"""LDS bank-conflict check of the activation-image swizzle (csrc/asvrl_lds.h swz / img_off / RowA / TrA), restated
here: every access shape the feature-split kernels make on a 64-row image of P = 64, 128 or 256 bf16 positions,
against the lane groups and bank widths of MI355X_MICROARCH.md's LDS table:
  row reads   ds_read_b128        4 groups of 16 lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, +32; 64 banks
  row stores  ds_write_b128       8 groups of 8 consecutive lanes;                                  32 banks
  transposed  ds_read_b64_tr_b16  2 groups of 32 lanes;                                             64 banks
Lane l of a row access takes row 32 j + (l & 31), positions 16 ks + 8 (l >> 5) .. + 7 (asvrl_lds.h RowA); of a
transposed access rows 16 kk + 8 (g >> 1) + q (+ 4), columns 32 n + 16 (g & 1) + 4 p (tr_frag). Reports the extra
LDS cycles (a group's extra distinct dwords on its busiest bank) per access shape.

    python tools/lds_swizzle_check.py            # the shipped swizzle and the round-2..5 one
"""
import json

RD128 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
RD128 = RD128 + [[lane + 32 for lane in g] for g in RD128]
WR128 = [list(range(k, k + 8)) for k in range(0, 64, 8)]
TR = [list(range(0, 32)), list(range(32, 64))]


def swz_shipped(P, r):
    """asvrl_lds.h swz<P> (round 6)."""
    if P == 64:
        return (((r >> 1) & 1) << 2) | (((r >> 2) & 3) ^ ((r & 1) << 1))
    return ((r & 3) << 2) | (((r >> 2) & 3) ^ (r & 2))


def swz_round5(P, r):
    """The swizzle of rounds 2-5."""
    if P == 64:
        return (((r >> 1) & 1) << 2) | ((r >> 2) & 3)
    return ((r & 3) << 2) | ((r >> 2) & 3)


def img_off(P, r, p, swz):
    return r * P + (((p >> 3) ^ swz(P, r)) << 3) + (p & 7)


def extra_cycles(addrs, groups, nbytes, nbanks):
    extra = 0
    for g in groups:
        banks = {}
        for lane in g:
            for d in range(nbytes // 4):
                dw = addrs[lane] // 4 + d
                banks.setdefault(dw % nbanks, set()).add(dw)
        extra += max(len(s) for s in banks.values()) - 1
    return extra


def check(swz):
    out = {}
    for P in (64, 128, 256):
        rd = wr = tr = 0
        for j in range(2):
            for ks in range(P // 16):
                a = [2 * img_off(P, 32 * j + (lane & 31), 16 * ks + 8 * (lane >> 5), swz) for lane in range(64)]
                rd += extra_cycles(a, RD128, 16, 64)
                wr += extra_cycles(a, WR128, 16, 32)
        for kk in range(4):
            for n in range(P // 32):
                for hi in (0, 4):
                    a = []
                    for lane in range(64):
                        g, i = lane >> 4, lane & 15
                        q, p = i >> 2, i & 3
                        a.append(2 * img_off(P, 16 * kk + 8 * (g >> 1) + q + hi, 32 * n + 16 * (g & 1) + 4 * p, swz))
                    tr += extra_cycles(a, TR, 8, 64)
        out[P] = {"row_read_extra": rd, "row_store_extra": wr, "transposed_read_extra": tr}
    return out


def main():
    print(json.dumps({"shipped": check(swz_shipped), "round5": check(swz_round5)}))


if __name__ == "__main__":
    main()
