"""CPU: the activation-image swizzle (csrc/asvrl_lds.h, restated in tools/lds_swizzle_check.py) leaves every access
shape of the feature-split kernels -- row reads, row stores, transposed reads -- free of LDS bank conflicts; the
round-5 swizzle conflicted on every 16-byte row store (2-way: 8 extra cycles per store instruction)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_shipped_swizzle_is_conflict_free():
    import lds_swizzle_check as c
    for P, r in c.check(c.swz_shipped).items():
        assert r == {"row_read_extra": 0, "row_store_extra": 0, "transposed_read_extra": 0}, (P, r)
    old = c.check(c.swz_round5)
    assert all(old[P]["row_store_extra"] == 8 * 2 * (P // 16) for P in (64, 128, 256))   # 2-way on every store


def test_swizzle_is_a_permutation_of_each_row():
    import lds_swizzle_check as c
    for P in (64, 128, 256):
        for r in range(64):
            offs = sorted(c.img_off(P, r, p, c.swz_shipped) - r * P for p in range(P))
            assert offs == list(range(P)), (P, r)
