"""CPU check of the rank-fold tree plan (k_rank_tree_mw's indexing, exported
by the test hook pdplqr_debug_rank_tree): for every R <= 17 and rank r, the
levels reduce the prefix list e_0 .. e_{r-1} and the suffix list e_{r+1} ..
e_{R-1} by combines of ADJACENT ranges only (earlier operand first), carry odd
partials, never overwrite a slot that the same level still reads, write the
final prefix to `left` and suffix to `right`, take the P, p-only form exactly
when the later operand ends at the real terminal (rank R - 1), and finish in
max(ceil(log2 r), ceil(log2(R - 1 - r))) levels."""
import ctypes as C
import math

import pytest


def _lib():
    from pdplqr._lib import lib

    L = lib()
    L.pdplqr_debug_rank_tree.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.pdplqr_debug_rank_tree.restype = C.c_int
    return L


def _clog2(x):
    return 0 if x <= 1 else math.ceil(math.log2(x))


@pytest.mark.parametrize("R", list(range(1, 18)))
def test_rank_tree_plan_reduces_prefix_and_suffix(R):
    L = _lib()
    out = (C.c_int * 6)()
    for r in range(R):
        prev = {}  # level > 0 inputs: slot -> (lo, hi) rank range
        final = {}
        level = 0
        while True:
            per = L.pdplqr_debug_rank_tree(R, r, level, 0, out)
            if per == 0:
                break
            cur, reads = {}, set()
            for q in range(per):
                assert L.pdplqr_debug_rank_tree(R, r, level, q, out) == per
                suf, carry, fcf, a, b, dst = list(out)
                rng = (lambda i: (i, i)) if level == 0 else (lambda i: prev[i])
                ra = rng(a)
                reads.add(a)
                if carry:
                    res = ra
                else:
                    rb = rng(b)
                    reads.add(b)
                    assert ra[1] + 1 == rb[0], (R, r, level, q)
                    res = (ra[0], rb[1])
                    assert bool(fcf) == (rb[1] != R - 1), (R, r, level, q)
                    assert not (not fcf and not suf)
                if dst < 0:
                    key = "right" if suf else "left"
                    assert key not in final
                    final[key] = res
                else:
                    assert dst not in cur
                    cur[dst] = res
            if level > 0:  # outputs go to the other ping-pong buffer; inputs were all read
                assert reads <= set(prev)
            prev = cur
            level += 1
        assert level == max(_clog2(r), _clog2(R - 1 - r)), (R, r, level)
        if r >= 2:
            assert final["left"] == (0, r - 1)
        else:
            assert "left" not in final
        if R - 1 - r >= 2:
            assert final["right"] == (r + 1, R - 1)
        else:
            assert "right" not in final
