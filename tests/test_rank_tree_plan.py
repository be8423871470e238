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


@pytest.mark.parametrize("S", list(range(2, 70)))
def test_sklansky_scan_plan_builds_every_suffix(S):
    """The suffix scan's Sklansky rounds (scan_round_operands through the hook
    pdplqr_debug_scan_round): the first round (sk = 1, elements -> buffer)
    writes every entry once -- the pair combines in the first S // 2 blocks,
    the copies after them -- and each later round (sk = 2, in place) combines
    entry i with an entry j holding the adjacent range, so after ceil(log2 S)
    rounds entry i covers segments [i, S - 1]."""
    L = _lib()
    L.pdplqr_debug_scan_round.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.pdplqr_debug_scan_round.restype = C.c_int
    out = (C.c_int * 2)()
    cov = {}
    per = L.pdplqr_debug_scan_round(S, 1, 1, 0, out)
    assert per == S
    for q in range(per):
        L.pdplqr_debug_scan_round(S, 1, 1, q, out)
        i, j = out[0], out[1]
        assert i not in cov
        assert (j >= 0) == (q < S // 2)  # combines first
        cov[i] = (i, i) if j < 0 else (i, j)
        if j >= 0:
            assert j == i + 1
    assert sorted(cov) == list(range(S))
    d = 2
    while d < S:
        per = L.pdplqr_debug_scan_round(S, d, 2, 0, out)
        new = dict(cov)
        for q in range(per):
            L.pdplqr_debug_scan_round(S, d, 2, q, out)
            i, j = out[0], out[1]
            if i < 0:
                continue
            assert cov[i][1] + 1 == j, (S, d, q)  # adjacent ranges, earlier operand first
            new[i] = (cov[i][0], cov[j][1])
        cov = new
        d *= 2
    assert all(cov[i] == (i, S - 1) for i in range(S)), S


@pytest.mark.parametrize("n", [4, 12, 16, 24, 32, 40, 100])
def test_map_radix_takes_the_fewest_rounds(n):
    """map_radix (the per-solve radix of the boundary-map composition,
    k_map_scanR): the fewest rounds its kernel's largest radix allows (17 for
    n <= 16, 4 for 24 x 24 maps and the wide / XL kernels), then the smallest
    radix with that many rounds; every round count covers J entries."""
    L = _lib()
    L.pdplqr_debug_map_radix.argtypes = [C.c_int, C.c_int]
    L.pdplqr_debug_map_radix.restype = C.c_int
    rmax = 17 if n <= 16 else 4

    def rounds(R, J):
        r, d = 0, 1
        while d < J:
            d *= R
            r += 1
        return r

    for J in list(range(2, 300)) + [411, 513, 1025, 4097]:
        R = L.pdplqr_debug_map_radix(n, J)
        if n > 32:  # the wide / XL composition kernels run radix-4 rounds only
            assert R == 4, (n, J, R)
            continue
        assert 2 <= R <= rmax, (n, J, R)
        assert rounds(R, J) == rounds(rmax, J), (n, J, R)
        assert R == 2 or rounds(R - 1, J) > rounds(R, J), (n, J, R)
