"""Device-side value fill from A (slu_plan_set_a_pattern / slu_plan_fill_a,
csrc/fill.h; SURVEY 8(f) row 1, the SamePattern_SameRowPerm branch of
SRC/pddistribute.c:545-672).

Checker: the front-end's host distribution of the same matrix (the layout of
SRC/pddistribute.c), bit-exact -- the fill is a copy, no arithmetic.  Then the
filled storage is factored and compared with the reference's golden factors.
2D grids: tests/test_grid.py runs golden cases with every rank filling its
own storage from A.
"""
import numpy as np
import pytest

import cases
from superlu_dist_amd.engine import Plan
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order
from test_oracle import TOL, load_golden

pytestmark = pytest.mark.gpu


def _filled_plan(A, S):
    lu = S.distribute()
    p = Plan(lu)
    cp, ri, v = A.permuted(S.perm_c).arrays()
    p.set_a_pattern(cp, ri)
    p.fill_a(v)  # no upload: the device storage starts uninitialised
    return p, lu, (cp, ri, v)


@pytest.mark.parametrize("name", ["g20_1x1_d", "g20_1x1_small_d", "g20_1x1_s", "cg20_1x1_z",
                                  "lap3d_14_1x1_d", "lap2d_32_1x1_d", "st27_8_1x1_s",
                                  "helm3d_8_1x1_z"])
def test_fill_equals_host_distribute(name):
    A, perm, dtype, _, relax, maxsup, _ = cases.build(name)
    S = Symbolic(A, perm, relax, maxsup)
    p, lu, _ = _filled_plan(A, S)
    p.download()
    ref = S.distribute()
    assert np.array_equal(lu.Lval, ref.Lval) and np.array_equal(lu.Uval, ref.Uval)
    assert p.stats()["t_fill_ms"] > 0


@pytest.mark.parametrize("name", ["g20_1x1_d", "cg20_1x1_z", "lap3d_14_1x1_d", "st27_8_1x1_s"])
def test_fill_then_factor_matches_reference(name):
    meta, ref = load_golden(name)
    A, perm, dtype, _, relax, maxsup, tiny = cases.build(name)
    S = Symbolic(A, perm, relax, maxsup)
    p, lu, _ = _filled_plan(A, S)
    info, ntiny = p.factor(cases.anorm(A))
    p.download()
    assert info == meta["ref_info"] and ntiny == meta["ref_tiny"]
    err = cases.factor_error([lu], ref)
    assert err < TOL[dtype], err


def test_refill_new_values_same_pattern():
    """Refactor with new values of the same pattern (the reference's
    SamePattern_SameRowPerm use): after one factorization, refill the same
    plan with A' = 2A + I and factor again; the factors equal those of a fresh
    plan filled with A' (up to the order of atomic additions)."""
    A = Csc.stencil(STENCIL_3D7, 12, 12, 12)
    S = Symbolic(A, nd_order(12, 12, 12), 60, 256)
    p, lu, (cp, ri, v) = _filled_plan(A, S)
    assert p.factor(12.0) == (0, 0)
    v2 = 2.0 * v
    for j in range(A.n):
        sl = slice(cp[j], cp[j + 1])
        v2[sl][ri[sl] == j] += 1.0
    p.fill_a(v2)
    assert p.factor(25.0) == (0, 0)
    p.download()
    lu2 = S.distribute()
    q = Plan(lu2)
    q.set_a_pattern(cp, ri)
    q.fill_a(v2)
    assert q.factor(25.0) == (0, 0)
    q.download()
    for a, b in ((lu.Lval, lu2.Lval), (lu.Uval, lu2.Uval)):
        assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max()


def test_fill_duplicate_entry_keeps_last():
    A = Csc.stencil(STENCIL_3D7, 6, 6, 6)
    S = Symbolic(A, nd_order(6, 6, 6), 60, 256)
    p, lu, (cp, ri, v) = _filled_plan(A, S)
    j = 5
    at = cp[j + 1]  # append a duplicate of column j's first entry
    cp2 = cp.copy()
    cp2[j + 1:] += 1
    ri2 = np.insert(ri, at, ri[cp[j]])
    v2 = np.insert(v, at, 99.0)
    p.set_a_pattern(cp2, ri2)
    p.fill_a(v2)
    p.download()
    L2, U2 = lu.Lval.copy(), lu.Uval.copy()
    v3 = v.copy()
    v3[cp[j]] = 99.0
    p.set_a_pattern(cp, ri)
    p.fill_a(v3)
    p.download()
    assert np.array_equal(L2, lu.Lval) and np.array_equal(U2, lu.Uval)


def test_fill_rejects_entries_outside_the_structure():
    A = Csc.stencil(STENCIL_3D7, 6, 6, 6)
    S = Symbolic(A, nd_order(6, 6, 6), 60, 256)
    p, lu, (cp, ri, v) = _filled_plan(A, S)
    n = A.n
    with pytest.raises(RuntimeError, match="out of range"):
        bad = ri.copy()
        bad[0] = n
        p.set_a_pattern(cp, bad)
    rejected = 0
    for r in range(0, n, 7):  # column 0 against every 7th row: some are structural zeros
        cp2 = cp.copy()
        cp2[1:] += 1
        ri2 = np.insert(ri, cp[1], r)
        try:
            p.set_a_pattern(cp2, ri2)
        except RuntimeError as e:
            assert "outside" in str(e)
            rejected += 1
    assert rejected > 0
