"""Engine-side supernode amalgamation on process grids (csrc/amalg.h,
"grids"), on the CPU: every rank of a Pr x Pc grid in one process
(GridAmalgamation, csrc/amalg_api.cpp slu_gamalg_*), the same phases the
grid plan runs per rank with its transport between them.

* the coarse partition is coarser than the caller's and sums the caller
  partition's algorithmic flops exactly as the 1x1 amalgamation does;
* expand (pack -> all-to-all -> unpack) then compress gives back every
  caller value bit for bit;
* the oracle's grid factorization of the coarse LUstructs, compressed into
  every rank's caller layout, equals the oracle's grid factorization of the
  caller's LUstructs (stencils d / s / z on 1x2 .. 2x4);
* on the reference's own grid LUstructs (tests/golden/refdump_*: MC64 row
  permutations, unsymmetric structures) the compressed coarse factors match
  the REFERENCE's factors, info included.
"""
import numpy as np
import pytest

import pyoracle
from refdump import Fixture
from superlu_dist_amd.frontend import (STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Amalgamation, Csc,
                                       GridAmalgamation, Symbolic, nd_order)

TOL = {0: 1e-12, 1: 1e-5, 2: 1e-12}


def _case(kind, dims, dtype):
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), 60, 256, reference=True)
    colptr, _, val = A.arrays()
    an = float(np.add.reduceat(np.abs(val), colptr[:-1]).max())
    return A, S, an


def _rel(pairs):
    """normwise-max relative difference; a, b may each carry the spare
    trailing element of the LUstruct value arrays (compared over the
    values both hold)"""
    worst = 0.0
    for (L, U), (Lr, Ur) in pairs:
        for a, b in ((L, Lr), (U, Ur)):
            k = min(len(a), len(b)) - (1 if len(a) == len(b) else 0)
            if k > 0:
                d = np.abs(a[:k].astype(np.complex128) - b[:k].astype(np.complex128)).max()
                worst = max(worst, d / max(np.abs(b[:k]).max(), 1e-300))
    return worst


GRID_CASES = [
    (STENCIL_3D7, (12, 12, 12), 0, (2, 2)),
    (STENCIL_3D7, (16, 16, 16), 0, (2, 4)),
    (STENCIL_3D7, (14, 14, 14), 0, (3, 2)),
    (STENCIL_3D7, (10, 10, 10), 0, (1, 3)),
    (STENCIL_2D5, (40, 40, 1), 0, (2, 1)),
    (STENCIL_3D27, (10, 10, 10), 1, (2, 2)),
    (STENCIL_3D7, (10, 10, 10), 2, (1, 2)),
]


@pytest.mark.parametrize("kind,dims,dtype,grid", GRID_CASES)
def test_grid_amalgamation_roundtrip_and_flops(kind, dims, dtype, grid):
    A, S, _ = _case(kind, dims, dtype)
    pr, pc = grid
    lus = [S.distribute(pr, pc, r, c) for r in range(pr) for c in range(pc)]
    G = GridAmalgamation(lus, pr, pc)
    one = Amalgamation(S.distribute())
    assert G.ns1 == S.nsupers and G.ns2 < G.ns1
    # chains never cross an analysis range end: at most P - 1 more groups
    assert one.ns2 <= G.ns2 <= one.ns2 + pr * pc - 1
    assert G.flops() == pytest.approx(one.flops(), rel=1e-12)
    rng = np.random.default_rng(7)
    for lu in lus:
        lu.Lval[:] = rng.standard_normal(lu.Lval.size)
        lu.Uval[:] = rng.standard_normal(lu.Uval.size)
    G.expand()
    outs = [(np.zeros_like(lu.Lval), np.zeros_like(lu.Uval)) for lu in lus]
    G.compress(outs)
    for (L, U), lu in zip(outs, lus):
        np.testing.assert_array_equal(L[:-1], lu.Lval[:-1])
        np.testing.assert_array_equal(U[:-1], lu.Uval[:-1])
    # every coarse position that no caller value maps to is zero
    nz = sum(np.count_nonzero(m.Lval) + np.count_nonzero(m.Uval) for m in G.merged)
    assert nz == sum(np.count_nonzero(lu.Lval[:-1]) + np.count_nonzero(lu.Uval[:-1]) for lu in lus)


@pytest.mark.parametrize("kind,dims,dtype,grid", GRID_CASES)
def test_grid_amalgamation_factors_match_oracle(kind, dims, dtype, grid):
    A, S, an = _case(kind, dims, dtype)
    pr, pc = grid
    lus = [S.distribute(pr, pc, r, c) for r in range(pr) for c in range(pc)]
    ref = [S.distribute(pr, pc, r, c) for r in range(pr) for c in range(pc)]
    G = GridAmalgamation(lus, pr, pc)
    G.expand()
    o1 = pyoracle.oracle_factor(G.merged, pr, pc, A.n, False, an)
    o2 = pyoracle.oracle_factor(ref, pr, pc, A.n, False, an)
    assert o1["info"] == o2["info"] == 0
    outs = [(np.zeros_like(lu.Lval), np.zeros_like(lu.Uval)) for lu in lus]
    G.compress(outs)
    err = _rel(zip(outs, [(r.Lval, r.Uval) for r in ref]))
    assert err < TOL[dtype], err


REFDUMP_GRIDS = ["big_2x2_d", "big_1x2_s", "cd2d_24_2x2_d", "cd2d_20_2x1_z", "g20_2x3_small_d",
                 "lap3d_12_2x2_d", "cg20_2x2_z", "zeropiv2_2x2_d"]


@pytest.mark.parametrize("name", REFDUMP_GRIDS)
def test_grid_amalgamation_on_reference_lustructs(name):
    """The reference's own pddistribute output on its grid; the coarse
    factors (oracle), compressed, against the reference pdgstrf's factors."""
    fx = Fixture(name)
    pr, pc = fx.pr, fx.pc
    lus = fx.lus("pre")
    G = GridAmalgamation(lus, pr, pc)   # (unsymmetric structures stay unmerged)
    G.expand()
    o = pyoracle.oracle_factor(G.merged, pr, pc, fx.n, fx.replace_tiny, fx.anorm)
    assert o["info"] == fx.info
    assert o["tiny"] == fx.tiny
    if fx.info:
        return
    outs = [(np.zeros_like(lu.Lval), np.zeros_like(lu.Uval)) for lu in lus]
    G.compress(outs)
    err = _rel(zip(outs, fx.ref_factors()))
    assert err < TOL[fx.dtype], err
