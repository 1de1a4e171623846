"""Engine-side supernode amalgamation (csrc/amalg.h), on the CPU: the coarse
LUstruct the plan factors instead of the reference's fine partition, and the
expand / compress programs between the two layouts.

* expand then compress gives back every original value bit for bit;
* the oracle's factorization of the coarse LUstruct, compressed into the
  original layout, equals the oracle's factorization of the original within
  the parity tolerance (structural zeros stay exact zeros);
* on the reference's own LUstructs (tests/golden/refdump_*, 1x1) the
  compressed coarse factors match the REFERENCE's factors.
"""
import glob
import os
import sys

import numpy as np
import pytest

import pyoracle
from refdump import Fixture
from superlu_dist_amd.frontend import (STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Amalgamation, Csc,
                                       Symbolic, nd_order)

TOL = {0: 1e-12, 1: 1e-5, 2: 1e-12}
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _stencil_lu(kind, dims, dtype):
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), 60, 256, reference=True)
    colptr, _, val = A.arrays()
    an = float(np.add.reduceat(np.abs(val), colptr[:-1]).max())
    return S.distribute(1, 1, 0, 0), A.n, an


CASES = [(STENCIL_3D7, (12, 12, 12), 0), (STENCIL_3D7, (16, 16, 16), 0),
         (STENCIL_2D5, (40, 40, 1), 0), (STENCIL_3D27, (10, 10, 10), 1),
         (STENCIL_3D7, (10, 10, 10), 2)]


@pytest.mark.parametrize("kind,dims,dtype", CASES)
def test_expand_compress_roundtrip(kind, dims, dtype):
    lu, n, _ = _stencil_lu(kind, dims, dtype)
    am = Amalgamation(lu)
    assert am.ns2 < am.ns1 and am.groups > 0
    am.expand()
    L, U = np.zeros_like(lu.Lval), np.zeros_like(lu.Uval)
    am.compress(L, U)
    np.testing.assert_array_equal(L[:-1], lu.Lval[:-1])
    np.testing.assert_array_equal(U[:-1], lu.Uval[:-1])
    # every merged position that no original value maps to is zero
    nz = np.count_nonzero(am.merged.Lval) + np.count_nonzero(am.merged.Uval)
    assert nz == np.count_nonzero(lu.Lval) + np.count_nonzero(lu.Uval)


@pytest.mark.parametrize("kind,dims,dtype", CASES)
def test_amalgamated_factors_match_oracle(kind, dims, dtype):
    lu, n, an = _stencil_lu(kind, dims, dtype)
    ref, _, _ = _stencil_lu(kind, dims, dtype)
    am = Amalgamation(lu)
    am.expand()
    o1 = pyoracle.oracle_factor([am.merged], 1, 1, n, False, an)
    o0 = pyoracle.oracle_factor([ref], 1, 1, n, False, an)
    assert o1["info"] == o0["info"] == 0
    # the plan reports the original partition's work, the oracle's accounting
    assert abs(am.flops() - o0["flops"]) <= 1e-9 * o0["flops"] + 10
    L, U = np.zeros_like(lu.Lval), np.zeros_like(lu.Uval)
    am.compress(L, U)
    err = max(_rel(L[:-1], ref.Lval[:-1]), _rel(U[:-1], ref.Uval[:-1]))
    assert err < TOL[dtype], err
    assert am.ns2 < am.ns1


REFDUMP_1X1 = sorted(os.path.basename(p)[len("refdump_"):-4]
                     for p in glob.glob(os.path.join(GOLDEN, "refdump_*_1x1_*.npz")))


@pytest.mark.parametrize("name", REFDUMP_1X1)
def test_amalgamated_reference_lustructs(name):
    """The reference's own LUstructs (MC64 row permutations, unsymmetric
    structures: those supernodes stay as they are)."""
    fx = Fixture(name)
    lu = fx.lu(0, "pre")
    try:
        am = Amalgamation(lu)
    except RuntimeError as e:
        assert "nothing merges" in str(e)
        pytest.skip("no chain qualifies")
    am.expand()
    o = pyoracle.oracle_factor([am.merged], 1, 1, fx.n, fx.replace_tiny, fx.anorm)
    assert o["tiny"] == fx.tiny
    assert o["info"] == fx.info
    L, U = np.zeros_like(lu.Lval), np.zeros_like(lu.Uval)
    am.compress(L, U)
    post = fx.lu(0, "post")
    if o["info"] == 0:
        err = max(_rel(L[:-1], post.Lval[:-1]), _rel(U[:-1], post.Uval[:-1]))
        assert err < TOL[fx.dtype], err


@pytest.mark.parametrize("kind,dims,dtype", CASES)
def test_coarse_symbolic_is_the_engine_amalgamation(kind, dims, dtype):
    """Symbolic(reference=True, coarse=True) lays out exactly the coarse
    LUstruct a 1x1 plan factors internally (structure and values bit for
    bit), and keeps the reference partition's work for the rate."""
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    p = nd_order(*dims)
    fine = Symbolic(A, p, 60, 256, reference=True)
    coarse = Symbolic(A, p, 60, 256, reference=True, coarse=True)
    am = Amalgamation(fine.distribute(1, 1, 0, 0))
    am.expand()
    lu = coarse.distribute(1, 1, 0, 0)
    assert coarse.nsupers == am.ns2 and coarse.ref_flops()["nsupers"] == fine.nsupers
    np.testing.assert_array_equal(coarse.xsup, am.merged.xsup)
    for a, b in ((lu.Lidx, am.merged.Lidx), (lu.Loff, am.merged.Loff), (lu.Uoff, am.merged.Uoff)):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(lu.Lval[:am.lval2], am.merged.Lval[:am.lval2])
    np.testing.assert_array_equal(lu.Uval[:am.uval2], am.merged.Uval[:am.uval2])
    # U index: the same blocks and segments (the distribute writes the -1 end marker)
    assert abs(lu.Uidx.size - am.merged.Uidx.size) <= 1
    assert abs(coarse.ref_flops()["total"] - am.flops()) <= 1e-9 * am.flops()


def test_coarse_grid_distribution_matches_1x1():
    """The coarse partition on a 2x2 grid (the bench's N > 1 LUstructs):
    the oracle's grid factorization equals its 1x1 one, block by block."""
    A = Csc.stencil(STENCIL_3D7, 12, 12, 12)
    S = Symbolic(A, nd_order(12, 12, 12), 60, 256, reference=True, coarse=True)
    one = S.distribute(1, 1, 0, 0)
    pyoracle.oracle_factor([one], 1, 1, A.n, False, 12.0)
    lus = [S.distribute(2, 2, r // 2, r % 2) for r in range(4)]
    pyoracle.oracle_factor(lus, 2, 2, A.n, False, 12.0)
    c = pyoracle.compare_blocksums(pyoracle.blocksums(one),
                                   np.concatenate([pyoracle.blocksums(lu) for lu in lus]))
    assert c["match"] and c["rel_err"] <= 1e-13, c


@pytest.mark.parametrize("kind,dims,dtype", CASES)
def test_reference_symbolic_work_is_the_oracle_accounting(kind, dims, dtype):
    """Symbolic(reference=True).ref_flops(): the reference partition's work
    (bench.py's rate) equals the oracle's count on that LUstruct."""
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), 60, 256, reference=True)
    lu = S.distribute(1, 1, 0, 0)
    o = pyoracle.oracle_factor([lu], 1, 1, A.n, False, 1.0)
    f = S.ref_flops()
    assert f["nsupers"] == S.nsupers
    assert abs(f["total"] - o["flops"]) <= 1e-9 * o["flops"] + 10
