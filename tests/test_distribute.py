"""Structural pddistribute (csrc/distribute.cpp) against
the reference's own: for every reference-dumped fixture (tests/golden/
refdump_*, made by oracle/_ref/ref_dump from the reference's p?gssvx), the
symbolic factorization is recomputed with the reference-exact symbfact and
distributed onto each rank of the fixture's grid; index arrays, block order,
values, ToRecv / ToSendD / ToSendR and bufmax must equal what the reference's
pddistribute left, bit for bit.  CPU only.

A in the LUstruct's coordinates is read off the fixture's pre-factor
LUstructs (lusolve.lu_coords_matrix_from_lus), joined with the pattern of the
original matrix file (explicit zeros; tests/golden/matrices) and the diagonal
(the reference's A always has it, symbfact aborts otherwise).  Within each
column the rows are put in the order pdgssvx's global copy GA has them --
ascending original row, relabelled by perm_r and perm_c (pdCompRow_loc_to_
CompCol_global, SRC/pdutil.c:79-195; SRC/pdgssvx.c:801-802, 1050-1058) --
because symbfact's depth-first search, and with it the order of the L
subscripts, follows that order.  The fixture's own xsup / supno are the first
check of that reconstruction.
"""
import glob
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from lusolve import lu_coords_matrix_from_lus
from refdump import Fixture
from superlu_dist_amd import symbolic as sy
from superlu_dist_amd.frontend import LUStruct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = sorted(os.path.basename(p)[len("refdump_"):-4]
               for p in glob.glob(os.path.join(GOLDEN, "refdump_*.npz")))


def with_diagonal(n, cp, ri, v):
    """A's CSC with an explicit (zero) diagonal entry added where missing."""
    cols = np.repeat(np.arange(n), np.diff(cp))
    has = np.zeros(n, bool)
    has[cols[ri == cols]] = True
    miss = np.nonzero(~has)[0]
    r = np.concatenate([ri, miss])
    c = np.concatenate([cols, miss])
    vv = np.concatenate([v, np.zeros(len(miss), v.dtype)])
    o = np.lexsort((r, c))
    cp2 = np.zeros(n + 1, np.int64)
    np.add.at(cp2, c[o] + 1, 1)
    return np.cumsum(cp2), r[o].astype(np.int64), vv[o]


def lu_coords_matrix(fx):
    """CSC of A in the LUstruct's coordinates (values from the pre-factor
    LUstructs, pattern also from the matrix file), rows of each column in
    GA's order (ascending original row)."""
    n = fx.n
    cp, ri, v = with_diagonal(n, *lu_coords_matrix_from_lus(fx.lus("pre"), fx.pr, fx.pc))
    perm_r, perm_c = fx.arr(0, "perm_r"), fx.arr(0, "perm_c")
    src = fx.meta["matrix"]
    if src.startswith("file:"):          # explicit zeros of the file join the pattern
        from superlu_dist_amd.hbio import read_hb
        _, fcp, fri, _, _ = read_hb(os.path.join(GOLDEN, "matrices", src[5:]))
        fcol = np.repeat(np.arange(n), np.diff(fcp))
        cols = np.repeat(np.arange(n), np.diff(cp))
        key = np.concatenate([cols * n + ri, perm_c[fcol] * n + perm_c[perm_r[fri]]])
        keys, first = np.unique(key, return_index=True)
        vals = np.concatenate([v, np.zeros(len(fri), v.dtype)])[first]
        cols, ri, v = keys // n, keys % n, vals
        cp = np.zeros(n + 1, np.int64)
        np.add.at(cp, cols + 1, 1)
        cp = np.cumsum(cp)
    orig = np.empty(n, np.int64)          # LUstruct row -> original row
    orig[perm_c[perm_r]] = np.arange(n)
    cols = np.repeat(np.arange(n), np.diff(cp))
    o = np.lexsort((orig[ri], cols))
    return cp, ri[o].astype(np.int64), v[o]


def reference_symbolic(fx):
    """(CSC of A in LU coordinates, reference-exact Glu) for the fixture."""
    cp, ri, v = lu_coords_matrix(fx)
    r0 = fx.meta["ranks"][0]
    co = sy.sp_colorder(fx.n, fx.n, cp, ri, np.arange(fx.n), colperm=sy.MY_PERMC)
    # the LUstruct's coordinates are already postordered: the post-pass keeps them
    assert np.array_equal(co.perm_c, np.arange(fx.n))
    S = sy.symbfact(fx.n, fx.n, co.colbeg, co.colend, sy.relabel_rows(ri, co.perm_c), co.etree,
                    r0["relax"], r0["maxsup"])
    return (cp, ri, v), S


def _blocks_L(lu, Lidx, Loff, Lval, Lvoff, ljb, w):
    """(index array, values) of local L block column ljb from flat arrays."""
    ix = Lidx[Loff[ljb]:]
    p = 2
    for _ in range(int(ix[0])):
        p += 2 + int(ix[p + 1])
    ln = p
    return ix[:ln], Lval[Lvoff[ljb]:Lvoff[ljb] + int(ix[1]) * w]


@pytest.mark.parametrize("name", NAMES)
def test_distribute_matches_reference_pddistribute(name):
    fx = Fixture(name)
    (cp, ri, v), S = reference_symbolic(fx)
    np.testing.assert_array_equal(S.xsup, fx.arr(0, "xsup"))
    np.testing.assert_array_equal(S.supno[:fx.n], fx.arr(0, "supno")[:fx.n])
    xs = S.xsup
    for p in range(fx.nranks):
        myrow, mycol = p // fx.pc, p % fx.pc
        lu = LUStruct.from_glu(S, cp, ri, v, fx.dtype, fx.pr, fx.pc, myrow, mycol)
        ref = fx.lu(p, "pre")
        assert lu.nlc == ref.nlc and lu.nlr == ref.nlr
        for ljb in range(lu.nlc):
            assert (lu.Loff[ljb] < 0) == (ref.Loff[ljb] < 0), (p, ljb)
            if lu.Loff[ljb] < 0:
                continue
            w = int(xs[ljb * fx.pc + mycol + 1] - xs[ljb * fx.pc + mycol])
            mi, mv = _blocks_L(lu, lu.Lidx, lu.Loff, lu.Lval, lu.Lvoff, ljb, w)
            ri_, rv = _blocks_L(ref, ref.Lidx, ref.Loff, ref.Lval, ref.Lvoff, ljb, w)
            np.testing.assert_array_equal(mi, ri_, err_msg=f"rank {p} L column {ljb} index")
            np.testing.assert_array_equal(mv, rv, err_msg=f"rank {p} L column {ljb} values")
        for lb in range(lu.nlr):
            assert (lu.Uoff[lb] < 0) == (ref.Uoff[lb] < 0), (p, lb)
            if lu.Uoff[lb] < 0:
                continue
            mi = lu.Uidx[lu.Uoff[lb]:]
            rr = ref.Uidx[ref.Uoff[lb]:]
            ln = int(rr[2])
            np.testing.assert_array_equal(mi[:ln], rr[:ln], err_msg=f"rank {p} U row {lb} index")
            assert mi[ln] == -1                                # the reference's end marker
            nv = int(rr[1])
            np.testing.assert_array_equal(lu.Uval[lu.Uvoff[lb]:lu.Uvoff[lb] + nv],
                                          ref.Uval[ref.Uvoff[lb]:ref.Uvoff[lb] + nv],
                                          err_msg=f"rank {p} U row {lb} values")
        np.testing.assert_array_equal(lu.ToRecv, fx.arr(p, "ToRecv"))
        np.testing.assert_array_equal(lu.ToSendD, fx.arr(p, "ToSendD"))
        np.testing.assert_array_equal(lu.to_sendr().ravel(), fx.arr(p, "ToSendR"))
        np.testing.assert_array_equal(lu.bufmax, fx.arr(p, "bufmax"))
        # the *_dat arrays are contiguous in local block order with one spare element
        assert lu.view.Lval_cnt == sum(int(lu.Lidx[o + 1]) * int(xs[j * fx.pc + mycol + 1] -
                                                                 xs[j * fx.pc + mycol])
                                       for j, o in enumerate(lu.Loff) if o >= 0) + 1


ASAN_DRV = os.path.join(ROOT, "oracle", "_ref", "distribute_destroy_asan")


@pytest.mark.skipif(not os.path.exists(ASAN_DRV) or not os.path.exists("/opt/conda/bin/mpiexec"),
                    reason="ASAN driver not built (make -C oracle asan)")
@pytest.mark.parametrize("nprocs,grid", [(1, (1, 1)), (4, (2, 2))])
@pytest.mark.parametrize("refill", [False, True])
@pytest.mark.parametrize("t,matrix", [("d", "g20.rua"), ("d", "big.rua"), ("s", "g20.rua"),
                                      ("z", "cg20.cua")])
def test_distribute_ownership_under_asan(t, matrix, refill, nprocs, grid):
    """The LUstruct this library's p?distribute builds is freed by the
    REFERENCE's p?Destroy_LU (SRC/pdutil.c:485, psutil.c:435, pzutil.c:483)
    without a bad free, double free or overflow: the reference's p?gssvx
    (nrhs = 0) around our p?distribute (and the SamePattern_SameRowPerm
    refill), our p?gstrf skipped (SUPERLU_MI355X_FACTOR_SKIP=1, no GPU), in
    a process built with AddressSanitizer (oracle/gen/distribute_destroy_main.c).
    With the s / z per-block allocation of commit 1947008 reverted this run
    aborts with 'attempting free on address which was not malloc()-ed'."""
    env = dict(os.environ, SUPERLU_MI355X_FACTOR_SKIP="1", ASAN_OPTIONS="detect_leaks=0",
               OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    args = ["-t", t, "-R", str(grid[0]), "-C", str(grid[1])] + (["-r"] if refill else [])
    cmd = ["/opt/conda/bin/mpiexec", "-n", str(nprocs), ASAN_DRV] + args + \
          [os.path.join(ROOT, "tests", "golden", "matrices", matrix)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-3000:]
    assert r.returncode == 0 and out.count(": OK") == nprocs, out[-3000:]
