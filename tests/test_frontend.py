"""Front-end (matrix generation, nested dissection, symbolic factorization,
2D block-cyclic distribution) produces LUstructs in the reference layout."""
import numpy as np
import pytest

import cases
from superlu_dist_amd.frontend import (STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Csc, Symbolic,
                                       nd_order)


@pytest.mark.parametrize("kind,nx,ny,nz,nnb", [(STENCIL_2D5, 7, 5, 1, 5), (STENCIL_3D7, 4, 5, 6, 7),
                                               (STENCIL_3D27, 4, 4, 3, 27)])
def test_stencil_symmetric_and_degree(kind, nx, ny, nz, nnb):
    A = Csc.stencil(kind, nx, ny, nz)
    D = A.to_dense()
    assert np.array_equal(D, D.T)
    assert (np.count_nonzero(D, axis=0) <= nnb).all()
    assert D[0, 0] == {0: 4.0, 1: 6.0, 2: 26.0}[kind]


@pytest.mark.parametrize("dims", [(10, 10, 1), (6, 7, 8), (1, 1, 1), (33, 2, 1)])
def test_nd_is_a_permutation(dims):
    p = nd_order(*dims)
    assert np.array_equal(np.sort(p), np.arange(np.prod(dims)))


def test_symbolic_supernodes_partition_columns():
    A = Csc.stencil(STENCIL_3D7, 9, 9, 9)
    S = Symbolic(A, nd_order(9, 9, 9), relax=20, maxsup=32)
    w = np.diff(S.xsup)
    assert S.xsup[0] == 0 and S.xsup[-1] == A.n and (w >= 1).all() and (w <= 32).all()
    assert np.array_equal(S.supno[S.xsup[:-1]], np.arange(S.nsupers))


@pytest.mark.parametrize("grid", [(1, 1), (2, 3)])
def test_distribution_reassembles_permuted_matrix(grid):
    """Every entry of P A P^T lands in exactly one rank's L or U storage."""
    A = Csc.stencil(STENCIL_2D5, 9, 9, 1)
    S = Symbolic(A, nd_order(9, 9, 1), relax=6, maxsup=8)
    B = A.permuted(S.perm_c).to_dense()
    pr, pc = grid
    R = np.zeros_like(B)
    xs = S.xsup
    for r in range(pr):
        for c in range(pc):
            lu = S.distribute(pr, pc, r, c)
            for ljb in range(lu.nlc):
                if lu.Loff[ljb] < 0:
                    continue
                jb = ljb * pc + c
                idx = lu.Lidx[lu.Loff[ljb]:]
                nb, ld = idx[0], idx[1]
                vals = lu.Lval[lu.Lvoff[ljb]:lu.Lvoff[ljb] + ld * (xs[jb + 1] - xs[jb])]
                vals = vals.reshape(xs[jb + 1] - xs[jb], ld).T
                p, rs = 2, 0
                for _ in range(nb):
                    gb, nr = idx[p], idx[p + 1]
                    assert gb % pr == r
                    rows = idx[p + 2:p + 2 + nr]
                    R[np.ix_(rows, np.arange(xs[jb], xs[jb + 1]))] += vals[rs:rs + nr]
                    rs += nr
                    p += 2 + nr
            for lb in range(lu.nlr):
                if lu.Uoff[lb] < 0:
                    continue
                gb = lb * pr + r
                idx = lu.Uidx[lu.Uoff[lb]:]
                nb = idx[0]
                v = lu.Uval[lu.Uvoff[lb]:]
                p, q = 3, 0
                for _ in range(nb):
                    jb = idx[p]
                    assert jb % pc == c and jb > gb
                    for cc in range(xs[jb + 1] - xs[jb]):
                        fst = idx[p + 2 + cc]
                        seg = xs[gb + 1] - fst
                        R[fst:xs[gb + 1], xs[jb] + cc] += v[q:q + seg]
                        q += seg
                    p += 2 + xs[jb + 1] - xs[jb]
    assert np.array_equal(R, B)


def test_bufmax_and_comm_schedule_consistent():
    A, S, lus = cases.distribute("lap3d_10_2x4_small_d")
    for lu in lus:
        assert (lu.bufmax == lus[0].bufmax).all()
        assert lu.ToRecv.min() >= 0 and lu.ToRecv.max() <= 2
        tsr = lu.to_sendr()
        assert set(np.unique(tsr)) <= {-1, 1}


@pytest.mark.parametrize("dims", [(12, 12, 12), (9, 11, 7)])
def test_multichild_partition_holds_all_fill(dims):
    """Symbolic(multichild=True) on the library's METIS_NodeND ordering (the
    bench's --ordering graph): fewer supernodes than the default partition,
    and a structure that holds every fill entry -- the oracle factorization
    on it solves A x = b to backward error ~eps (a missing fill position
    would drop an update and spoil the solution).  CPU only."""
    import pyoracle
    from lusolve import backward_error, solve_1x1
    from superlu_dist_amd.symbolic import at_plus_a, metis_nodend
    A = Csc.stencil(STENCIL_3D7, *dims)
    cp, ri, _ = A.arrays()
    perm = metis_nodend(A.n, *at_plus_a(A.n, cp, ri))[0]
    S0 = Symbolic(A, perm, 60, 256)
    S = Symbolic(A, perm, 60, 256, multichild=True)
    assert S.nsupers <= S0.nsupers
    lu = S.distribute()
    o = pyoracle.oracle_factor([lu], 1, 1, A.n, False, cases.anorm(A))
    assert o["info"] == 0
    xt = np.random.default_rng(2).standard_normal(A.n)
    B = A.permuted(S.perm_c)
    bcp, bri, bv = B.arrays()
    b = np.zeros(A.n)
    for j in range(A.n):
        b[bri[bcp[j]:bcp[j + 1]]] += bv[bcp[j]:bcp[j + 1]] * xt[j]
    x = solve_1x1(lu, b)
    assert backward_error(A, S.perm_c, x, b) < 1e-14
