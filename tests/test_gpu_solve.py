"""Device triangular solve with the HBM-resident factors (slu_plan_solve,
csrc/solve.h; SURVEY 8(f) row 2, the L/U sweeps of SRC/pdgstrs.c).

Checker: the host supernodal solve in tests/lusolve.py (scipy
solve_triangular per diagonal block, numpy panel updates) on the same
downloaded factors.  The device solve accumulates panel contributions with
atomics, so the summation order differs: tolerance is normwise relative
1e-12 fp64 / complex, 1e-4 fp32 (the solve amplifies the factor rounding by
the triangular condition numbers), plus the backward error of the result.
"""
import numpy as np
import pytest

from lusolve import backward_error, solve_1x1
from superlu_dist_amd.engine import Plan
from superlu_dist_amd.frontend import STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Csc, Symbolic, nd_order

pytestmark = pytest.mark.gpu

TOL = {0: 1e-12, 1: 1e-4, 2: 1e-12}
DT = {0: np.float64, 1: np.float32, 2: np.complex128}


def _rhs(A, perm, xt):
    B = A.permuted(perm)
    cp, ri, v = B.arrays()
    b = np.zeros(A.n, dtype=np.result_type(v, xt))
    for j in range(A.n):
        b[ri[cp[j]:cp[j + 1]]] += v[cp[j]:cp[j + 1]] * xt[j]
    return b


@pytest.mark.parametrize("kind,dims,dtype,relax,maxsup,nrhs", [
    (STENCIL_3D7, (12, 12, 12), 0, 60, 256, 1),
    (STENCIL_3D7, (16, 16, 16), 0, 4, 24, 3),     # narrow supernodes, many levels
    (STENCIL_3D7, (20, 20, 20), 0, 60, 320, 2),   # supernodes wider than 256
    (STENCIL_2D5, (40, 40, 1), 0, 60, 256, 1),
    (STENCIL_3D27, (10, 10, 10), 1, 60, 256, 2),
    (STENCIL_3D7, (10, 10, 10), 2, 60, 256, 2),
    (STENCIL_3D7, (12, 12, 12), 0, 60, 256, 10),  # batches of 8 + 2 right-hand sides
    (STENCIL_3D27, (8, 8, 8), 1, 60, 256, 9),
    (STENCIL_3D7, (8, 8, 8), 2, 60, 256, 5),      # complex: batches of 2
    # supernodes wider than 256 whose last 32-column panel starts in the upper
    # half of a wave (width 300 / 100: j0 % 64 == 32) -- complex and fp32
    (STENCIL_3D7, (20, 20, 20), 2, 60, 300, 3),
    (STENCIL_3D7, (20, 20, 20), 1, 60, 300, 3),
])
def test_device_solve_matches_host_solve(kind, dims, dtype, relax, maxsup, nrhs):
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), relax, maxsup)
    lu = S.distribute()
    p = Plan(lu)
    p.upload()
    assert p.factor(12.0) == (0, 0)
    p.download()
    rng = np.random.default_rng(7)
    xt = rng.standard_normal((A.n, nrhs))
    if dtype == 2:
        xt = xt + 1j * rng.standard_normal((A.n, nrhs))
    b = np.stack([_rhs(A, S.perm_c, xt[:, r]) for r in range(nrhs)], axis=1).astype(DT[dtype])
    x = p.solve(b)
    assert x.shape == b.shape and x.dtype == DT[dtype]
    for r in range(nrhs):
        xh = solve_1x1(lu, b[:, r])
        err = np.abs(x[:, r] - xh).max() / np.abs(xh).max()
        assert err < TOL[dtype], (r, err)
        berr = backward_error(A, S.perm_c, x[:, r].astype(xh.dtype), b[:, r])
        assert berr < (1e-5 if dtype == 1 else 1e-14), (r, berr)
    assert p.stats()["t_solve_ms"] > 0


def test_device_solve_backward_error_32():
    """Property at a size the host checker is slow on: backward error and
    forward error against the generating solution."""
    A = Csc.stencil(STENCIL_3D7, 32, 32, 32)
    S = Symbolic(A, nd_order(32, 32, 32), 60, 256)
    lu = S.distribute()
    p = Plan(lu)
    p.upload()
    assert p.factor(12.0) == (0, 0)
    xt = np.random.default_rng(3).standard_normal(A.n)
    b = _rhs(A, S.perm_c, xt)
    x = p.solve(b)
    assert backward_error(A, S.perm_c, x, b) < 1e-14
    assert np.abs(x - xt).max() / np.abs(xt).max() < 1e-10


def test_device_solve_empty_rhs():
    A = Csc.stencil(STENCIL_3D7, 6, 6, 6)
    S = Symbolic(A, nd_order(6, 6, 6), 60, 256)
    p = Plan(S.distribute())
    p.upload()
    assert p.factor(12.0) == (0, 0)
    x = p.solve(np.zeros((A.n, 0)))
    assert x.shape == (A.n, 0)
