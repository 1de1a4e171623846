"""Device iterative refinement (slu_plan_refine; SURVEY 8(f) row 2, the
refinement loop of SRC/pdgsrfs.c:197-253) on the HBM-resident factors.

Checker: a numpy restatement of the same loop (host residual, host
supernodal solve from tests/lusolve.py on the downloaded factors).  The
residual sums run in a different order, so the stopping decision near eps
may differ by a step: the final solutions are compared within 1e-12
(fp64 / complex) / 1e-5 (fp32), and the returned berr against the
componentwise backward error of the returned x recomputed in extended
precision, within a few eps.
"""
import numpy as np
import pytest

from lusolve import solve_1x1
from superlu_dist_amd.engine import Plan
from superlu_dist_amd.frontend import STENCIL_3D7, STENCIL_3D27, Csc, Symbolic, nd_order

pytestmark = pytest.mark.gpu

EPS = {0: 2.0 ** -53, 1: 2.0 ** -24, 2: 2.0 ** -53}
DT = {0: np.float64, 1: np.float32, 2: np.complex128}


def _abs1(v):
    return np.abs(v.real) + np.abs(v.imag) if np.iscomplexobj(v) else np.abs(v)


def _berr(cp, ri, v, x, b, hi=np.longdouble):
    """componentwise backward error as SRC/pdgsrfs.c:213-230 (safe guards
    irrelevant here), residual accumulated in extended precision."""
    n = len(b)
    cplx = np.iscomplexobj(v)
    dt = np.clongdouble if cplx else hi
    r = np.array(b, dtype=dt)
    s = _abs1(np.asarray(b)).astype(hi)
    for j in range(n):
        sl = slice(cp[j], cp[j + 1])
        r[ri[sl]] -= v[sl].astype(dt) * dt(x[j])
        s[ri[sl]] += _abs1(v[sl]).astype(hi) * hi(_abs1(np.asarray(x[j])))
    return float(np.max(_abs1(r).astype(hi) / s))


def _host_refine(lu, cp, ri, v, b, x, eps):
    """numpy restatement of the pdgsrfs loop on the host factors."""
    n = len(b)
    lstres, count = 3.0, 0
    while True:
        r = np.array(b, dtype=np.result_type(v, x))
        s = _abs1(b).astype(np.float64)
        for j in range(n):
            sl = slice(cp[j], cp[j + 1])
            r[ri[sl]] -= v[sl] * x[j]
            s[ri[sl]] += _abs1(v[sl]) * _abs1(x[j])
        be = float(np.max(_abs1(r) / s))
        if not (be > eps and be * 2 <= lstres and count < 20):
            return x, be, count
        x = x + solve_1x1(lu, r).astype(x.dtype)
        lstres = be
        count += 1


@pytest.mark.parametrize("kind,dims,dtype,start", [
    (STENCIL_3D7, (12, 12, 12), 0, "solve"),
    (STENCIL_3D7, (10, 10, 10), 0, "zero"),     # x0 = 0: first step is the solve itself
    (STENCIL_3D27, (10, 10, 10), 1, "solve"),   # fp32 factors: refinement has work to do
    (STENCIL_3D7, (8, 8, 8), 2, "solve"),
])
def test_device_refine_matches_host_loop(kind, dims, dtype, start):
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), 60, 256)
    lu = S.distribute()
    p = Plan(lu)
    cp, ri, v = A.permuted(S.perm_c).arrays()
    p.set_a_pattern(cp, ri)
    p.fill_a(v)
    assert p.factor(12.0)[0] == 0
    p.download()
    rng = np.random.default_rng(11)
    xt = rng.standard_normal(A.n)
    if dtype == 2:
        xt = xt + 1j * rng.standard_normal(A.n)
    b = np.zeros(A.n, dtype=np.result_type(v, xt))
    for j in range(A.n):
        b[ri[cp[j]:cp[j + 1]]] += v[cp[j]:cp[j + 1]] * xt[j]
    b = b.astype(DT[dtype])
    x0 = p.solve(b) if start == "solve" else np.zeros_like(b)
    x, berr, steps = p.refine(b, x0)
    assert 0 <= steps[0] <= 20 and p.stats()["t_refine_ms"] > 0
    if start == "zero":
        assert steps[0] >= 1
    eps = EPS[dtype]
    # the device residual is summed in working precision: up to ~(row nnz + 1)
    # roundings relative to |A||x| + |b|
    tol_b = 2 * (int(np.diff(cp).max()) + 1) * eps
    assert abs(_berr(cp, ri, v, x, b) - berr[0]) <= tol_b
    assert berr[0] <= (1e-6 if dtype == 1 else 8 * eps), berr
    xh, bh, sh = _host_refine(lu, cp, ri, v, b, x0.copy(), eps)
    tol = 1e-5 if dtype == 1 else 1e-12
    assert np.abs(x - xh).max() / np.abs(xh).max() < tol
    if dtype == 1:  # fp32 factors: refinement reduces the error of the plain solve
        assert _berr(cp, ri, v, x, b) <= _berr(cp, ri, v, x0, b) + tol_b


def test_refine_needs_values():
    A = Csc.stencil(STENCIL_3D7, 6, 6, 6)
    S = Symbolic(A, nd_order(6, 6, 6), 60, 256)
    p = Plan(S.distribute())
    p.upload()
    assert p.factor(12.0) == (0, 0)
    with pytest.raises(RuntimeError, match="fill_a"):
        p.refine(np.ones(A.n), np.zeros(A.n))


def test_refine_reports_nonfinite_backward_error():
    """A NaN / Inf in x must surface in berr (SUPERLU_MAX passes NaN through,
    SRC/pdgsrfs.c:222-226), not look like convergence."""
    A = Csc.stencil(STENCIL_3D7, 6, 6, 6)
    S = Symbolic(A, nd_order(6, 6, 6), 60, 256)
    p = Plan(S.distribute())
    cp, ri, v = A.permuted(S.perm_c).arrays()
    p.set_a_pattern(cp, ri)
    p.fill_a(v)
    assert p.factor(12.0)[0] == 0
    b = np.ones(A.n)
    x0 = p.solve(b)
    x0[5] = np.nan
    _, berr, steps = p.refine(b, x0)
    assert not np.isfinite(berr[0]) and steps[0] == 0


def test_device_state_is_checked():
    """solve / refine only on factors of the values they describe."""
    A = Csc.stencil(STENCIL_3D7, 6, 6, 6)
    S = Symbolic(A, nd_order(6, 6, 6), 60, 256)
    p = Plan(S.distribute())
    cp, ri, v = A.permuted(S.perm_c).arrays()
    p.set_a_pattern(cp, ri)
    p.fill_a(v)
    with pytest.raises(RuntimeError, match="factor first"):
        p.solve(np.ones(A.n))
    assert p.factor(12.0)[0] == 0
    with pytest.raises(RuntimeError, match="already factored"):
        p.factor(12.0)
    p.fill_a(2 * v)                       # refilled, not factored
    with pytest.raises(RuntimeError, match="factor first"):
        p.refine(np.ones(A.n), np.zeros(A.n))
    assert p.factor(12.0)[0] == 0
    x, berr, _ = p.refine(np.ones(A.n), np.zeros(A.n))
    assert berr[0] < 1e-14
    p.upload()                            # values of unknown origin
    assert p.factor(12.0)[0] == 0
    with pytest.raises(RuntimeError, match="fill_a"):
        p.refine(np.ones(A.n), np.zeros(A.n))
