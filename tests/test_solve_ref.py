"""The device value fill, solve and refinement pinned to the REFERENCE
(SURVEY 8(f) rows 1-2), on the 1x1 refdump fixtures: the reference's own
pddistribute output (pre-factor L/U values), its pdgstrs solution
(IterRefine = NOREFINE, x_norefine) and its pdgsrfs-refined solution (x,
berr), all from oracle/_ref/ref_dump running p?gssvx.

* CPU: the coordinate maps of pdgssvx (Pc Pr diag(R) A diag(C) Pc^T) applied
  to the reference's factors with a host supernodal solve reproduce the
  reference's x_norefine -- pins the test's own plumbing.
* GPU: slu_plan_fill_a on the fixture's A reproduces the reference's
  pddistribute values bit for bit; the device factorization of them, the
  device solve and the device refinement reproduce the reference's x within
  the accuracy the reference itself reaches (||x_ref - xtrue||), and the
  refined backward error is at the reference's level.
* GPU, 2D grids: the distributed device solve (lsum partial sums reduced
  along process rows to the diagonal owners, solved pieces down the process
  columns, as pdgstrs) on the engine's factors of the reference's grid
  LUstructs (values filled on the device from the reference's A)
  reproduces the reference's pdgstrs x_norefine on the same grid, and the
  grid refinement (residual from each rank's entries of A, reduced to the
  owners, as pdgsmv) the reference's pdgsrfs x, berr and step count.
"""
import numpy as np
import pytest

from lusolve import from_lu_coords, lu_coords_matrix, solve_1x1, to_lu_coords
from refdump import Fixture, names

CASES = [n for n in names() if "_1x1_" in n and not n.startswith("zeropiv")]
EPS = {0: 2.2e-16, 1: 1.2e-7, 2: 2.2e-16}


def _rhs(fx):
    R = fx.z.get("r0_R")
    C = fx.z.get("r0_C")
    return fx.arr(0, "b"), R, C, fx.arr(0, "perm_r"), fx.arr(0, "perm_c")


def _close(x, xref, xtrue, dtype):
    """x agrees with the reference's x to the accuracy the reference has."""
    nx = np.abs(xref).max()
    ref_err = np.abs(xref - xtrue).max() / nx
    d = np.abs(x - xref).max() / nx
    return d, max(10 * ref_err, 50 * EPS[dtype])


@pytest.mark.parametrize("name", CASES)
def test_host_solve_of_reference_factors_is_reference_pdgstrs(name):
    fx = Fixture(name)
    lu = fx.lu(0, "post")
    b, R, C, pr, pc = _rhs(fx)
    y = solve_1x1(lu, to_lu_coords(b, pr, pc, R))
    x = from_lu_coords(y, pc, C)
    d, tol = _close(x, fx.arr(0, "x_norefine"), fx.arr(0, "xtrue"), fx.dtype)
    assert d < tol, (d, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_fill_solve_refine_match_reference(name):
    from superlu_dist_amd.engine import Plan
    fx = Fixture(name)
    lu = fx.lu(0, "pre")
    pre_L, pre_U = lu.Lval.copy(), lu.Uval.copy()
    lu.Lval[:] = np.nan        # the fill must produce every value itself
    lu.Uval[:] = np.nan
    p = Plan(lu, replace_tiny=fx.replace_tiny)
    cp, ri, v = lu_coords_matrix(fx)
    p.set_a_pattern(cp, ri)
    p.fill_a(v)
    p.download()
    # SamePattern_SameRowPerm refill == the reference's pddistribute, bit for bit
    np.testing.assert_array_equal(lu.Lval[:-1], pre_L[:-1])
    np.testing.assert_array_equal(lu.Uval[:-1], pre_U[:-1])
    info, tiny = p.factor(fx.anorm)
    assert (info, tiny) == (fx.info, fx.tiny)
    b, R, C, pr, pc = _rhs(fx)
    bl = to_lu_coords(b, pr, pc, R).astype(lu.Lval.dtype)
    y = p.solve(bl)
    x = from_lu_coords(y, pc, C)
    xtrue = fx.arr(0, "xtrue")
    d, tol = _close(x, fx.arr(0, "x_norefine"), xtrue, fx.dtype)
    assert d < tol, ("solve", d, tol)
    yr, berr, steps = p.refine(bl, y)
    xr = from_lu_coords(yr, pc, C)
    d, tol = _close(xr, fx.arr(0, "x"), xtrue, fx.dtype)
    assert d < tol, ("refine", d, tol)
    ref_berr = float(fx.arr(0, "berr")[0])
    assert berr[0] <= max(4 * ref_berr, 4 * EPS[fx.dtype]), (berr[0], ref_berr)
    assert abs(int(steps[0]) - fx.meta["ranks"][0]["refine_steps"]) <= 1


GRID_CASES = [n for n in names() if "_1x1_" not in n and not n.startswith("zeropiv")]


@pytest.mark.parametrize("name", GRID_CASES)
def test_grid_fixture_rhs_reassembles(name):
    """The per-rank pieces of the reference's distributed B / X put back
    together solve the reference's own factored system (host check)."""
    fx = Fixture(name)
    b, R, C, perm_r, perm_c, xnr, xtrue = fx.full_rhs()
    assert b.shape == xnr.shape == xtrue.shape == (fx.n,)
    d, tol = _close(xnr, xnr, xtrue, fx.dtype)
    assert d == 0 and np.isfinite(xnr).all()
    assert np.abs(xnr - xtrue).max() / np.abs(xtrue).max() < max(1e-6, 1e3 * EPS[fx.dtype])


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["bcast", "p2p"])
@pytest.mark.parametrize("name", GRID_CASES)
def test_gpu_grid_solve_matches_reference(name, transport, tmp_path):
    from gridrun import run_grid
    fx = Fixture(name)
    out = run_grid(f"refdump:{name}", fx.pr, fx.pc, tmp_path, device=0, solve=True,
                   transport=transport)
    _, _, _, _, _, xnr, xtrue = fx.full_rhs()
    xref = np.concatenate([fx.arr(p, "x") for p in sorted(range(fx.nranks),
                                                        key=lambda q: fx.meta["ranks"][q]["fst_row"])])
    ref_berr = float(fx.arr(0, "berr")[0])
    for p, o in enumerate(out):  # x comes back replicated on every rank
        assert int(o["info"]) == fx.info
        d, tol = _close(o["x"], xnr, xtrue, fx.dtype)
        assert d < tol, ("solve", p, d, tol)
        # refinement on the grid (pdgsrfs + the distributed residual of pdgsmv)
        d, tol = _close(o["xr"], xref, xtrue, fx.dtype)
        assert d < tol, ("refine", p, d, tol)
        assert o["berr"] <= max(4 * ref_berr, 4 * EPS[fx.dtype]), (o["berr"], ref_berr)
        assert abs(int(o["steps"]) - fx.meta["ranks"][0]["refine_steps"]) <= 1


@pytest.mark.parametrize("name", GRID_CASES)
def test_grid_solve_algorithm_reproduces_reference_pdgstrs(name):
    """The engine's distributed solve scheme (lusolve.solve_grid_sim: partial
    sums per process row, reduced to the diagonal owner; solved pieces down
    the owner's process column), run on the reference's own factors of its
    grid LUstructs, gives the reference's pdgstrs x_norefine (CPU)."""
    from lusolve import solve_grid_sim
    fx = Fixture(name)
    b, R, C, perm_r, perm_c, xnr, xtrue = fx.full_rhs()
    y = solve_grid_sim(fx.lus("post"), fx.pr, fx.pc, to_lu_coords(b, perm_r, perm_c, R))
    d, tol = _close(from_lu_coords(y, perm_c, C), xnr, xtrue, fx.dtype)
    assert d < tol, (d, tol)
