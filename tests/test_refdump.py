"""Parity on LUstructs built by the REFERENCE's own front-end.

tests/golden/refdump_*.npz hold, per rank, the LUstruct that the reference's
p?gssvx hands pdgstrf (equilibration, MC64 row permutation, MMD ordering,
unsymmetric symbfact, pddistribute's block layout; SRC/pdgssvx.c:718-1180)
and the reference factorization's output (oracle/gen/make_refdump.py).  The
engine gets those arrays verbatim (slu_lustruct_build), not our front-end's.

* CPU: the fixtures cover the input family (unsymmetric structure, MC64
  perm_r != identity, multi-rank grids); the oracle (C restatement)
  reproduces the reference's factors on them.
* GPU: the drop-in symbols pdgstrf / psgstrf / pzgstrf on every 1x1 fixture,
  and the engine on every grid fixture (host-staged transport), against the
  reference's factors, info and TinyPivots.
Tolerance (north star): normwise-max relative 1e-12 fp64 / complex, 1e-5 fp32.
"""
import numpy as np
import pytest

import cases
import pyoracle
from refdump import Fixture, names
from test_oracle import TOL

ALL = names()
ONE = [n for n in ALL if "_1x1_" in n]
GRIDS = [n for n in ALL if n not in ONE]


def _blocks(fx):
    """Global sets of L blocks (ib, k) and U blocks (k, jb) over all ranks."""
    xsup = fx.arr(0, "xsup")
    lblocks, ublocks = set(), set()
    for rank in range(fx.nranks):
        lu = fx.lu(rank)
        myrow, mycol = rank // fx.pc, rank % fx.pc
        for lk in range(lu.nlc):
            if lu.Loff[lk] >= 0:
                ix, p = lu.Lidx[lu.Loff[lk]:], 2
                for _ in range(int(ix[0])):
                    lblocks.add((int(ix[p]), lk * fx.pc + mycol))
                    p += 2 + int(ix[p + 1])
        for lk in range(lu.nlr):
            if lu.Uoff[lk] >= 0:
                ix, p = lu.Uidx[lu.Uoff[lk]:], 3
                for _ in range(int(ix[0])):
                    jb = int(ix[p])
                    ublocks.add((lk * fx.pr + myrow, jb))
                    p += 2 + int(xsup[jb + 1] - xsup[jb])
    return lblocks, ublocks


def test_fixture_family_covers_unsymmetric_and_row_permuted_inputs():
    """The input family SURVEY 8(a) a13 asks for: LUstructs with MC64 row
    permutations, structurally unsymmetric L/U block patterns, multi-rank."""
    assert len(ALL) >= 12
    blk_unsym = elem_unsym = rowperm = multi = 0
    for nm in ALL:
        fx = Fixture(nm)
        pr = fx.arr(0, "perm_r")
        rowperm += int(not np.array_equal(pr, np.arange(len(pr))))
        multi += int(fx.nranks > 1)
        lb, ub = _blocks(fx)
        blk_unsym += int(any((j, k) not in lb for (k, j) in ub) or
                         any((k, i) not in ub for (i, k) in lb if i != k))
        # element level: stored L entries below the diagonal blocks vs U entries
        w = np.diff(fx.arr(0, "xsup"))
        nl = sum(len(fx.arr(p, "pre_Lval")) for p in range(fx.nranks)) - int((w * w).sum())
        nu = sum(len(fx.arr(p, "pre_Uval")) for p in range(fx.nranks))
        elem_unsym += int(nl != nu)
    assert rowperm >= 3 and multi >= 6 and blk_unsym >= 2 and elem_unsym >= 3, \
        (rowperm, multi, blk_unsym, elem_unsym)


@pytest.mark.parametrize("name", ALL)
def test_oracle_matches_reference_on_reference_lustructs(name):
    """Pins the C restatement on the reference's own block layouts."""
    fx = Fixture(name)
    lus = fx.lus("pre")
    o = pyoracle.oracle_factor(lus, fx.pr, fx.pc, fx.n, fx.replace_tiny, fx.anorm)
    assert o["tiny"] == fx.tiny
    if name.startswith("zeropiv"):
        assert o["info"] > 0 and fx.info > 0
        return
    assert o["info"] == fx.info == 0
    err = cases.factor_error(lus, fx.ref_factors())
    assert err < TOL[fx.dtype], err


@pytest.mark.gpu
@pytest.mark.parametrize("strips", ["1", "2"])
@pytest.mark.parametrize("name", ONE)
def test_gpu_dropin_pdgstrf_on_reference_lustructs(name, strips, monkeypatch):
    """The exported pdgstrf / psgstrf / pzgstrf, called as pdgssvx calls them,
    factor the reference-built LUstruct in place to the reference's factors.
    strips 2: every real diagonal block through k_diag_strips (its zero- /
    tiny-pivot semantics against the reference's)."""
    monkeypatch.setenv("SLU_DIAG_STRIPS", strips)
    from superlu_dist_amd import capi
    fx = Fixture(name)
    lu = fx.lu(0)
    o = capi.default_options()
    o.ReplaceTinyPivot = capi.YES if fx.replace_tiny else capi.NO
    rv, info, st = capi.pxgstrf(lu, fx.anorm, options=o)
    assert rv == 0
    assert info == fx.info
    assert st["TinyPivots"] == fx.tiny
    assert st["num_look_aheads"] == 10
    if info == 0:
        err = cases.factor_error([lu], fx.ref_factors())
        assert err < TOL[fx.dtype], err


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["bcast", "p2p"])
@pytest.mark.parametrize("name", GRIDS)
def test_gpu_grid_on_reference_lustructs(name, transport, tmp_path):
    """bcast: host-staged broadcasts (the drop-in's MPI path when ranks share
    a GPU); p2p: the RCCL transport's send / receive pairs in its order,
    host-staged over gloo isend / irecv."""
    from gridrun import run_grid
    fx = Fixture(name)
    out = run_grid(f"refdump:{name}", fx.pr, fx.pc, tmp_path, device=0, transport=transport)
    assert all(int(o["info"]) == fx.info for o in out)
    assert sum(int(o["tiny"]) for o in out) == fx.tiny
    if fx.info == 0:
        worst = 0.0
        for o, (Lr, Ur) in zip(out, fx.ref_factors()):
            for mine, r in ((o["L"], Lr), (o["U"], Ur)):
                if len(r):
                    mine = mine[:len(r)]  # library-built arrays carry one spare element
                    assert np.isfinite(mine).all()
                    d = np.abs(mine.astype(np.complex128) - r.astype(np.complex128)).max()
                    worst = max(worst, d / max(np.abs(r).max(), 1e-300))
        assert worst < TOL[fx.dtype], worst
