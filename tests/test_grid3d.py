"""3D process grids (pdgstrf3d, SRC/pdgstrf3d.c:121).

Pz layers of a Pr x Pc grid each hold the whole LUstruct; the supernodal
etree is cut into forests (SRC/supernodalForest.c:794), every layer factors
its leaf forest, partial updates of the ancestors are reduced pairwise between
layers and the surviving layers factor the forests above
(SRC/pd3dcomm.c:786).  After slu_plan_gather3d layer 0 holds the factors.

* CPU: schedule-only plans over the point-to-point host transport (gloo
  isend / irecv) replay every layer's level exchanges and the inter-layer
  reductions in factor()'s order with checked bytes; the layers' factored
  supernodes partition the whole set.
* GPU: the factors gathered on layer 0 against the oracle's 2D factors (the
  update sums run in another order, so within the dtype tolerance, not bit
  for bit), info and flops.
"""
import functools

import pytest

import cases
import pyoracle
from gridrun import run_grid
from superlu_dist_amd.frontend import STENCIL_3D7, STENCIL_3D27, Symbolic
from test_oracle import TOL


def _stencil_recipe(kind, dims, dtype, grid, relax, maxsup):
    return cases.stencil_case(kind, dims, dtype, grid, relax, maxsup)


def _recipe(case):
    """(recipe, pr, pc) of a stencil or reference-dump case name."""
    if case.startswith("refdump_"):
        from refdump import Fixture
        name = case[len("refdump_"):]
        fx = Fixture(name)
        return f"refdump:{name}", fx.pr, fx.pc
    _, kind, nx, g = case.split("_")
    pr, pc = int(g[0]), int(g[2])
    kind = STENCIL_3D7 if kind == "3d7" else STENCIL_3D27
    return functools.partial(_stencil_recipe, kind, (int(nx),) * 3, 0, (pr, pc), 60, 256), pr, pc


@pytest.mark.parametrize("case,pz", [
    ("stencil_3d7_12_1x1", 2), ("stencil_3d7_12_1x1", 4), ("stencil_3d7_10_2x1", 2),
    ("stencil_3d27_8_1x2", 2), ("refdump_g20_2x3_small_d", 2), ("refdump_cd2d_24_2x2_d", 2),
])
def test_grid3d_schedule_through_p2p_transport_cpu(case, pz, tmp_path):
    rec, pr, pc = _recipe(case)
    out = run_grid(rec, pr, pc, tmp_path, device=None, transport="schedule", timeout=180, pz=pz)
    P = pr * pc
    # identical levels within a layer; the layers' factored sets partition
    # the supernodes (each layer reports the count it factors)
    for z in range(pz):
        assert len({int(o["nlevels"]) for o in out[z * P:(z + 1) * P]}) == 1
    counts = [int(out[z * P]["nsupers"]) for z in range(pz)]
    assert all(c > 0 for c in counts)
    if isinstance(rec, str):
        from refdump import Fixture
        total = Fixture(rec.split(":", 1)[1]).nsupers
    else:
        A, perm, _, _, relax, maxsup, _ = rec()
        total = Symbolic(A, perm, relax, maxsup).nsupers
    assert sum(counts) == total
    # the reductions moved data (received on the even layers)
    assert sum(int(o["nsec"]) for o in out[:P]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind,dims,dtype,grid,pz", [
    (STENCIL_3D7, (16, 16, 16), 0, (1, 1), 2),
    (STENCIL_3D7, (16, 16, 16), 0, (1, 1), 4),
    (STENCIL_3D7, (14, 14, 14), 0, (2, 1), 2),
    (STENCIL_3D27, (10, 10, 10), 1, (1, 2), 2),
    (STENCIL_3D7, (10, 10, 10), 2, (1, 1), 4),
])
def test_grid3d_matches_oracle_stencil(kind, dims, dtype, grid, pz, tmp_path):
    pr, pc = grid
    rec = functools.partial(_stencil_recipe, kind, dims, dtype, grid, 60, 256)
    out = run_grid(rec, pr, pc, tmp_path, device=0, transport="p2p", pz=pz)
    A, perm, dt, _, _, _, _ = rec()
    S = Symbolic(A, perm, 60, 256)
    lus = [S.distribute(pr, pc, r, c) for r in range(pr) for c in range(pc)]
    o = pyoracle.oracle_factor(lus, pr, pc, A.n, False, cases.anorm(A))
    assert o["info"] == 0 and all(int(x["info"]) == 0 for x in out)
    layer0 = out[:pr * pc]
    err = cases.factor_error([_Fac(x) for x in layer0], [(lu.Lval, lu.Uval) for lu in lus])
    assert err < TOL[dtype], err
    # the layers' algorithmic work sums to the oracle's total
    tot = sum(float(x["flops"]) for x in out)
    assert abs(tot - o["flops"]) <= 1e-9 * o["flops"] + 10
    assert sum(float(x["comm_bytes"]) for x in out) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,pz", [("g20_2x3_small_d", 2), ("lap3d_12_2x2_d", 2),
                                     ("cd2d_20_2x1_z", 2)])
def test_grid3d_on_reference_lustructs(name, pz, tmp_path):
    """The reference's own LUstructs (pdgssvx front-end dumps), factored on
    3D grids of their 2D grid shape, against the reference's factors."""
    from refdump import Fixture
    fx = Fixture(name)
    out = run_grid(f"refdump:{name}", fx.pr, fx.pc, tmp_path, device=0, transport="p2p", pz=pz)
    P = fx.pr * fx.pc
    assert all(int(x["info"]) == fx.info for x in out)
    err = cases.factor_error([_Fac(x) for x in out[:P]], fx.ref_factors())
    assert err < TOL[fx.dtype], err


class _Fac:
    def __init__(self, d):
        self.Lval, self.Uval = d["L"], d["U"]
