"""2D process grids: every rank factors its own LUstruct on the
GPU and exchanges diagonal blocks and panels with its process row / column.

* GPU (``-m gpu``): all multi-rank golden cases (reference factors from
  /root/reference, tests/golden/ref_*_RxC_*.npz) and larger seeded stencils
  against the oracle, through the engine's host-staged test transport (one
  GPU box, several ranks; RCCL refuses two ranks on one device).  The kernels
  and the exchange schedule are the ones the RCCL transport runs.
* CPU: the gloo row/column group plumbing of the test harness (world 4).
"""
import functools

import numpy as np
import pytest

import cases
import pyoracle
from gridrun import run_grid
from superlu_dist_amd.frontend import STENCIL_3D7, STENCIL_3D27, Symbolic
from test_oracle import TOL, load_golden

GRID_CASES = sorted(n for n, c in cases.CASES.items() if c[2] != (1, 1))


def test_gloo_grid_groups_cpu(tmp_path):
    """Row / column broadcasts of the test transport reach the right ranks."""
    rec = functools.partial(cases.build, "lap3d_8_2x2_d")
    out = run_grid(rec, 2, 2, tmp_path, device=None)
    for rank, o in enumerate(out):
        r, c = rank // 2, rank % 2
        assert int(o["row_root"]) == r * 2 + 0       # row broadcast from column 0
        assert int(o["col_root"]) == 1 * 2 + c       # column broadcast from row 1


REFDUMP_GRIDS = ["refdump_big_2x2_d", "refdump_big_1x2_s", "refdump_cd2d_24_2x2_d",
                 "refdump_cd2d_20_2x1_z", "refdump_g20_2x3_small_d", "refdump_lap3d_12_2x2_d",
                 "refdump_zeropiv2_2x2_d", "refdump_cg20_2x2_z"]


@pytest.mark.parametrize("case", REFDUMP_GRIDS + ["stencil_3d7_12_2x4", "stencil_3d27_8_2x2"])
def test_exchange_schedule_through_p2p_transport_cpu(case, tmp_path):
    """No GPU: every rank builds a schedule-only plan over the point-to-point
    host transport (the RCCL send / receive pairs, gloo isend / irecv) --
    the plan-time index / need / edge all-gathers go through it -- and then
    replays every level's diagonal-package and panel exchange of factor()
    with patterned bytes that each receiver checks.  A section sent to the
    wrong rank, in the wrong order or with the wrong size fails; one that is
    never sent hangs until run_grid's timeout."""
    if case.startswith("refdump_"):
        name = case[len("refdump_"):]
        from refdump import Fixture
        fx = Fixture(name)
        pr, pc = fx.pr, fx.pc
        rec = f"refdump:{name}"
    else:
        _, kind, nx, g = case.split("_")
        pr, pc = int(g[0]), int(g[2])
        kind = STENCIL_3D7 if kind == "3d7" else STENCIL_3D27
        rec = functools.partial(_stencil_recipe, kind, (int(nx),) * 3, 0, (pr, pc), 60, 256)
    out = run_grid(rec, pr, pc, tmp_path, device=None, transport="schedule", timeout=120)
    assert len({int(o["nlevels"]) for o in out}) == 1        # identical levels on every rank
    assert sum(int(o["nsec"]) for o in out) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,fill", [(n, False) for n in GRID_CASES] +
                         [("lap3d_10_2x4_small_d", True), ("cg20_2x2_small_z", True)])
def test_grid_matches_reference_fixture(name, fill, tmp_path):
    """fill: every rank loads its values from A on the device (slu_plan_fill_a,
    the SamePattern_SameRowPerm refill) instead of uploading its LUstruct."""
    meta, ref = load_golden(name)
    pr, pc = meta["grid"]
    out = run_grid(functools.partial(cases.build, name), pr, pc, tmp_path, device=0, fill=fill)
    assert all(int(o["info"]) == meta["ref_info"] for o in out)
    assert sum(int(o["tiny"]) for o in out) == meta["ref_tiny"]
    worst = 0.0
    for o, (Lr, Ur) in zip(out, ref):
        for mine, r in ((o["L"], Lr), (o["U"], Ur)):
            if len(r):
                d = np.abs(mine.astype(np.complex128) - r.astype(np.complex128)).max()
                worst = max(worst, d / max(np.abs(r).max(), 1e-300))
    assert worst < TOL[meta["dtype"]], worst


def _stencil_recipe(kind, dims, dtype, grid, relax, maxsup):
    return cases.stencil_case(kind, dims, dtype, grid, relax, maxsup)


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["bcast", "p2p"])
@pytest.mark.parametrize("kind,dims,dtype,grid,relax,maxsup", [
    (STENCIL_3D7, (16, 16, 16), 0, (2, 2), 60, 256),
    (STENCIL_3D7, (20, 20, 20), 0, (2, 4), 60, 256),   # 128x128 Schur tiles on 8 ranks
    (STENCIL_3D7, (14, 14, 14), 0, (1, 2), 60, 320),   # > 256-column supernodes
    (STENCIL_3D27, (12, 12, 12), 1, (2, 2), 60, 256),
    (STENCIL_3D7, (10, 10, 10), 2, (2, 1), 60, 256),
])
def test_grid_matches_oracle_stencil(kind, dims, dtype, grid, relax, maxsup, transport, tmp_path):
    rec = functools.partial(_stencil_recipe, kind, dims, dtype, grid, relax, maxsup)
    pr, pc = grid
    out = run_grid(rec, pr, pc, tmp_path, device=0, transport=transport)
    A, perm, dt, _, _, _, _ = rec()
    S = Symbolic(A, perm, relax, maxsup)
    lus = [S.distribute(pr, pc, r, c) for r in range(pr) for c in range(pc)]
    o = pyoracle.oracle_factor(lus, pr, pc, A.n, False, cases.anorm(A))
    assert o["info"] == 0 and all(int(x["info"]) == 0 for x in out)
    err = cases.factor_error([_Fac(x) for x in out], [(lu.Lval, lu.Uval) for lu in lus])
    assert err < TOL[dtype], err
    # per-rank algorithmic work sums to the oracle's total
    tot = sum(float(x["flops"]) for x in out)
    assert abs(tot - o["flops"]) <= 1e-9 * o["flops"] + 10


class _Fac:
    def __init__(self, d):
        self.Lval, self.Uval = d["L"], d["U"]
