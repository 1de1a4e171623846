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


def _read_trace(fn):
    """[(phase, level, [(kind, group, peer world rank, bytes), ...]), ...]"""
    out = []
    for ln in open(fn):
        t = ln.split()
        if t[0] == "F":
            out.append((" ".join(t[2:-1]), int(t[-1]), []))
        else:
            out[-1][2].append((t[0], int(t[1]), int(t[2]), int(t[3])))
    return out


@pytest.mark.parametrize("case,pr,pc", [("refdump:big_2x2_d", 2, 2), ("stencil", 2, 4)])
def test_rccl_call_sequence_is_the_tested_one_cpu(case, pr, pc, tmp_path, monkeypatch):
    """the RCCL branch's ncclSend / ncclRecv list (recorded
    by a dry run of flush_rccl, SLU_XPORT_TRACE) equals, group by group, the
    list the point-to-point test transport runs, on every rank; and across
    ranks every send A -> B of a group has its receive on B from A, in the
    same order, of the same size, in the same phase and level -- the
    condition under which RCCL's in-order point-to-point matching neither
    hangs nor mixes sections up (the plan-time all-gathers included: no
    ncclBroadcast is left)."""
    trace = tmp_path / "trace"
    trace.mkdir()
    monkeypatch.setenv("SLU_XPORT_TRACE", str(trace))
    if case == "stencil":
        rec = functools.partial(_stencil_recipe, STENCIL_3D7, (12,) * 3, 0, (pr, pc), 60, 256)
    else:
        rec = case
    run_grid(rec, pr, pc, tmp_path, device=None, transport="schedule", timeout=120)
    P = pr * pc
    host = [_read_trace(trace / f"xport_host.{r}") for r in range(P)]
    rccl = [_read_trace(trace / f"xport_rccl.{r}") for r in range(P)]
    for r in range(P):
        assert host[r] == rccl[r], f"rank {r}: RCCL call list differs from the tested one"
        assert len(host[r]) > 10
    # cross-rank pairing per (group, sender, receiver) stream
    sends, recvs = {}, {}
    for r in range(P):
        for phase, level, calls in host[r]:
            for kind, g, peer, nbytes in calls:
                if kind == "S":
                    sends.setdefault((g, r, peer), []).append((nbytes, phase, level))
                else:
                    recvs.setdefault((g, peer, r), []).append((nbytes, phase, level))
    assert set(sends) == set(recvs)
    for key in sends:
        g, a, b = key
        if g == 1:
            assert a // pc == b // pc       # row group: same process row
        elif g == 2:
            assert a % pc == b % pc         # column group: same process column
        assert sends[key] == recvs[key], key
    nlev = {lv for r in range(P) for _, lv, _ in host[r] if lv >= 0}
    assert len(nlev) > 3                     # the per-level exchanges are in it
    # the chunked panel exchange (SLU_PANEL_CHUNKS, default 4): on the
    # stencil some level's panels go out in more than one group
    from collections import Counter
    per = Counter((r, lv) for r in range(P) for ph, lv, _ in host[r] if ph.startswith("L/U panel"))
    if case == "stencil":
        assert max(per.values()) > 1, per


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


def _stencil_recipe(kind, dims, dtype, grid, relax, maxsup, reference=False):
    return cases.stencil_case(kind, dims, dtype, grid, relax, maxsup, reference)


@pytest.mark.parametrize("grid,nx", [((2, 2), 16), ((2, 4), 16), ((1, 2), 12), ((3, 2), 12)])
def test_grid_amalgamation_schedule_through_p2p_transport_cpu(grid, nx, tmp_path):
    """The structure pdgssvx builds (reference symbfact + pddistribute: many
    width-1 supernodes) on a grid: every rank's schedule-only plan runs the
    grid amalgamation over the point-to-point transport (structure to the
    analysis owners, partition all-gather, pieces to the coarse owners) and
    replays the coarse plan's exchanges with checked bytes.  The ranks agree
    on a partition coarser than the caller's, and their shares of the
    caller partition's flops add up to the 1x1 count."""
    from superlu_dist_amd.frontend import Amalgamation, Csc, nd_order
    pr, pc = grid
    rec = functools.partial(_stencil_recipe, STENCIL_3D7, (nx,) * 3, 0, grid, 60, 256, True)
    out = run_grid(rec, pr, pc, tmp_path, device=None, transport="schedule", timeout=180)
    ns = {int(o["nsupers"]) for o in out}
    nin = {int(o["nsupers_in"]) for o in out}
    assert len(ns) == 1 and len(nin) == 1 and ns.pop() < nin.pop()
    assert len({int(o["nlevels"]) for o in out}) == 1
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    one = Amalgamation(Symbolic(A, nd_order(nx, nx, nx), 60, 256, reference=True).distribute())
    assert sum(float(o["flops"]) for o in out) == pytest.approx(one.flops(), rel=1e-12)


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


@pytest.mark.gpu
@pytest.mark.skipif(not pyoracle.have_reference_harness(), reason="oracle/_ref not built")
@pytest.mark.parametrize("grid", [(2, 2), (2, 4)])
def test_grid_amalgamation_fingerprints_match_reference_pdgstrf(grid, tmp_path):
    """The north-star path at a test size: the LUstruct pdgssvx builds for a
    24^3 Laplacian (reference symbfact + pddistribute: the fine partition)
    on a 2x2 / 2x4 grid, every rank factoring on the GPU through the grid
    amalgamation (coarse partition, relayout over the point-to-point
    transport); the factors, back in every rank's caller layout, against
    the REFERENCE pdgstrf on the same grid through per-block fingerprints."""
    pr, pc = grid
    rec = functools.partial(_stencil_recipe, STENCIL_3D7, (24, 24, 24), 0, grid, 60, 256, True)
    out = run_grid(rec, pr, pc, tmp_path, device=0, transport="p2p", timeout=600)
    assert all(int(o["info"]) == 0 for o in out)
    assert all(int(o["nsupers"]) < int(o["nsupers_in"]) for o in out)
    A, perm = rec()[:2]
    S = Symbolic(A, perm, 60, 256, reference=True)
    mine = np.concatenate([pyoracle.blocksums(S.distribute(pr, pc, k // pc, k % pc), o["L"], o["U"])
                           for k, o in enumerate(out)])
    st, _ = pyoracle.run_reference(A, perm, pr, pc, symb_flags=2, want_factors=False,
                                   want_blocksums=True, timeout=600)
    c = pyoracle.compare_blocksums(mine, st["blocksums"])
    assert c["match"] and c["rel_err"] <= 1e-12, c


def test_watchdog_reports_a_dropped_section_cpu(tmp_path, monkeypatch, capfd):
    """the exchange watchdog (csrc/watchdog.h).  A first
    schedule-only run over the point-to-point transport records every send of
    rank 0; the second run drops rank 0's last section of the replay (and what follows it to that peer)
    of factor()'s last exchanges.  The receiver's watchdog must fire within
    its bound (SLU_WATCHDOG_S = 3) with the phase, the level and the pending
    section (peer, bytes), and end that rank with exit status 86 instead of a
    hang."""
    (tmp_path / "a").mkdir()
    out = run_grid("refdump:big_2x2_d", 2, 2, tmp_path / "a", device=None, transport="schedule",
                   timeout=120)
    sends = out[0]["sends"]
    # the last section of the replay (the 8-byte all-gathers after it are the
    # plan's closing statistics)
    k = max(i for i in range(len(sends)) if sends[i][1] > 8)
    peer, nbytes = (int(x) for x in sends[k])
    (tmp_path / "b").mkdir()
    monkeypatch.setenv("SLU_TEST_DROP_SEND", f"0:{k}")
    monkeypatch.setenv("SLU_WATCHDOG_S", "3")
    capfd.readouterr()
    with pytest.raises(RuntimeError) as ei:
        run_grid("refdump:big_2x2_d", 2, 2, tmp_path / "b", device=None, transport="schedule",
                 timeout=90)
    msg = str(ei.value)
    assert f"rank {peer}: exit 86" in msg, msg
    err = capfd.readouterr().err
    line = [ln for ln in err.splitlines() if ln.startswith(f"[slu watchdog] rank {peer} ")
            and "oldest open exchange" in ln]
    assert line, err[-4000:]
    assert "exchange (replay) of level" in line[0], line[0]
    assert f"receive from" in line[0] and f"(rank 0): {nbytes} bytes" in line[0], line[0]
    assert "has not completed after" in err
