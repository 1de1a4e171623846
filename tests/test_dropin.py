"""The drop-in promise end to end: the reference's own drivers
EXAMPLE/p[dsz]drive.c, linked against libslu_mi355x.so FIRST and then the
reference library with pdgstrf.o / psgstrf.o / pzgstrf.o removed
(oracle/_ref/p?drive_mi355x, built by `make -C oracle dropin`), run the
reference's whole pipeline -- matrix read, equilibration, MC64, MMD, the
reference sp_colorder / symbfact / pddistribute, OUR p?gstrf, the reference
pdgstrs / pdgsrfs -- and must solve as accurately as the same drivers linked
with the reference factorization (oracle/_ref/p?drive_ref).  The opt-in
libslu_mi355x_full.so (p?drive_mi355x_full) also replaces sp_colorder /
symbfact and provides METIS_NodeND for the drivers' default ordering.

GPU: 1 rank (1x1 grid), and 4 ranks on a 2x2 grid sharing the box's one GPU
(the library then carries the panel broadcasts over MPI instead of RCCL).
CPU: the links themselves (which symbols each binary binds from where).
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

REF = os.path.join(ROOT, "oracle", "_ref")
MPIEXEC = "/opt/conda/bin/mpiexec"
MAT = os.path.join(ROOT, "tests", "golden", "matrices")


def _have(*names):
    return all(os.path.exists(os.path.join(REF, n)) for n in names) and os.path.exists(MPIEXEC)


def _run(exe, nprocs, args, matrix, timeout=240):
    env = dict(os.environ)
    env.update({"OMP_NUM_THREADS": "1", "MKL_NUM_THREADS": "1", "MKL_THREADING_LAYER": "SEQUENTIAL",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    cmd = [MPIEXEC, "-n", str(nprocs), os.path.join(REF, exe)] + args + [os.path.join(MAT, matrix)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"{exe} failed ({r.returncode}):\n{out[-3000:]}"
    assert "ERROR: INFO" not in out, out[-2000:]
    errs = [float(x) for x in re.findall(r"\|\|X ?- ?Xtrue\|\| ?/ ?\|\|X\|\| = ([0-9.eE+-]+)", out)]
    assert errs, out[-2000:]
    m = re.search(r"FACTOR time\s+([0-9.]+)", out)
    return max(errs), (float(m.group(1)) if m else None), out


def _binding(exe):
    exe = os.path.join(REF, exe)
    dyn = subprocess.run(["readelf", "-d", exe], capture_output=True, text=True).stdout
    und = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True,
                         text=True).stdout.split()
    defined = subprocess.run(["nm", "--defined-only", exe], capture_output=True, text=True).stdout
    return dyn, und, defined


@pytest.mark.skipif(not _have("pddrive_mi355x"), reason="drop-in drivers not built")
def test_dropin_driver_binds_our_pdgstrf():
    """Default drop-in: pdgstrf comes from libslu_mi355x.so, the symbolic
    factorization stays the reference's own (linked from the archive)."""
    dyn, und, defined = _binding("pddrive_mi355x")
    assert "libslu_mi355x.so" in dyn and "libslu_mi355x_full.so" not in dyn
    assert "pdgstrf" in und                          # resolved at load time from the library
    assert not re.search(r"\bT pdgstrf\b", defined)  # no reference copy inside
    for sym in ("symbfact", "sp_colorder", "pddistribute"):
        assert sym not in und and re.search(rf"\bT {sym}\b", defined), sym


@pytest.mark.skipif(not _have("pddrive_mi355x_full"), reason="opt-in drivers not built")
def test_optin_driver_binds_our_symbolic():
    dyn, und, defined = _binding("pddrive_mi355x_full")
    assert "libslu_mi355x_full.so" in dyn
    for sym in ("pdgstrf", "symbfact", "sp_colorder", "METIS_NodeND"):
        assert sym in und, sym                       # from libslu_mi355x_full.so
        assert not re.search(rf"\bT {sym}\b", defined)


CASES = [
    # driver, matrix, extra args
    ("pddrive", "g20.rua", []),
    ("pddrive", "big.rua", []),
    ("psdrive", "g20.rua", []),
    ("pzdrive", "cg20.cua", []),
]


@pytest.mark.gpu
@pytest.mark.skipif(not _have("pddrive_mi355x", "pddrive_ref"), reason="drivers not built")
@pytest.mark.parametrize("nprocs,grid", [(1, ["-r", "1", "-c", "1"]), (4, ["-r", "2", "-c", "2"])])
@pytest.mark.parametrize("drv,matrix,extra", CASES)
def test_reference_driver_with_our_factorization(drv, matrix, extra, nprocs, grid):
    args = grid + ["-q", "2"] + extra      # MMD_AT_PLUS_A: METIS is not in the image
    ref_err, ref_t, _ = _run(f"{drv}_ref", nprocs, args, matrix)
    my_err, my_t, out = _run(f"{drv}_mi355x", nprocs, args, matrix)
    tol = 1e-4 if drv == "psdrive" else 1e-12
    print(f"{drv} {matrix} {nprocs} ranks: ||x-xtrue||/||x|| ref {ref_err:.3e} mi355x {my_err:.3e}; "
          f"FACTOR time ref {ref_t} s, mi355x {my_t} s")
    assert my_err <= max(10 * ref_err, tol), (my_err, ref_err)


@pytest.mark.gpu
@pytest.mark.skipif(not _have("pddrive_mi355x_full", "pddrive_ref"), reason="drivers not built")
@pytest.mark.parametrize("drv,matrix", [("pddrive", "g20.rua"), ("pddrive", "big.rua"),
                                        ("pzdrive", "cg20.cua")])
def test_reference_driver_default_ordering_through_our_metis(drv, matrix):
    """No -q: the drivers' default ColPerm = METIS_AT_PLUS_A, which calls
    METIS_NodeND (SRC/get_perm_c.c:524-541).  METIS is not in the image, so
    only the library's nested dissection can serve it; the driver with the
    reference's factorization and solve runs MMD (-q 2) for the accuracy
    yardstick."""
    ref_err, _, _ = _run(f"{drv}_ref", 1, ["-r", "1", "-c", "1", "-q", "2"], matrix)
    my_err, _, out = _run(f"{drv}_mi355x_full", 1, ["-r", "1", "-c", "1"], matrix)
    print(f"{drv} {matrix} METIS_AT_PLUS_A via the library: {my_err:.3e} (reference, MMD: {ref_err:.3e})")
    assert my_err <= max(10 * ref_err, 1e-12), (my_err, ref_err)


# ---- device solve behind pdgssvx: p?drive_mi355x_solve
# links libslu_mi355x_solve.so, whose p?gstrs solves on the factors the
# preceding p?gstrf left in HBM (1 rank; on the 2x2 grid a plan adopts the
# host factors); the reference's pdgsrfs calls it for every refinement step.

@pytest.mark.skipif(not _have("pddrive_mi355x_solve"), reason="solve drop-in drivers not built")
def test_dropin_solve_driver_binds_our_pdgstrs():
    dyn, und, defined = _binding("pddrive_mi355x_solve")
    assert "libslu_mi355x_solve.so" in dyn
    for sym in ("pdgstrf", "pdgstrs", "pdCompute_Diag_Inv", "pddistribute"):
        assert sym in und and not re.search(rf"\bT {sym}\b", defined), sym
    for sym in ("pdgsrfs", "pdgssvx", "symbfact"):
        assert re.search(rf"\bT {sym}\b", defined), sym   # the reference's own
    assert not re.search(r"\bT pdReDistribute_B_to_X\b", defined)  # pdgstrs.o not linked


@pytest.mark.gpu
@pytest.mark.skipif(not _have("pddrive_mi355x_solve", "pddrive_ref"), reason="drivers not built")
@pytest.mark.parametrize("nprocs,grid", [(1, ["-r", "1", "-c", "1"]), (4, ["-r", "2", "-c", "2"])])
@pytest.mark.parametrize("drv,matrix,extra", CASES)
def test_reference_driver_with_our_factorization_and_solve(drv, matrix, extra, nprocs, grid):
    args = grid + ["-q", "2"] + extra
    ref_err, _, ref_out = _run(f"{drv}_ref", nprocs, args, matrix)
    my_err, _, out = _run(f"{drv}_mi355x_solve", nprocs, args, matrix)
    tol = 1e-4 if drv == "psdrive" else 1e-12
    t = lambda o, k: (re.search(rf"{k} time\s+([0-9.]+)", o) or [None, None])[1]  # noqa: E731
    steps = lambda o: (re.search(r"REFINEMENT time\s+[0-9.]+\s+Steps\s+(\d+)", o) or [None, None])[1]  # noqa: E731
    print(f"{drv} {matrix} {nprocs} ranks: ||x-xtrue||/||x|| ref {ref_err:.3e} mi355x {my_err:.3e}; "
          f"SOLVE ref {t(ref_out, 'SOLVE')} s / mi355x {t(out, 'SOLVE')} s, REFINEMENT ref "
          f"{t(ref_out, 'REFINEMENT')} s ({steps(ref_out)} steps) / mi355x {t(out, 'REFINEMENT')} s "
          f"({steps(out)} steps)")
    assert my_err <= max(10 * ref_err, tol), (my_err, ref_err)


@pytest.mark.gpu
@pytest.mark.skipif(not _have("pddrive3_mi355x_solve", "pddrive3_ref_nd"), reason="drivers not built")
@pytest.mark.parametrize("nprocs,grid", [(1, ["-r", "1", "-c", "1"]), (4, ["-r", "2", "-c", "2"])])
# (EXAMPLE/pddrive2.c, SamePattern, fails with the reference library alone:
# its second pdgssvx call reports an illegal parameter 5 and aborts)
@pytest.mark.parametrize("drv", ["pddrive1", "pddrive3"])
@pytest.mark.parametrize("matrix", ["big.rua", "g20.rua"])
def test_reference_reentry_drivers_with_our_distribute_factor_solve(drv, matrix, nprocs, grid):
    """pdgssvx called again on one LUstruct: pddrive1 (Fact = FACTORED, new
    right-hand sides on the kept factors), pddrive3 (SamePattern_SameRowPerm: pddistribute's value
    refill on the existing structure, then the plan cache's refactorization)
    with pddistribute, pdgstrf and pdgstrs from libslu_mi355x_solve.so."""
    ref_err, _, ref_out = _run(f"{drv}_ref_nd", nprocs, grid, matrix)
    my_err, _, out = _run(f"{drv}_mi355x_solve", nprocs, grid, matrix)
    ref_all = [float(x) for x in re.findall(r"\|\|X-Xtrue\|\|/\|\|X\|\| = ([0-9.eE+-]+)", ref_out)]
    my_all = [float(x) for x in re.findall(r"\|\|X-Xtrue\|\|/\|\|X\|\| = ([0-9.eE+-]+)", out)]
    dist = lambda o: re.findall(r"DISTRIBUTE time\s+([0-9.]+)", o)  # noqa: E731
    print(f"{drv} {matrix} {nprocs} ranks: errors ref {ref_all} mi355x {my_all}; "
          f"DISTRIBUTE ref {dist(ref_out)} mi355x {dist(out)}")
    assert len(my_all) == len(ref_all) > 0
    for m, r in zip(my_all, ref_all):
        assert m <= max(10 * r, 1e-12), (my_all, ref_all)


# ---- 3D (pdgstrf3d): the reference's EXAMPLE/pddrive3d.c
# (pdgssvx3d: 3D matrix distribution, dinitTrf3Dpartition's forests, its
# ancestor zeroing, pdgstrf3d, dgatherAllFactoredLU, pdgstrs / pdgsrfs on
# layer 0) with pdgstrf3d from libslu_mi355x_3d.so (oracle/_ref/
# pddrive3d_mi355x, `make -C oracle dropin3d`) against the driver with the
# reference's pdgstrf3d (pddrive3d_ref, `make -C oracle ref3d`; the _nd
# variants of both take METIS_NodeND from libslu_mi355x_metis.so, so for them
# the yardstick is the reference everywhere except the ordering).  Several ranks share the
# box's GPU: the library carries the layer exchanges and the ancestor
# reductions over MPI point to point.

@pytest.mark.skipif(not _have("pddrive3d_mi355x"), reason="3D drop-in driver not built")
def test_dropin3d_driver_binds_our_pdgstrf3d():
    dyn, und, defined = _binding("pddrive3d_mi355x")
    assert "libslu_mi355x_3d.so" in dyn
    assert "pdgstrf3d" in und and not re.search(r"\bT pdgstrf3d\b", defined)
    for sym in ("pdgssvx3d", "dinitTrf3Dpartition", "dgatherAllFactoredLU", "pdgstrs"):
        assert re.search(rf"\bT {sym}\b", defined), sym   # the reference's own


def _run_schedule(exe, nprocs, args, matrix, timeout=240):
    """SUPERLU_MI355X_SCHEDULE_ONLY=1: pdgstrf3d builds schedule-only plans
    (no GPU) over the MPI point-to-point transport and replays every
    exchange with checked bytes, then returns without factoring."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1",
               SUPERLU_MI355X_SCHEDULE_ONLY="1")
    cmd = [MPIEXEC, "-n", str(nprocs), os.path.join(REF, exe)] + args + [os.path.join(MAT, matrix)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"{exe} failed ({r.returncode}):\n{out[-3000:]}"
    return re.findall(r"layer (\d+): (\d+) supernodes factored in (\d+) levels, (\d+) sections / "
                      r"(\d+) bytes received, exchange checked", out)


# (driver, matrix, ordering args): MMD (-q 2) and the default METIS_AT_PLUS_A
# served by libslu_mi355x_metis.so (the _nd drivers)
CASES3D = [("pddrive3d", "big.rua", ["-q", "2"]), ("pddrive3d", "g20.rua", ["-q", "2"]),
           ("pddrive3d", "lap3d12.rua", ["-q", "2"]), ("pddrive3d_nd", "lap3d12.rua", [])]
GRIDS3D = [(1, 1, 2), (1, 2, 2), (2, 1, 2), (1, 1, 4), (2, 2, 2)]


@pytest.mark.skipif(not _have("pddrive3d_mi355x", "pddrive3d_mi355x_nd"), reason="3D drivers not built")
@pytest.mark.parametrize("grid", GRIDS3D)
@pytest.mark.parametrize("drv,matrix,order", CASES3D)
def test_dropin3d_exchange_schedule_cpu(drv, matrix, order, grid):
    """No GPU: the reference's pdgssvx3d up to pdgstrf3d (its forests, its
    3D LUstruct from dp3dScatter on every layer), then our schedule-only
    plans replay the layer exchanges and the ancestor reductions over MPI."""
    r, c, d = grid
    exe = drv.replace("pddrive3d", "pddrive3d_mi355x")
    rows = _run_schedule(exe, r * c * d, ["-r", str(r), "-c", str(c), "-d", str(d)] + order, matrix)
    assert len(rows) == r * c * d
    layers = {}
    for z, ns, nl, nsec, nb in rows:
        layers.setdefault(int(z), set()).add(int(ns))
    assert sorted(layers) == list(range(d))
    assert all(len(v) == 1 for v in layers.values())     # one count per layer
    assert sum(next(iter(v)) for v in layers.values()) > 0


@pytest.mark.gpu
@pytest.mark.skipif(not _have("pddrive3d_mi355x", "pddrive3d_ref"), reason="3D drivers not built")
@pytest.mark.parametrize("grid", GRIDS3D)
@pytest.mark.parametrize("drv,matrix,order", CASES3D)
def test_reference_3d_driver_with_our_pdgstrf3d(drv, matrix, order, grid):
    r, c, d = grid
    args = ["-r", str(r), "-c", str(c), "-d", str(d)] + order
    ref_err, ref_t, _ = _run(drv.replace("pddrive3d", "pddrive3d_ref"), r * c * d, args, matrix)
    my_err, my_t, out = _run(drv.replace("pddrive3d", "pddrive3d_mi355x"), r * c * d, args, matrix)
    print(f"{drv} {matrix} {r}x{c}x{d}: ||x-xtrue||/||x|| ref {ref_err:.3e} mi355x {my_err:.3e}; "
          f"FACTOR time ref {ref_t} s, mi355x {my_t} s")
    assert my_err <= max(10 * ref_err, 1e-12), (my_err, ref_err)


# ---- two LUstructs in one process: on a 1x1 grid the
# factors of the last pdgstrf live only in HBM, in the cached plan.  Factoring
# a second LUstruct evicts that plan; a FACTORED solve of the first must then
# fail loudly instead of solving with A's values (oracle/gen/evict_solve_main.c).
def _evict(env_extra):
    env = dict(os.environ)
    env.update({"OMP_NUM_THREADS": "1", "MKL_NUM_THREADS": "1", "MKL_THREADING_LAYER": "SEQUENTIAL",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, **env_extra)
    cmd = [MPIEXEC, "-n", "1", os.path.join(REF, "evict_solve"),
           os.path.join(MAT, "g20.rua"), os.path.join(MAT, "big.rua")]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240)
    out = r.stdout + r.stderr
    errs = {int(k): float(v) for k, v in re.findall(r"system (\d): err ([0-9.eE+-]+)", out)}
    return r.returncode, errs, out


@pytest.mark.skipif(not _have("evict_solve"), reason="eviction driver not built")
def test_evict_driver_binds_our_solve():
    dyn, und, _ = _binding("evict_solve")
    assert "libslu_mi355x_solve.so" in dyn
    for sym in ("pdgstrf", "pdgstrs", "pddistribute"):
        assert sym in und, sym


@pytest.mark.gpu
@pytest.mark.skipif(not _have("evict_solve"), reason="eviction driver not built")
def test_factored_solve_after_eviction_fails_loudly():
    rc, errs, out = _evict({})
    assert errs.get(1, 1) < 1e-10 and errs.get(2, 1) < 1e-10, out[-3000:]
    assert rc != 0 and 3 not in errs, out[-3000:]
    assert "kept only in GPU memory" in out, out[-3000:]


@pytest.mark.gpu
@pytest.mark.skipif(not _have("evict_solve"), reason="eviction driver not built")
def test_factored_solve_after_eviction_with_host_factors():
    rc, errs, out = _evict({"SUPERLU_MI355X_HOST_FACTORS": "1"})
    assert rc == 0, out[-3000:]
    assert sorted(errs) == [1, 2, 3] and max(errs.values()) < 1e-10, out[-3000:]


# The grid life cycle twice in one process (oracle/gen/regrid_main.c): each
# round gridinit -> pdgssvx (DOFACT) -> pdgssvx (SamePattern_SameRowPerm, a
# plan-cache hit) -> gridexit.  gridexit destroys the engine communicators,
# and the cached plan built on them goes with them: the
# next round's first call builds a new plan even when MPI reuses the
# communicator handle and malloc the LUstruct addresses.
#
# The second system in a process also needs the caller's libc rand()
# sequence to be the same on every rank: the reference's pddistribute draws
# its solve trees' seeds from it (SRC/pddistribute.c:1557), and the HSA
# runtime reseeds it whenever it creates a queue (any HIP stream).  The
# driver draws one rand() per rank after every pdgssvx and reports whether
# the ranks agree ("rand same"); without the library's guard the ranks'
# sequences part after the first factorization and round 1's solve errs ~1.
def _regrid(nprocs, pr, pc, **extra):
    env = dict(os.environ)
    env.update({"OMP_NUM_THREADS": "1", "MKL_NUM_THREADS": "1", "MKL_THREADING_LAYER": "SEQUENTIAL",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0", "SUPERLU_MI355X_TIMING": "1"}, **extra)
    cmd = [MPIEXEC, "-n", str(nprocs), os.path.join(REF, "regrid"), os.path.join(MAT, "big.rua"),
           str(pr), str(pc)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    return r.returncode, r.stdout + r.stderr


@pytest.mark.skipif(not _have("regrid"), reason="grid life-cycle driver not built")
def test_regrid_driver_binds_our_pdgstrf():
    dyn, und, _ = _binding("regrid")
    assert "libslu_mi355x.so" in dyn and "pdgstrf" in und


@pytest.mark.gpu
@pytest.mark.parametrize("pr,pc", [(1, 1), (2, 2)])
@pytest.mark.skipif(not _have("regrid"), reason="grid life-cycle driver not built")
def test_grid_exit_evicts_the_cached_plan(pr, pc):
    rc, out = _regrid(pr * pc, pr, pc)
    assert rc == 0, out[-3000:]
    res = re.findall(r"round (\d) call (\d): info (\d+) err ([0-9.eE+-]+)", out)
    summary = "\n".join(f"round {a} call {b}: info {c} err {d}" for a, b, c, d in res)
    assert len(res) == 4, out[-3000:]
    for _, _, info, err in res:
        assert int(info) == 0 and float(err) < 1e-10, summary + "\n" + out[-2500:]
    assert re.findall(r"err [0-9.eE+-]+ rand (\w+)", out) == ["same"] * 4, out[-3000:]
    # rank 0's plan per call: built, reused, then (new grid) built, reused
    plans = re.findall(r"\[PDGSTRF rank 0\] digest [0-9.]+ ms, plan (built|reused)", out)
    if pr * pc > 1:
        assert plans == ["built", "reused", "built", "reused"], out[-3000:]
    else:  # 1x1: the transport is per device and outlives the grid: the plan may stay
        assert plans[0] == "built" and plans[1] == plans[3] == "reused", out[-3000:]


@pytest.mark.gpu
def test_device_resident_system_through_solve_library():
    """bench.py's device-resident leg at a test size: libslu_mi355x_solve.so's
    pddistribute (keeps A), pdgstrf (device fill, factors kept in HBM) and
    pdgstrs, driven through capi as pdgssvx drives them, then the
    SamePattern_SameRowPerm refactorization; the solutions are accurate."""
    import numpy as np
    import scipy.sparse as sp
    from superlu_dist_amd import capi
    from superlu_dist_amd import symbolic as SY
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, nd_order
    nx = 16
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    n = A.n
    cp, ri, v = A.arrays()
    co = SY.sp_colorder(n, n, cp, ri, nd_order(nx, nx, nx), SY.MY_PERMC)
    sb = SY.symbfact(n, n, co.colbeg, co.colend, SY.relabel_rows(ri, co.perm_c), co.etree, 60, 256)
    s = capi.DeviceResidentSystem(n, cp, co.perm_c[ri], v, co.perm_c, co.etree, sb.xsup, sb.supno,
                                  sb.xlsub, sb.lsub, sb.xusub, sb.usub, 12.0)
    xt = np.random.default_rng(0).standard_normal(n)
    b = sp.csc_matrix((v, ri, cp), shape=(n, n)) @ xt
    for fact in (0, capi.SAMEPATTERN_SAMEROWPERM):
        s.distribute(fact)
        rv, info, ops = s.factor()
        assert rv == 0 and info == 0 and ops > 0
        x = s.solve(b)
        assert np.abs(x - xt).max() <= 1e-10 * np.abs(xt).max()


@pytest.mark.gpu
@pytest.mark.skipif(not _have("regrid"), reason="grid life-cycle driver not built")
def test_grid_refactorization_without_plan_cache():
    """The same life cycle on 2x2 with the plan cache off
    (SUPERLU_MI355X_PLAN_CACHE=0): every call builds its plan."""
    rc, out = _regrid(4, 2, 2, SUPERLU_MI355X_PLAN_CACHE="0")
    assert rc == 0, out[-3000:]
    res = re.findall(r"round (\d) call (\d): info (\d+) err ([0-9.eE+-]+)", out)
    summary = "\n".join(f"round {a} call {b}: info {c} err {d}" for a, b, c, d in res)
    assert len(res) == 4 and all(int(i) == 0 and float(e) < 1e-10 for _, _, i, e in res), summary
    assert re.findall(r"err [0-9.eE+-]+ rand (\w+)", out) == ["same"] * 4, out[-3000:]


@pytest.mark.gpu
@pytest.mark.skipif(not _have("regrid"), reason="grid life-cycle driver not built")
def test_second_system_on_the_same_grid():
    """Two systems one after the other on ONE 2x2 grid (REGRID_SAMEGRID:
    new LUstruct / SOLVEstruct, same communicators): the second solve is
    as accurate as the first and the ranks' rand() sequences agree."""
    rc, out = _regrid(4, 2, 2, REGRID_SAMEGRID="1")
    assert rc == 0, out[-3000:]
    res = re.findall(r"round (\d) call (\d): info (\d+) err ([0-9.eE+-]+) rand (\w+)", out)
    summary = "\n".join(" ".join(r) for r in res)
    assert len(res) == 4 and all(int(i) == 0 and float(e) < 1e-10 and rs == "same"
                                 for _, _, i, e, rs in res), summary


_DEFER_CHILD = r"""
import numpy as np
from superlu_dist_amd import capi
from superlu_dist_amd import symbolic as SY
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, nd_order
nx = 8
def system():
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    n = A.n
    cp, ri, v = A.arrays()
    co = SY.sp_colorder(n, n, cp, ri, nd_order(nx, nx, nx), SY.MY_PERMC)
    sb = SY.symbfact(n, n, co.colbeg, co.colend, SY.relabel_rows(ri, co.perm_c), co.etree, 60, 256)
    return capi.DeviceResidentSystem(n, cp, co.perm_c[ri], v, co.perm_c, co.etree, sb.xsup, sb.supno,
                                     sb.xlsub, sb.lsub, sb.xusub, sb.usub, 12.0)
s1, s2 = system(), system()
s1.distribute(0)
s2.distribute(0)  # replaces the A kept for s1's device fill
print("factoring s1", flush=True)
s1.factor()
print("s1 factored", flush=True)
"""


@pytest.mark.gpu
def test_deferred_a_replaced_fails_loudly():
    """libslu_mi355x_solve.so's pddistribute keeps A for the device fill
    instead of placing it into the host value arrays: a
    pdgstrf on an LUstruct whose kept A another pddistribute has replaced
    stops with a message instead of factoring the zero host arrays."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", _DEFER_CHILD], capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert "factoring s1" in r.stdout, r.stdout + r.stderr
    assert "s1 factored" not in r.stdout and r.returncode != 0
    assert "another pddistribute has replaced" in r.stderr, r.stderr[-2000:]
