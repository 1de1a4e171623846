"""Parity of the MI355X engine (libslu_mi355x.so, through its C ABI) with the
reference pdgstrf / psgstrf / pzgstrf.

* every 1x1 golden case: factors vs the REFERENCE's factors
  (tests/golden/ref_*.npz), info and TinyPivots exact;
* larger seeded stencils: factors vs the oracle (C restatement);
* full-size-style property: backward error of the solve with the GPU factors.
Tolerances (north star): normwise-max relative 1e-12 fp64 / complex, 1e-5 fp32.
"""
import numpy as np
import pytest

import cases
import pyoracle
from lusolve import backward_error, solve_1x1
from superlu_dist_amd.engine import Plan, factor_lustruct
from superlu_dist_amd.frontend import STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Csc, Symbolic, nd_order
from test_oracle import TOL, load_golden

pytestmark = pytest.mark.gpu

ONE_BY_ONE = sorted(n for n, c in cases.CASES.items() if c[2] == (1, 1))


@pytest.mark.parametrize("name", ONE_BY_ONE)
def test_gpu_matches_reference_fixture(name):
    meta, ref = load_golden(name)
    A, S, lus = cases.distribute(name)
    assert cases.structure_digest(lus) == meta["digest"]
    info, tiny, st = factor_lustruct(lus[0], anorm=meta["anorm"], replace_tiny=meta["replace_tiny"])
    assert info == meta["ref_info"]
    assert tiny == meta["ref_tiny"]
    if info == 0:
        err = cases.factor_error(lus, ref)
        assert err < TOL[meta["dtype"]], err


@pytest.mark.parametrize("kind,dims,dtype,relax,maxsup", [
    (STENCIL_3D7, (20, 20, 20), 0, 60, 256),
    (STENCIL_3D7, (20, 20, 20), 0, 60, 320),   # supernodes > 256 columns: generic panel path
    (STENCIL_3D7, (24, 24, 24), 0, 60, 256),   # 128x128 Schur tiles
    (STENCIL_3D27, (16, 16, 16), 1, 60, 256),  # fp32 128x128 Schur tiles
    (STENCIL_3D7, (20, 20, 20), 2, 60, 320),
    (STENCIL_3D7, (16, 16, 16), 0, 4, 24),
    (STENCIL_2D5, (60, 60, 1), 0, 60, 256),
    (STENCIL_3D27, (12, 12, 12), 1, 60, 256),
    (STENCIL_3D7, (12, 12, 12), 2, 60, 256),
])
def test_gpu_matches_oracle_stencil(kind, dims, dtype, relax, maxsup):
    kw = {}
    if dtype == 2:
        kw = dict(diag=6 - 0.25, diag_im=-0.0025)
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), relax, maxsup)
    gpu, ref = S.distribute(), S.distribute()
    an = cases.anorm(A)
    info, tiny, st = factor_lustruct(gpu, anorm=an)
    o = pyoracle.oracle_factor([ref], 1, 1, A.n, False, an)
    assert info == o["info"] == 0
    err = cases.factor_error([gpu], [(ref.Lval, ref.Uval)])
    assert err < TOL[dtype], err
    # the plan's algorithmic flop count equals the oracle's accounting
    assert abs(st["schur_flops"] + st["panel_flops"] - o["flops"]) <= 1e-9 * o["flops"] + 10


def test_gpu_backward_error_3d():
    """Size-independent property at a size the oracle would be slow on."""
    A = Csc.stencil(STENCIL_3D7, 32, 32, 32)
    S = Symbolic(A, nd_order(32, 32, 32), 60, 256)
    lu = S.distribute()
    info, tiny, st = factor_lustruct(lu, anorm=12.0)
    assert info == 0
    rng = np.random.default_rng(1)
    xt = rng.standard_normal(A.n)
    B = A.permuted(S.perm_c)
    cp, ri, v = B.arrays()
    b = np.zeros(A.n)
    for j in range(A.n):
        b[ri[cp[j]:cp[j + 1]]] += v[cp[j]:cp[j + 1]] * xt[j]
    x = solve_1x1(lu, b)
    berr = backward_error(A, S.perm_c, x, b)
    assert berr < 1e-14, berr
    assert np.abs(x - xt).max() / np.abs(xt).max() < 1e-10


def test_gpu_refactor_same_plan_is_reproducible_without_atomics():
    """A plan can be re-uploaded and re-factored (SamePattern reuse)."""
    A = Csc.stencil(STENCIL_3D7, 10, 10, 10)
    S = Symbolic(A, nd_order(10, 10, 10), 60, 256)
    lu = S.distribute()
    L0, U0 = lu.Lval.copy(), lu.Uval.copy()
    p = Plan(lu)
    outs = []
    for _ in range(2):
        lu.Lval[:] = L0
        lu.Uval[:] = U0
        p.upload()
        assert p.factor(12.0) == (0, 0)
        p.download()
        outs.append((lu.Lval.copy(), lu.Uval.copy()))
    assert np.allclose(outs[0][0], outs[1][0], rtol=0, atol=1e-13)
    assert np.allclose(outs[0][1], outs[1][1], rtol=0, atol=1e-13)


@pytest.mark.parametrize("kind,dims,dtype", [
    (STENCIL_3D7, (10, 10, 10), 0),
    (STENCIL_3D7, (10, 10, 10), 1),
    (STENCIL_3D27, (10, 10, 10), 1),
    (STENCIL_3D7, (8, 8, 8), 2),
    (STENCIL_2D5, (30, 30, 1), 1),
])
def test_gpu_factors_finite_with_poisoned_lds(kind, dims, dtype):
    """Every kernel must only read LDS it wrote: with the LDS of every CU
    filled with NaN before the factorization, the factors still match the
    oracle (a stale-LDS read, even one multiplied by zero, gives NaN)."""
    from superlu_dist_amd.lib import lib
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), 60, 256)
    gpu, ref = S.distribute(), S.distribute()
    an = cases.anorm(A)
    p = Plan(gpu)
    p.upload()
    assert lib().slu_debug_poison_lds(0) == 0
    assert p.factor(an) == (0, 0)
    p.download()
    assert np.isfinite(gpu.Lval).all() and np.isfinite(gpu.Uval).all()
    pyoracle.oracle_factor([ref], 1, 1, A.n, False, an)
    err = cases.factor_error([gpu], [(ref.Lval, ref.Uval)])
    assert err < TOL[dtype], err


@pytest.mark.parametrize("slot_kb,dtype", [(64, 0), (1024, 1), (256, 2), (0, 0)])
def test_gpu_overlapped_upload_download(slot_kb, dtype, monkeypatch):
    """The drop-in path's copies (hostio.h): the values go up beside the plan
    build, each level's factors come back while later levels run, through
    pinned slots (tiny slots here, so blocks split across fills)."""
    if slot_kb:
        monkeypatch.setenv("SLU_D2H_SLOT_KB", str(slot_kb))
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(STENCIL_3D7, 14, 14, 14, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(14, 14, 14), 60, 256)
    gpu, ref = S.distribute(), S.distribute()
    an = cases.anorm(A)
    p = Plan(gpu, overlap_upload=True, overlap_download=True)
    p.upload()
    gpu.Lval[:] = np.nan                   # the write-back must cover every value
    gpu.Uval[:] = np.nan
    assert p.factor(an) == (0, 0)
    p.download()                           # a no-op: already written back
    st = p.stats()
    vb = (gpu.Lval.size - 1 + gpu.Uval.size - 1) * gpu.Lval.itemsize  # the caller's values
    assert st["d2h_bytes"] == vb and st["h2d_bytes"] == vb
    pyoracle.oracle_factor([ref], 1, 1, A.n, False, an)
    err = cases.factor_error([gpu], [(ref.Lval[:-1], ref.Uval[:-1])])
    assert err < TOL[dtype], err


def _graph_case(kind, dims, dtype):
    from superlu_dist_amd.symbolic import at_plus_a, metis_nodend
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    cp, ri, _ = A.arrays()
    return A, metis_nodend(A.n, *at_plus_a(A.n, cp, ri))[0]


@pytest.mark.parametrize("kind,dims,dtype", [
    (STENCIL_3D7, (16, 16, 16), 0),
    (STENCIL_3D7, (24, 24, 24), 0),    # 128x128 Schur tiles
    (STENCIL_3D27, (14, 14, 14), 1),
    (STENCIL_3D7, (12, 12, 12), 2),
])
def test_gpu_graph_ordering_multichild_matches_oracle(kind, dims, dtype):
    """The bench's --ordering graph configuration: the library's
    METIS_NodeND on A'+A and the multi-child chain partition
    (Symbolic(multichild=True)); factors against the oracle, then the solve
    with the GPU factors (backward and forward error)."""
    A, perm = _graph_case(kind, dims, dtype)
    S = Symbolic(A, perm, 60, 256, multichild=True)
    gpu, ref = S.distribute(), S.distribute()
    an = cases.anorm(A)
    info, tiny, st = factor_lustruct(gpu, anorm=an)
    o = pyoracle.oracle_factor([ref], 1, 1, A.n, False, an)
    assert info == o["info"] == 0
    err = cases.factor_error([gpu], [(ref.Lval, ref.Uval)])
    assert err < TOL[dtype], err
    assert abs(st["schur_flops"] + st["panel_flops"] - o["flops"]) <= 1e-9 * o["flops"] + 10
    if dtype == 0:
        xt = np.random.default_rng(3).standard_normal(A.n)
        cp, ri, v = A.permuted(S.perm_c).arrays()
        b = np.zeros(A.n)
        for j in range(A.n):
            b[ri[cp[j]:cp[j + 1]]] += v[cp[j]:cp[j + 1]] * xt[j]
        x = solve_1x1(gpu, b)
        assert backward_error(A, S.perm_c, x, b) < 1e-14
        assert np.abs(x - xt).max() / np.abs(xt).max() < 1e-10


@pytest.mark.parametrize("kind,dims,dtype,amalg", [
    (STENCIL_3D7, (20, 20, 20), 0, True),
    (STENCIL_3D7, (20, 20, 20), 0, False),
    (STENCIL_3D7, (24, 24, 24), 0, True),
    (STENCIL_3D27, (14, 14, 14), 1, True),
    (STENCIL_3D27, (14, 14, 14), 1, False),
    (STENCIL_3D7, (12, 12, 12), 2, True),
    (STENCIL_2D5, (60, 60, 1), 0, True),
])
def test_gpu_reference_structure_matches_oracle(kind, dims, dtype, amalg, monkeypatch):
    """The LUstruct the reference's pdgssvx builds for a given perm_c (its
    own sp_colorder + symbfact + pddistribute, bench.py's headline
    structure): many width-1 supernodes from the separators' borders.  The
    plan factors the engine's coarse partition (csrc/amalg.h) and relays the
    values into the caller's layout; SLU_AMALG=0 factors the fine one."""
    monkeypatch.setenv("SLU_AMALG", "1" if amalg else "0")
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    S = Symbolic(A, nd_order(*dims), 60, 256, reference=True)
    gpu, ref = S.distribute(), S.distribute()
    an = cases.anorm(A)
    info, tiny, st = factor_lustruct(gpu, anorm=an)
    o = pyoracle.oracle_factor([ref], 1, 1, A.n, False, an)
    assert info == o["info"] == 0
    err = cases.factor_error([gpu], [(ref.Lval, ref.Uval)])
    assert err < TOL[dtype], err
    assert abs(st["schur_flops"] + st["panel_flops"] - o["flops"]) <= 1e-9 * o["flops"] + 10
    assert st["nsupers_in"] == S.nsupers
    assert (st["nsupers"] < S.nsupers) == amalg


@pytest.mark.skipif(not pyoracle.have_reference_harness(), reason="oracle/_ref not built")
def test_gpu_reference_structure_fingerprints_match_reference_pdgstrf():
    """bench.py's full-size parity check at a test size: the drop-in pdgstrf's
    factors against the REFERENCE pdgstrf's (2x2 MPI grid) through the
    per-block fingerprints (oracle/blocksum.h)."""
    from superlu_dist_amd import capi
    A = Csc.stencil(STENCIL_3D7, 24, 24, 24)
    p = nd_order(24, 24, 24)
    S = Symbolic(A, p, 60, 256, reference=True)
    lu = S.distribute()
    rv, info, _ = capi.pxgstrf(lu, 12.0)
    assert rv == 0 and info == 0
    st, _ = pyoracle.run_reference(A, p, 2, 2, symb_flags=2, want_factors=False,
                                   want_blocksums=True, timeout=300)
    c = pyoracle.compare_blocksums(pyoracle.blocksums(lu), st["blocksums"])
    assert c["match"] and c["rel_err"] <= 1e-12, c


def test_dropin_plan_cache_refactors_new_values(monkeypatch, capfd):
    """The drop-in keeps its last 1x1 plan (pdgssvx's SamePattern_SameRowPerm
    refactorization, abi.cpp): a second pdgstrf on the same LUstruct with new
    values must factor the NEW values -- with Fact = DOFACT (full structure
    digest) and with Fact = SamePattern_SameRowPerm (shallow digest: the
    caller's contract is the previous L & U structures) -- and a second
    LUstruct of the same pattern (its own arrays) must not be served by the
    first one's plan."""
    from superlu_dist_amd import capi
    monkeypatch.setenv("SUPERLU_MI355X_TIMING", "1")
    A = Csc.stencil(STENCIL_3D7, 16, 16, 16)
    S = Symbolic(A, nd_order(16, 16, 16), 60, 256, reference=True)
    lu, ref = S.distribute(), S.distribute()
    L0, U0 = lu.Lval.copy(), lu.Uval.copy()
    opt = capi.default_options()
    for fact, scale in ((0, 1.0), (0, 2.0), (2, 0.5), (2, 3.0)):   # same structure, new values
        lu.Lval[:] = L0 * scale
        lu.Uval[:] = U0 * scale
        ref.Lval[:] = L0 * scale
        ref.Uval[:] = U0 * scale
        opt.Fact = fact
        capfd.readouterr()
        rv, info, _ = capi.pxgstrf(lu, 12.0 * scale, options=opt)
        assert rv == 0 and info == 0
        if scale != 1.0:
            assert "plan reused" in capfd.readouterr().err, (fact, scale)
        pyoracle.oracle_factor([ref], 1, 1, A.n, False, 12.0 * scale)
        err = cases.factor_error([lu], [(ref.Lval, ref.Uval)])
        assert err < TOL[0], (scale, err)
    other = S.distribute()                     # same pattern, other arrays
    rv, info, _ = capi.pxgstrf(other, 12.0)
    lu.Lval[:] = L0
    lu.Uval[:] = U0
    ref.Lval[:] = L0
    ref.Uval[:] = U0
    pyoracle.oracle_factor([ref], 1, 1, A.n, False, 12.0)
    assert rv == 0 and info == 0
    err = cases.factor_error([other], [(ref.Lval, ref.Uval)])
    assert err < TOL[0], err


@pytest.mark.parametrize("mode", ["0", "1", "2"])
@pytest.mark.parametrize("kind,dims,dtype", [
    (STENCIL_3D7, (24, 24, 24), 0),
    (STENCIL_3D27, (14, 14, 14), 1),
])
def test_gpu_diag_strips_match_oracle(kind, dims, dtype, mode, monkeypatch):
    """The multi-workgroup diagonal LU (k_diag_strips, csrc/diag_strips.h) on
    the reference structure: off (0), the default levels (1: wide blocks, few
    per level) and every fast level (2, narrow blocks and the leaves' many
    blocks too) -- factors against the oracle."""
    monkeypatch.setenv("SLU_DIAG_STRIPS", mode)
    A = Csc.stencil(kind, *dims, dtype=dtype)
    S = Symbolic(A, nd_order(*dims), 60, 256, reference=True)
    gpu, ref = S.distribute(), S.distribute()
    an = cases.anorm(A)
    info, tiny, st = factor_lustruct(gpu, anorm=an)
    o = pyoracle.oracle_factor([ref], 1, 1, A.n, False, an)
    assert info == o["info"] == 0
    err = cases.factor_error([gpu], [(ref.Lval, ref.Uval)])
    assert err < TOL[dtype], err
