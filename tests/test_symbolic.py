"""Column ordering post-pass and symbolic factorization
against the REFERENCE: tests/golden/symb_*.npz hold the reference's own
sp_colorder / symbfact outputs on the same patterns and perm_c
(oracle/gen/make_symb_golden.py, oracle/_ref/symb_dump running
SRC/sp_colorder.c and SRC/symbfact.c as pdgssvx does).  Bit-exact: every
array, the return value and nnzLU.  CPU only (host code)."""
import glob
import os

import numpy as np
import pytest

from superlu_dist_amd import symbolic as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(os.path.basename(f)[5:-4] for f in glob.glob(os.path.join(GOLDEN, "symb_*.npz")))


def _load(name):
    z = np.load(os.path.join(GOLDEN, f"symb_{name}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def test_goldens_present():
    assert len(CASES) >= 10


@pytest.mark.parametrize("name", CASES)
def test_sp_colorder_matches_reference(name):
    g = _load(name)
    n, colperm = int(g["meta"][0]), int(g["meta"][1])
    co = S.sp_colorder(n, n, g["colptr"], g["rowind"], g["perm_c_in"], colperm)
    np.testing.assert_array_equal(co.etree, g["etree"])
    np.testing.assert_array_equal(co.perm_c, g["perm_c"])
    np.testing.assert_array_equal(co.colbeg, g["colbeg"])
    np.testing.assert_array_equal(co.colend, g["colend"])


@pytest.mark.parametrize("name", CASES)
def test_symbfact_matches_reference(name):
    g = _load(name)
    n, relax, maxsup = int(g["meta"][0]), int(g["meta"][2]), int(g["meta"][3])
    ret, nnzlu, relax_eff, maxsup_eff = (int(x) for x in g["scalars"])
    assert relax_eff == min(relax, maxsup) and maxsup_eff == maxsup
    ri = S.relabel_rows(g["rowind"], g["perm_c"])
    sb = S.symbfact(n, n, g["colbeg"], g["colend"], ri, g["etree"], relax_eff, maxsup_eff)
    ns = int(g["supno"][n]) + 1
    assert sb.nsupers == ns
    np.testing.assert_array_equal(sb.xsup, g["xsup"][:ns + 1])
    np.testing.assert_array_equal(sb.supno, g["supno"])
    np.testing.assert_array_equal(sb.xlsub, g["xlsub"])
    np.testing.assert_array_equal(sb.lsub, g["lsub"])
    np.testing.assert_array_equal(sb.xusub, g["xusub"])
    np.testing.assert_array_equal(sb.usub, g["usub"])
    assert sb.nnzLU == nnzlu
    assert sb.ret == ret


def test_symbfact_end_to_end_from_pattern():
    """sp_colorder -> relabel -> symbfact on the golden's input alone
    reproduces the reference (the path pdgssvx takes)."""
    g = _load("rand2000_mmd")
    n, relax, maxsup = int(g["meta"][0]), int(g["meta"][2]), int(g["meta"][3])
    co = S.sp_colorder(n, n, g["colptr"], g["rowind"], g["perm_c_in"], S.MMD_AT_PLUS_A)
    sb = S.symbfact(n, n, co.colbeg, co.colend, S.relabel_rows(g["rowind"], co.perm_c), co.etree,
                    min(relax, maxsup), maxsup)
    np.testing.assert_array_equal(sb.lsub, g["lsub"])
    np.testing.assert_array_equal(sb.usub, g["usub"])


def test_symbfact_zero_diagonal_raises():
    # column 1 has no diagonal entry and nothing fills it: the reference
    # ABORTs in pivotL (SRC/symbfact.c:724-727); the library reports it
    colptr = np.array([0, 1, 2], np.int64)
    rowind = np.array([0, 0], np.int64)
    co = S.sp_colorder(2, 2, colptr, rowind, np.arange(2), S.NATURAL)
    with pytest.raises(RuntimeError, match="zero diagonal"):
        S.symbfact(2, 2, co.colbeg, co.colend, S.relabel_rows(rowind, co.perm_c), co.etree, 1, 10)


def test_dropin_symbols_with_reference_types():
    """The exported sp_colorder / symbfact themselves, called as pdgssvx calls
    them (SRC/pdgssvx.c:1046-1076) with the reference's structs: NCformat in,
    NCPformat AC out, rows relabelled in place, Glu_persist / Glu_freeable
    filled with malloc'ed arrays; relax / maxsup taken from the options."""
    import ctypes as C

    from superlu_dist_amd import capi
    from superlu_dist_amd.lib import lib
    L = lib()
    g = _load("big_r8s20")
    n, relax, maxsup = int(g["meta"][0]), int(g["meta"][2]), int(g["meta"][3])
    colptr = np.ascontiguousarray(g["colptr"], np.int64)
    rowind = np.ascontiguousarray(g["rowind"], np.int64).copy()
    i64p = C.POINTER(C.c_int64)
    As = capi.NCformat(len(rowind), None, rowind.ctypes.data_as(i64p), colptr.ctypes.data_as(i64p))
    A = capi.SuperMatrix(0, 1, 0, n, n, C.cast(C.pointer(As), C.c_void_p))
    AC = capi.SuperMatrix()
    opt = capi.default_options()
    opt.Fact = 0                      # DOFACT
    opt.ColPerm = 2                   # MMD_AT_PLUS_A (perm_c given)
    opt.superlu_relax, opt.superlu_maxsup = relax, maxsup
    perm_c = np.ascontiguousarray(g["perm_c_in"], np.int64).copy()
    etree = np.zeros(n, np.int64)
    L.sp_colorder.argtypes = [C.c_void_p] * 5
    L.sp_colorder(C.byref(opt), C.byref(A), perm_c.ctypes.data, etree.ctypes.data, C.byref(AC))
    assert AC.Stype == 1 and AC.nrow == n            # SLU_NCP
    S_ = C.cast(AC.Store, C.POINTER(capi.NCPformat)).contents
    cb = np.ctypeslib.as_array(S_.colbeg, (n,)).copy()
    ce = np.ctypeslib.as_array(S_.colend, (n,)).copy()
    np.testing.assert_array_equal(cb, g["colbeg"])
    np.testing.assert_array_equal(ce, g["colend"])
    np.testing.assert_array_equal(perm_c, g["perm_c"])
    np.testing.assert_array_equal(etree, g["etree"])
    rowind[:] = perm_c[rowind]        # SRC/pdgssvx.c:1053-1058 (AC shares rowind)
    gp, gf = capi.GluPersist(), capi.GluFreeable()
    L.symbfact.restype = C.c_int64
    L.symbfact.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 5
    ret = L.symbfact(C.byref(opt), 0, C.byref(AC), perm_c.ctypes.data, etree.ctypes.data,
                     C.byref(gp), C.byref(gf))
    assert ret == int(g["scalars"][0]) and gf.nnzLU == int(g["scalars"][1])
    arr = lambda p, k: np.ctypeslib.as_array(p, (k,)).copy()  # noqa: E731
    np.testing.assert_array_equal(arr(gp.supno, n + 1), g["supno"])
    ns = int(g["supno"][n]) + 1
    np.testing.assert_array_equal(arr(gp.xsup, ns + 1), g["xsup"][:ns + 1])
    xl, xu = arr(gf.xlsub, n + 1), arr(gf.xusub, n + 1)
    np.testing.assert_array_equal(xl, g["xlsub"])
    np.testing.assert_array_equal(xu, g["xusub"])
    np.testing.assert_array_equal(arr(gf.lsub, int(xl[n])), g["lsub"])
    np.testing.assert_array_equal(arr(gf.usub, int(xu[n])), g["usub"])
    assert gf.MemModel == 0 and gf.nzlmax >= xl[n] and gf.nzumax >= xu[n]
    libc = C.CDLL(None)               # the arrays are the caller's to free()
    for p in (gp.xsup, gp.supno, gf.lsub, gf.xlsub, gf.usub, gf.xusub, S_.colbeg, S_.colend):
        libc.free(C.cast(p, C.c_void_p))
    libc.free(C.c_void_p(AC.Store))


def _classic_vs_default(n, colptr, rowind, perm, colperm, relax, maxsup, monkeypatch):
    co = S.sp_colorder(n, n, colptr, rowind, perm, colperm)
    ri = S.relabel_rows(rowind, co.perm_c)
    monkeypatch.setenv("SLU_SYMB_CLASSIC", "1")
    a = S.symbfact(n, n, co.colbeg, co.colend, ri, co.etree, relax, maxsup)
    monkeypatch.delenv("SLU_SYMB_CLASSIC")
    b = S.symbfact(n, n, co.colbeg, co.colend, ri, co.etree, relax, maxsup)
    for f in ("xsup", "supno", "xlsub", "lsub", "xusub", "usub"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    assert (a.ret, a.nnzL, a.nnzU, a.nnzLU) == (b.ret, b.nnzL, b.nnzU, b.nnzLU)
    return a


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("relax,maxsup", [(1, 3), (4, 10), (8, 20), (60, 256), (2, 512)])
def test_symbfact_virtual_last_list_equals_classic(seed, relax, maxsup, monkeypatch):
    """The default walker keeps the current supernode's last list virtual
    (csrc/symbolic.cpp, column_v); SLU_SYMB_CLASSIC=1 runs the literal
    restatement of SRC/symbfact.c.  Random unsymmetric patterns (rows in
    random order within each column) with several relax / maxsup: every
    array and the returned lsub size are the same."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(50, 400))
    cols = []
    for c in range(n):
        k = int(rng.integers(1, 6))
        rows = set(rng.integers(0, n, k).tolist()) | {c}
        if c > 0 and rng.random() < 0.7:
            rows.add(c - 1)  # chains: supernodes of several columns
        r = list(rows)
        rng.shuffle(r)
        cols.append(r)
    colptr = np.zeros(n + 1, np.int64)
    colptr[1:] = np.cumsum([len(c) for c in cols])
    rowind = np.array([r for c in cols for r in c], np.int64)
    perm = rng.permutation(n).astype(np.int64)
    for colperm in (S.MMD_AT_PLUS_A, S.MMD_ATA):
        _classic_vs_default(n, colptr, rowind, perm, colperm, relax, maxsup, monkeypatch)


def test_symbfact_virtual_last_list_3d_stencil(monkeypatch):
    """Wide fundamental supernodes (a 3D 7-point grid in natural order,
    maxsup 256 and 16): the case the virtual list is for."""
    k = 14
    n = k ** 3
    idx = np.arange(n).reshape(k, k, k)
    cols = [[] for _ in range(n)]
    for d in ((0, 0, 0), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
        a = np.roll(idx, d, axis=(0, 1, 2))
        ok = np.ones((k, k, k), bool)
        for ax in range(3):
            if d[ax] == 1:
                ok[(slice(None),) * ax + (0,)] = False
            elif d[ax] == -1:
                ok[(slice(None),) * ax + (k - 1,)] = False
        for c, r in zip(idx[ok].ravel(), a[ok].ravel()):
            cols[c].append(int(r))
    colptr = np.zeros(n + 1, np.int64)
    colptr[1:] = np.cumsum([len(c) for c in cols])
    rowind = np.array([r for c in cols for r in c], np.int64)
    for relax, maxsup in ((60, 256), (4, 16)):
        s = _classic_vs_default(n, colptr, rowind, np.arange(n, dtype=np.int64), S.NATURAL, relax,
                                maxsup, monkeypatch)
        assert s.nsupers < n


def _tasks_vs_ordered(n, cb, ce, ri, etree, relax, maxsup, monkeypatch, tmin, tmax):
    monkeypatch.setenv("SLU_SYMB_TASKS", "0")
    a = S.symbfact(n, n, cb, ce, ri, etree, relax, maxsup)
    monkeypatch.setenv("SLU_SYMB_TASKS", "1")
    monkeypatch.setenv("SLU_SYMB_TASK_MIN", str(tmin))
    monkeypatch.setenv("SLU_SYMB_TASK_MAX", str(tmax))
    b = S.symbfact(n, n, cb, ce, ri, etree, relax, maxsup)
    for f in ("xsup", "supno", "xlsub", "lsub", "xusub", "usub"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    assert (a.ret, a.nnzL, a.nnzU, a.nnzLU) == (b.ret, b.nnzL, b.nnzU, b.nnzLU)
    return b


@pytest.mark.parametrize("name", CASES)
def test_symbfact_subtree_tasks_match_reference(name, monkeypatch):
    """Subtree tasks forced down to a few columns (csrc/symbolic.cpp,
    plan_tasks / import_task): every array still the REFERENCE's."""
    monkeypatch.setenv("SLU_SYMB_TASK_MIN", "2")
    g = _load(name)
    n = int(g["meta"][0])
    monkeypatch.setenv("SLU_SYMB_TASK_MAX", str(max(2, n // 16)))
    test_symbfact_matches_reference(name)


@pytest.mark.parametrize("relax,maxsup", [(60, 256), (4, 16), (1, 1), (8, 20)])
@pytest.mark.parametrize("tmin,tmax", [(2, 40), (8, 300), (64, 2000)])
def test_symbfact_subtree_tasks_equal_column_order(relax, maxsup, tmin, tmax, monkeypatch):
    """A 20^3 nested-dissection Laplacian and a 12^3 27-point one: the
    search with subtree tasks gives the same arrays as the one in column
    order, for several relax / maxsup and task sizes."""
    from superlu_dist_amd.frontend import STENCIL_3D7, STENCIL_3D27, Csc, nd_order
    for st, k in ((STENCIL_3D7, 20), (STENCIL_3D27, 12)):
        A = Csc.stencil(st, k, k, k)
        cp, ri, _ = A.arrays()
        co = S.sp_colorder(A.n, A.n, cp, ri, nd_order(k, k, k), S.MY_PERMC)
        rr = S.relabel_rows(ri, co.perm_c)
        _tasks_vs_ordered(A.n, co.colbeg, co.colend, rr, co.etree, relax, maxsup, monkeypatch, tmin, tmax)


@pytest.mark.parametrize("seed", range(4))
def test_symbfact_subtree_tasks_unsymmetric(seed, monkeypatch):
    """Random unsymmetric patterns (the A'+A and A'A etrees): tasks where
    the pattern allows them, the same arrays either way."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(300, 900))
    cols = []
    for c in range(n):
        rows = set(rng.integers(0, n, int(rng.integers(1, 5))).tolist()) | {c}
        if c > 0 and rng.random() < 0.7:
            rows.add(c - 1)
        cols.append(list(rows))
    colptr = np.zeros(n + 1, np.int64)
    colptr[1:] = np.cumsum([len(c) for c in cols])
    rowind = np.array([r for c in cols for r in c], np.int64)
    perm = rng.permutation(n).astype(np.int64)
    for colperm in (S.MMD_AT_PLUS_A, S.MMD_ATA):
        co = S.sp_colorder(n, n, colptr, rowind, perm, colperm)
        rr = S.relabel_rows(rowind, co.perm_c)
        for relax, maxsup in ((1, 3), (4, 10)):
            _tasks_vs_ordered(n, co.colbeg, co.colend, rr, co.etree, relax, maxsup, monkeypatch, 2, 30)


def _epilogue_device():
    from superlu_dist_amd.lib import lib
    return int(lib().slu_symbfact_last_epilogue_device())


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_symbfact_device_epilogue_matches_reference(name, monkeypatch):
    """symbfact's countnz + fixupL (SRC/util.c:95-199) on the GPU
    (csrc/symbolic_dev.hip, SLU_SYMB_DEVICE=1): every array, nnzLU and the
    return value equal the REFERENCE's on every symb_* golden."""
    monkeypatch.setenv("SLU_SYMB_DEVICE", "1")
    test_symbfact_matches_reference(name)
    assert _epilogue_device() == 1


@pytest.mark.gpu
def test_symbfact_device_epilogue_large(monkeypatch):
    """A 40^3 Laplacian in nested-dissection order (4 098 supernodes, wide
    top separators): the device epilogue equals the host one."""
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, nd_order
    k = 40
    A = Csc.stencil(STENCIL_3D7, k, k, k)
    cp, ri, _ = A.arrays()
    co = S.sp_colorder(A.n, A.n, cp, ri, nd_order(k, k, k), S.MY_PERMC)
    rr = S.relabel_rows(ri, co.perm_c)
    out = {}
    for dev in ("0", "1"):
        monkeypatch.setenv("SLU_SYMB_DEVICE", dev)
        out[dev] = S.symbfact(A.n, A.n, co.colbeg, co.colend, rr, co.etree, 60, 256)
        assert _epilogue_device() == int(dev)
    for f in ("xsup", "supno", "xlsub", "lsub", "xusub", "usub"):
        np.testing.assert_array_equal(getattr(out["0"], f), getattr(out["1"], f), err_msg=f)
    assert (out["0"].ret, out["0"].nnzLU) == (out["1"].ret, out["1"].nnzLU)
