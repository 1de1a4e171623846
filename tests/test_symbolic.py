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
