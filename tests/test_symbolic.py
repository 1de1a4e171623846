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
