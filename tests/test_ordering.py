"""The library's METIS_NodeND (csrc/ordering.cpp): the ordering the
reference's get_perm_c_dist asks for with ColPerm = METIS_AT_PLUS_A, its
default (SRC/get_perm_c.c:524-541; METIS itself is not in the image, so the
reference alone cannot run it here).  No reference output to pin it to
("parity unpinned": METIS's own orderings are not available); the tests
check a valid permutation on every graph shape and the fill it gives,
through the reference-exact symbolic factorization, against the
reference's MMD ordering of the same matrix (tests/golden/symb_*.npz).
CPU only."""
import os

import numpy as np
import pytest

from superlu_dist_amd import symbolic as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _grid3d(k):
    idx = np.arange(k ** 3).reshape(k, k, k)
    r, c = [idx.ravel()], [idx.ravel()]
    for ax in range(3):
        a = np.moveaxis(idx, ax, 0)
        r += [a[1:].ravel(), a[:-1].ravel()]
        c += [a[:-1].ravel(), a[1:].ravel()]
    r, c = np.concatenate(r), np.concatenate(c)
    o = np.lexsort((r, c))
    n = k ** 3
    colptr = np.zeros(n + 1, np.int64)
    np.add.at(colptr, c[o] + 1, 1)
    return n, np.cumsum(colptr), r[o].astype(np.int64)


def _nnzl(n, colptr, rowind, perm_c, relax=60, maxsup=256):
    co = S.sp_colorder(n, n, colptr, rowind, perm_c, S.MMD_AT_PLUS_A)
    sb = S.symbfact(n, n, co.colbeg, co.colend, S.relabel_rows(rowind, co.perm_c), co.etree,
                    relax, maxsup)
    return sb.nnzL


def _check_perm(n, perm_c, perm):
    assert np.array_equal(np.sort(perm_c), np.arange(n))
    assert np.array_equal(perm_c[perm], np.arange(n))   # iperm[perm[i]] = i


@pytest.mark.parametrize("kind", ["grid", "random", "components", "empty", "one", "star", "path"])
def test_nodend_returns_a_permutation(kind):
    rng = np.random.default_rng(3)
    if kind == "grid":
        n, colptr, rowind = _grid3d(9)
    elif kind == "random":
        n = 3000
        cols = [np.unique(np.append(rng.integers(0, n, 4), c)) for c in range(n)]
        colptr = np.zeros(n + 1, np.int64)
        colptr[1:] = np.cumsum([len(x) for x in cols])
        rowind = np.concatenate(cols).astype(np.int64)
    elif kind == "components":           # 40 disjoint paths of 50 + isolated vertices
        n = 2100
        r, c = list(range(n)), list(range(n))
        for p in range(40):
            for i in range(49):
                r.append(p * 50 + i)
                c.append(p * 50 + i + 1)
        r, c = np.array(r), np.array(c)
        o = np.lexsort((r, c))
        colptr = np.zeros(n + 1, np.int64)
        np.add.at(colptr, c[o] + 1, 1)
        colptr, rowind = np.cumsum(colptr), r[o].astype(np.int64)
    elif kind in ("empty", "one"):
        n = 1000 if kind == "empty" else 1
        colptr, rowind = np.arange(n + 1, dtype=np.int64), np.arange(n, dtype=np.int64)
    elif kind == "star":                  # one hub: no useful level separator
        n = 500
        r = np.concatenate([np.arange(n), np.zeros(n - 1, np.int64)])
        c = np.concatenate([np.arange(n), np.arange(1, n)])
        o = np.lexsort((r, c))
        colptr = np.zeros(n + 1, np.int64)
        np.add.at(colptr, c[o] + 1, 1)
        colptr, rowind = np.cumsum(colptr), r[o].astype(np.int64)
    else:                                 # path: deep bisection recursion
        n = 200000
        r = np.concatenate([np.arange(n), np.arange(1, n)])
        c = np.concatenate([np.arange(n), np.arange(n - 1)])
        o = np.lexsort((r, c))
        colptr = np.zeros(n + 1, np.int64)
        np.add.at(colptr, c[o] + 1, 1)
        colptr, rowind = np.cumsum(colptr), r[o].astype(np.int64)
    xadj, adj = S.at_plus_a(n, colptr, rowind)
    perm_c, perm = S.metis_nodend(n, xadj, adj)
    _check_perm(n, perm_c, perm)


def test_nodend_fill_against_reference_mmd():
    """3D 7-point 12^3 (the golden's pattern and the reference's MMD perm_c):
    nested dissection fills no more than the reference's MMD (137 k vs
    140 k; 60^3: 0.48x)."""
    z = np.load(os.path.join(GOLDEN, "symb_lap3d12_mmd.npz"), allow_pickle=False)
    n = int(z["meta"][0])
    colptr, rowind = z["colptr"], z["rowind"]
    mmd = _nnzl(n, colptr, rowind, z["perm_c_in"])
    xadj, adj = S.at_plus_a(n, colptr, rowind)
    nd = _nnzl(n, colptr, rowind, S.metis_nodend(n, xadj, adj)[0])
    assert nd <= mmd, (nd, mmd)


def test_nodend_fill_scales_like_nested_dissection():
    """24^3: well below the fill of the natural (banded) order and
    below the geometric grid dissection the benchmark uses."""
    from superlu_dist_amd.lib import as_i64p, lib
    k = 24
    n, colptr, rowind = _grid3d(k)
    xadj, adj = S.at_plus_a(n, colptr, rowind)
    nd = _nnzl(n, colptr, rowind, S.metis_nodend(n, xadj, adj)[0])
    geo = np.zeros(n, np.int64)
    lib().slu_order_nd_grid(k, k, k, as_i64p(geo))
    assert nd <= _nnzl(n, colptr, rowind, geo)
    assert nd * 3 < _nnzl(n, colptr, rowind, np.arange(n))   # banded natural order: 3.5x


def test_nodend_rejects_bad_input():
    xadj = np.array([0, 1, 2], np.int64)
    adj = np.array([1, 5], np.int64)      # 5 out of range
    with pytest.raises(RuntimeError):
        S.metis_nodend(2, xadj, adj)
    xadj = np.array([0, 2, 1], np.int64)  # decreasing pointers
    with pytest.raises(RuntimeError):
        S.metis_nodend(2, xadj, np.array([1, 0], np.int64))
