"""Column ordering post-pass and symbolic factorization,
mirroring the reference's functions of the same names:

* ``sp_colorder`` -- SRC/sp_colorder.c:81-221: etree of Pc(A'+A)Pc' (or
  the column etree of A Pc' for MMD_ATA / rectangular A), postorder folded
  into perm_c, column pointers of A Pc'.
* ``symbfact`` -- SRC/symbfact.c:81-215 on A Pc' with rows relabelled by
  perm_c (pdgssvx does the relabelling, SRC/pdgssvx.c:1048-1058): supernode
  partition, L subscripts per supernode, U segments per column.

Both run the C++ code in ``csrc/symbolic.cpp`` (host code: the symbolic
factorization is integer graph search on the host cores, sized by nnz(A)),
the same code the drop-in ``sp_colorder`` / ``symbfact`` symbols of
libslu_mi355x.so run for the reference's pdgssvx.
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from .lib import as_i64p, lib

NATURAL, MMD_ATA, MMD_AT_PLUS_A, MY_PERMC = 0, 1, 2, 7


def last_error():
    e = lib().slu_last_error()
    return e.decode() if e else "unknown error"


def at_plus_a(n, colptr, rowind):
    """Pattern of A'+A without the diagonal as CSR (xadj, adjncy), the graph
    get_perm_c_dist hands to METIS (at_plus_a_dist, SRC/get_perm_c.c:305)."""
    colptr = np.asarray(colptr, np.int64)
    rowind = np.asarray(rowind, np.int64)
    col = np.repeat(np.arange(n, dtype=np.int64), np.diff(colptr))
    r = np.concatenate([rowind, col])
    c = np.concatenate([col, rowind])
    keep = r != c
    key = np.unique(c[keep] * n + r[keep])
    cc, rr = key // n, key % n
    xadj = np.zeros(n + 1, np.int64)
    np.add.at(xadj, cc + 1, 1)
    return np.cumsum(xadj), rr


def metis_nodend(n, xadj, adjncy):
    """The library's METIS_NodeND (nested dissection, csrc/ordering.cpp):
    returns perm_c = iperm (perm_c[i] = new position of column i), as
    get_metis does (SRC/get_perm_c.c:91-97)."""
    xadj = np.ascontiguousarray(xadj, np.int64)
    adjncy = np.ascontiguousarray(adjncy, np.int64)
    nn = np.array([n], np.int64)
    perm = np.zeros(max(n, 1), np.int64)
    iperm = np.zeros(max(n, 1), np.int64)
    null = C.cast(None, C.POINTER(C.c_int64))
    rc = lib().METIS_NodeND(as_i64p(nn), as_i64p(xadj), as_i64p(adjncy) if len(adjncy) else null,
                            null, null, as_i64p(perm), as_i64p(iperm))
    if rc != 1:
        raise RuntimeError(f"METIS_NodeND returned {rc}")
    return iperm[:n], perm[:n]


@dataclass
class ColOrder:
    perm_c: np.ndarray  # postordered column permutation (perm_c[i] = new position of column i)
    etree: np.ndarray   # postordered etree, roots = n
    colbeg: np.ndarray  # A Pc' column j = rowind[colbeg[j]:colend[j]]
    colend: np.ndarray


def sp_colorder(m, n, colptr, rowind, perm_c, colperm=MMD_AT_PLUS_A, fact_dofact=True):
    colptr = np.ascontiguousarray(colptr, np.int64)
    rowind = np.ascontiguousarray(rowind, np.int64)
    pc = np.array(perm_c, np.int64)
    et = np.zeros(n, np.int64)
    cb = np.zeros(n, np.int64)
    ce = np.zeros(n, np.int64)
    if lib().slu_colorder(m, n, as_i64p(colptr), as_i64p(rowind), int(colperm == MMD_ATA),
                          int(fact_dofact), as_i64p(pc), as_i64p(et), as_i64p(cb), as_i64p(ce)):
        raise RuntimeError(last_error())
    return ColOrder(pc, et, cb, ce)


@dataclass
class Symb:
    xsup: np.ndarray
    supno: np.ndarray
    xlsub: np.ndarray
    lsub: np.ndarray
    xusub: np.ndarray
    usub: np.ndarray
    nnzL: int
    nnzU: int
    nnzLU: int
    ret: int  # symbfact's return value: -(lsub size before compression)

    @property
    def nsupers(self):
        return len(self.xsup) - 1


class _SymbHandle:
    """Frees a slu_symbfact result when the last array viewing it is gone."""

    def __init__(self, lib_, h):
        self.lib, self.h = lib_, h

    def __del__(self):
        if self.h:
            self.lib.slu_symbfact_free(self.h)
            self.h = None


def symbfact(m, n, colbeg, colend, rowind, etree, relax, maxsuper):
    """rowind: A Pc''s row indices already relabelled by perm_c."""
    cb = np.ascontiguousarray(colbeg, np.int64)
    ce = np.ascontiguousarray(colend, np.int64)
    ri = np.ascontiguousarray(rowind, np.int64)
    et = np.ascontiguousarray(etree, np.int64)
    L = lib()
    h = L.slu_symbfact(m, n, as_i64p(cb), as_i64p(ce), as_i64p(ri), as_i64p(et), relax, maxsuper)
    if not h:
        raise RuntimeError(last_error())
    # the library's arrays in place (no copy of the GBs of lsub / usub at
    # 100^3): each view's buffer keeps the owner alive, which frees the
    # handle when the last view goes
    sz = np.zeros(7, np.int64)
    L.slu_symbfact_sizes(h, as_i64p(sz))
    ns, nl, nu = int(sz[0]), int(sz[1]), int(sz[2])
    owner = _SymbHandle(L, h)
    ptrs = (C.c_void_p * 6)()
    L.slu_symbfact_views(h, ptrs)

    def view(i, ln):
        buf = (C.c_int64 * max(ln, 0)).from_address(ptrs[i]) if ln and ptrs[i] else (C.c_int64 * 0)()
        buf._owner = owner
        return np.frombuffer(buf, dtype=np.int64)
    xsup, supno, xlsub = view(0, n + 1), view(1, n + 1), view(2, n + 1)
    lsub, xusub, usub = view(3, nl), view(4, n + 1), view(5, nu)
    return Symb(xsup[:ns + 1], supno, xlsub, lsub[:nl], xusub, usub[:nu], int(sz[3]),
                int(sz[4]), int(sz[5]), -int(sz[6]))


def relabel_rows(rowind, perm_c):
    """pdgssvx's Pc relabelling of A Pc''s rows (SRC/pdgssvx.c:1053-1058);
    every entry of A lies in one column of A Pc', so all are relabelled."""
    return np.asarray(perm_c, np.int64)[np.asarray(rowind, np.int64)]
