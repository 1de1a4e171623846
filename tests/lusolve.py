"""Host-side supernodal triangular solves on a factored 1x1 LUstruct (test
helper for backward-error checks), and the coordinate maps of pdgssvx's
solve (SRC/pdgssvx.c): the LUstruct factors Pc Pr diag(R) A diag(C) Pc^T."""
import numpy as np
from scipy.linalg import solve_triangular


def solve_1x1(lu, b):
    """Solve (P A P^T) x = b with the factors held in lu (1x1 grid)."""
    xs = lu.xsup
    x = np.array(b, dtype=np.result_type(lu.Lval.dtype, np.float64 if lu.Lval.dtype != np.complex128 else np.complex128)).copy()
    ns = lu.nsupers
    cols = []
    for k in range(ns):
        w = xs[k + 1] - xs[k]
        idx = lu.Lidx[lu.Loff[k]:]
        ld = idx[1]
        blk = lu.Lval[lu.Lvoff[k]:lu.Lvoff[k] + ld * w].reshape(w, ld).T
        rows, p = [], 2
        for _ in range(idx[0]):
            nr = idx[p + 1]
            rows.extend(idx[p + 2:p + 2 + nr])
            p += 2 + nr
        cols.append((blk, np.array(rows)))
    for k in range(ns):  # forward: L y = b
        f, l = xs[k], xs[k + 1]
        blk, rows = cols[k]
        w = l - f
        x[f:l] = solve_triangular(blk[:w], x[f:l], lower=True, unit_diagonal=True)
        if len(rows) > w:
            x[rows[w:]] -= blk[w:] @ x[f:l]
    for k in range(ns - 1, -1, -1):  # backward: U x = y
        f, l = xs[k], xs[k + 1]
        blk, rows = cols[k]
        w = l - f
        if lu.Uoff[k] >= 0:
            idx = lu.Uidx[lu.Uoff[k]:]
            v = lu.Uval[lu.Uvoff[k]:]
            p, q = 3, 0
            for _ in range(idx[0]):
                jb = idx[p]
                for c in range(xs[jb + 1] - xs[jb]):
                    fst = idx[p + 2 + c]
                    seg = l - fst
                    if seg:
                        x[fst:l] -= v[q:q + seg] * x[xs[jb] + c]
                    q += seg
                p += 2 + xs[jb + 1] - xs[jb]
        x[f:l] = solve_triangular(blk[:w], x[f:l], lower=False)
    return x


def backward_error(A, perm, x_perm, b_perm):
    """||B x - b|| / (||B|| ||x||) (inf norms) for B = P A P^T."""
    B = A.permuted(perm)
    cp, ri, v = B.arrays()
    n = B.n
    r = -np.asarray(b_perm, dtype=np.result_type(v, x_perm)).copy()
    absrow = np.zeros(n)
    for j in range(n):
        sl = slice(cp[j], cp[j + 1])
        r[ri[sl]] += v[sl] * x_perm[j]
        absrow[ri[sl]] += np.abs(v[sl])
    return float(np.abs(r).max() / (absrow.max() * np.abs(x_perm).max()))


def to_lu_coords(b, perm_r, perm_c, R=None):
    """b (original row order) -> Pc Pr diag(R) b, the right-hand side of the
    factored system (row i of A is row perm_c[perm_r[i]] of the LUstruct)."""
    b = np.asarray(b)
    bb = b * (R if R is not None else 1.0)
    out = np.empty_like(bb)
    out[perm_c[perm_r]] = bb
    return out


def from_lu_coords(y, perm_c, C=None):
    """Solution of the factored system -> x = diag(C) Pc^T y."""
    x = np.asarray(y)[perm_c]
    return x * (C if C is not None else 1.0)


def lu_coords_matrix(fx):
    """CSC (colptr, rowind, values) of Pc Pr diag(R) A diag(C) Pc^T from a
    refdump fixture: pdgssvx leaves its local A scaled and with perm_c
    applied to the column indices (SRC/pdgssvx.c:1140); rows are mapped here.
    On a grid the ranks' row slices (NRformat_loc, rows fst_row .. fst_row +
    m_loc) are put back together."""
    order = sorted(range(fx.nranks), key=lambda p: fx.meta["ranks"][p]["fst_row"])
    rps, cis, avs, rws = [], [], [], []
    for p in order:
        rp = fx.arr(p, "A_rowptr")
        rws.append(fx.meta["ranks"][p]["fst_row"] + np.repeat(np.arange(len(rp) - 1), np.diff(rp)))
        cis.append(fx.arr(p, "A_colind"))
        avs.append(fx.arr(p, "A_val"))
    ci, av, grow = np.concatenate(cis), np.concatenate(avs), np.concatenate(rws)
    pr, pc = fx.arr(0, "perm_r"), fx.arr(0, "perm_c")
    n = fx.n
    rows = pc[pr[grow]]
    order = np.lexsort((rows, ci))
    cols_sorted = ci[order]
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(colptr, cols_sorted + 1, 1)
    colptr = np.cumsum(colptr)
    return colptr, rows[order].astype(np.int64), av[order]


def _lcol(lu, k, pc):
    """Local L column block of supernode k on this rank: (values nsupr x w,
    global rows, number of diagonal-block rows on top)."""
    ljb = k // pc
    if ljb >= len(lu.Loff) or lu.Loff[ljb] < 0:
        return None
    xs = lu.xsup
    w = xs[k + 1] - xs[k]
    idx = lu.Lidx[lu.Loff[ljb]:]
    ld = idx[1]
    blk = lu.Lval[lu.Lvoff[ljb]:lu.Lvoff[ljb] + ld * w].reshape(w, ld).T
    rows, p, top = [], 2, 0
    for _ in range(idx[0]):
        gb, nr = idx[p], idx[p + 1]
        if gb == k:
            top = nr
        rows.extend(idx[p + 2:p + 2 + nr])
        p += 2 + nr
    return blk, np.array(rows, dtype=np.int64), top


def solve_grid_sim(lus, pr, pc, b, fwd_only=False):
    """The distributed solve of the engine's 2D-grid path (engine.hip
    sweep_2d; pdgstrs's lsum scheme, SRC/pdgstrs.c) simulated over all ranks'
    LUstructs with one x vector per rank: block row k's partial sums live on
    process row k % pr and are added on the diagonal owner; the solved piece
    goes down the owner's process column.  Elimination order k = 0..ns-1 is
    one topological order of the engine's levels.  Returns x (full)."""
    ns = lus[0].nsupers
    xs = lus[0].xsup
    P = pr * pc
    dt = np.result_type(lus[0].Lval.dtype, np.float64)
    own = lambda k: (k % pr) * pc + k % pc  # noqa: E731
    x = [np.zeros(len(b), dtype=dt) for _ in range(P)]
    for k in range(ns):
        x[own(k)][xs[k]:xs[k + 1]] = b[xs[k]:xs[k + 1]]
    lcols = [{k: _lcol(lus[p], k, pc) for k in range(ns) if k % pc == p % pc} for p in range(P)]

    def reduce(k):
        f, l, o = xs[k], xs[k + 1], own(k)
        for c in range(pc):
            s = (k % pr) * pc + c
            if s != o:
                x[o][f:l] += x[s][f:l]

    def bcast(k):
        f, l, o = xs[k], xs[k + 1], own(k)
        for r in range(pr):
            x[r * pc + k % pc][f:l] = x[o][f:l]

    for k in range(ns):  # L y = b
        f, l, o = xs[k], xs[k + 1], own(k)
        w = l - f
        reduce(k)
        blk, rows, top = lcols[o][k]
        x[o][f:l] = solve_triangular(blk[:w], x[o][f:l], lower=True, unit_diagonal=True)
        bcast(k)
        for r in range(pr):
            p = r * pc + k % pc
            c = lcols[p].get(k)
            if c is None:
                continue
            blk, rows, top = c
            if len(rows) > top:
                x[p][rows[top:]] -= blk[top:] @ x[p][f:l]
    if fwd_only:
        out = np.empty(len(b), dtype=dt)
        for k in range(ns):
            out[xs[k]:xs[k + 1]] = x[own(k)][xs[k]:xs[k + 1]]
        return out
    for p in range(P):  # rows a rank does not own start the backward sweep at zero
        for k in range(ns):
            if own(k) != p:
                x[p][xs[k]:xs[k + 1]] = 0
    for k in range(ns - 1, -1, -1):  # U x = y
        f, l, o = xs[k], xs[k + 1], own(k)
        w = l - f
        for c in range(pc):
            p = (k % pr) * pc + c
            lu = lus[p]
            lb = k // pr
            if lb >= len(lu.Uoff) or lu.Uoff[lb] < 0:
                continue
            idx = lu.Uidx[lu.Uoff[lb]:]
            v = lu.Uval[lu.Uvoff[lb]:]
            q, qq = 3, 0
            for _ in range(idx[0]):
                jb = idx[q]
                for cc in range(xs[jb + 1] - xs[jb]):
                    fst = idx[q + 2 + cc]
                    seg = l - fst
                    if seg:
                        x[p][fst:l] -= v[qq:qq + seg] * x[p][xs[jb] + cc]
                    qq += seg
                q += 2 + xs[jb + 1] - xs[jb]
        reduce(k)
        blk, rows, top = lcols[o][k]
        x[o][f:l] = solve_triangular(blk[:w], x[o][f:l], lower=False)
        bcast(k)
    out = np.empty(len(b), dtype=dt)
    for k in range(ns):
        out[xs[k]:xs[k + 1]] = x[own(k)][xs[k]:xs[k + 1]]
    return out


def lu_coords_matrix_from_lus(lus, pr, pc):
    """CSC of A in the LUstruct's coordinates read off the pre-factor
    LUstructs of all ranks of a pr x pc grid (pddistribute scatters A's
    entries into zero-initialised L and U blocks, so the nonzeros of the
    pre-factor blocks are A's).  For grid fixtures, whose dumped local A is
    in pdgsmv's compressed column numbering."""
    xs = lus[0].xsup
    ns = lus[0].nsupers
    R, Cc, V = [], [], []
    for p, lu in enumerate(lus):
        myrow, mycol = p // pc, p % pc
        for ljb in range(len(lu.Loff)):
            k = ljb * pc + mycol
            if k >= ns or lu.Loff[ljb] < 0:
                continue
            c = _lcol(lu, k, pc)
            blk, rows, _ = c
            for j in range(blk.shape[1]):
                nz = np.nonzero(blk[:, j])[0]
                R.extend(rows[nz]); Cc.extend([xs[k] + j] * len(nz)); V.extend(blk[nz, j])
        for lb in range(len(lu.Uoff)):
            k = lb * pr + myrow
            if k >= ns or lu.Uoff[lb] < 0:
                continue
            idx = lu.Uidx[lu.Uoff[lb]:]
            v = lu.Uval[lu.Uvoff[lb]:]
            l = xs[k + 1]
            q, qq = 3, 0
            for _ in range(idx[0]):
                jb = idx[q]
                for cc in range(xs[jb + 1] - xs[jb]):
                    fst = idx[q + 2 + cc]
                    seg = v[qq:qq + l - fst]
                    nz = np.nonzero(seg)[0]
                    R.extend(fst + nz); Cc.extend([xs[jb] + cc] * len(nz)); V.extend(seg[nz])
                    qq += l - fst
                q += 2 + xs[jb + 1] - xs[jb]
    R, Cc, V = np.array(R, dtype=np.int64), np.array(Cc, dtype=np.int64), np.array(V)
    order = np.lexsort((R, Cc))
    n = len(lus[0].supno) if hasattr(lus[0], "supno") else int(xs[-1])
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(colptr, Cc[order] + 1, 1)
    return np.cumsum(colptr), R[order], V[order].astype(lus[0].Lval.dtype)
