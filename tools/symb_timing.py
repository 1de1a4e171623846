"""Times the column ordering post-pass + symbolic factorization: the
REFERENCE (oracle/_ref/symb_dump: SRC/sp_colorder.c + SRC/symbfact.c, as
pdgssvx runs them) against libslu_mi355x.so's restatement, on the 3D 7-pt
Laplacian k^3 with the reference's MMD_AT_PLUS_A perm_c, and checks that
every output array is identical at that size.  Host only.

    python tools/symb_timing.py [k ...]        (default 60 100)
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle", "gen"))

from make_symb_golden import MMD_AT_PLUS_A, read_dump, run  # noqa: E402
from superlu_dist_amd import symbolic as S  # noqa: E402


def lap3d(k):
    n = k ** 3
    idx = np.arange(n).reshape(k, k, k)
    rows, cols = [idx.ravel()], [idx.ravel()]
    for ax in range(3):
        for s in (-1, 1):
            a = np.roll(idx, s, axis=ax)
            m = np.ones_like(idx, bool)
            sl = [slice(None)] * 3
            sl[ax] = 0 if s == 1 else -1
            m[tuple(sl)] = False
            rows.append(a[m])
            cols.append(idx[m])
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    o = np.lexsort((r, c))
    r, c = r[o], c[o]
    colptr = np.zeros(n + 1, np.int64)
    np.add.at(colptr, c + 1, 1)
    return n, np.cumsum(colptr), r.astype(np.int64)


def main(ks):
    out = []
    for k in ks:
        n, colptr, rowind = lap3d(k)
        cols = [rowind[colptr[j]:colptr[j + 1]] for j in range(n)]
        d, (t_perm, t_col, t_sym) = run(f"lap3d{k}", n, cols, MMD_AT_PLUS_A, 60, 256)
        t0 = time.perf_counter()
        co = S.sp_colorder(n, n, colptr, rowind, d["perm_c_in"], MMD_AT_PLUS_A)
        t1 = time.perf_counter()
        ri = S.relabel_rows(rowind, co.perm_c)
        t2 = time.perf_counter()
        sb = S.symbfact(n, n, co.colbeg, co.colend, ri, co.etree, 60, 256)
        t3 = time.perf_counter()
        same = (np.array_equal(co.perm_c, d["perm_c"]) and np.array_equal(co.etree, d["etree"])
                and np.array_equal(sb.xsup, d["xsup"][:sb.nsupers + 1])
                and np.array_equal(sb.lsub, d["lsub"]) and np.array_equal(sb.usub, d["usub"])
                and np.array_equal(sb.xlsub, d["xlsub"]) and np.array_equal(sb.xusub, d["xusub"])
                and sb.ret == int(d["scalars"][0]))
        rec = {"k": k, "n": n, "nsupers": sb.nsupers, "lsub": len(sb.lsub), "usub": len(sb.usub),
               "ref_colperm_mmd_s": t_perm, "ref_sp_colorder_s": t_col, "ref_symbfact_s": t_sym,
               "ours_sp_colorder_s": t1 - t0, "ours_symbfact_s": t3 - t2,
               "identical": bool(same), "threads": 1}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [60, 100])
