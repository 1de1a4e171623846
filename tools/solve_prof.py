"""Device fill + triangular solve on the 100^3 Laplacian (SURVEY 8(f) rows
1-2), for rocprofv3 --kernel-trace --stats: one plan, one device fill from A,
one factorization, then --solves solves of one right-hand side."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superlu_dist_amd.engine import Plan  # noqa: E402
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=100)
    ap.add_argument("--solves", type=int, default=3)
    ap.add_argument("--nrhs", type=int, default=1)
    a = ap.parse_args()
    A = Csc.stencil(STENCIL_3D7, a.nx, a.nx, a.nx)
    S = Symbolic(A, nd_order(a.nx, a.nx, a.nx), 60, 256)
    p = Plan(S.distribute(), timing=1)
    cp, ri, v = A.permuted(S.perm_c).arrays()
    p.set_a_pattern(cp, ri)
    p.fill_a(v)
    fill = p.stats()["t_fill_ms"]
    assert p.factor(12.0) == (0, 0)
    p.sync()
    xt = np.random.default_rng(1).standard_normal(A.n)
    import scipy.sparse as sp
    B = sp.csc_matrix((v, ri, cp), shape=(A.n, A.n))
    b = B @ xt
    ts = []
    for _ in range(a.solves):
        t0 = time.perf_counter()
        x = p.solve(b) if a.nrhs == 1 else p.solve(np.repeat(b[:, None], a.nrhs, axis=1))[:, 0]
        ts.append((time.perf_counter() - t0) * 1e3, )
        dev = p.stats()["t_solve_ms"]
    berr = float(np.abs(B @ x - b).max() / (abs(B).sum(axis=1).max() * np.abs(x).max()))
    print(json.dumps({"nx": a.nx, "nrhs": a.nrhs, "fill_ms": fill, "solve_ms_device": dev,
                      "solve_ms_wall": min(ts), "berr": berr,
                      "fwd_err": float(np.abs(x - xt).max())}), flush=True)


if __name__ == "__main__":
    main()
