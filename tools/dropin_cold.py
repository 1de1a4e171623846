"""The drop-in pdgstrf's first call in a COLD process, as pddrive sees it:
no torch, no HIP before the call (runtime initialisation, fresh HBM and the
pinned pools are all inside utime[FACT]), then the SamePattern_SameRowPerm
refactorization.  usage: python tools/dropin_cold.py [nx]  (one JSON line)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superlu_dist_amd import capi  # noqa: E402
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order  # noqa: E402


def main():
    nx = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    t = time.perf_counter()
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx, dtype=0)
    S = Symbolic(A, nd_order(nx, nx, nx), 60, 256, reference=True)
    lu = S.distribute()
    t_setup = time.perf_counter() - t
    L0, U0 = lu.Lval.copy(), lu.Uval.copy()
    opt = capi.default_options()
    walls = []
    for fact in (0, 2):
        lu.Lval[:] = L0
        lu.Uval[:] = U0
        opt.Fact = fact
        t = time.perf_counter()
        rv, info, _ = capi.pxgstrf(lu, 12.0, options=opt)
        walls.append((time.perf_counter() - t) * 1e3)
        assert rv == 0 and info == 0, (rv, info)
    print(json.dumps({"nx": nx, "nsupers": int(S.nsupers), "setup_s": round(t_setup, 1),
                      "utime_fact_ms_cold_first_call": round(walls[0], 1),
                      "utime_fact_ms_samepattern_samerowperm": round(walls[1], 1)}))


if __name__ == "__main__":
    main()
