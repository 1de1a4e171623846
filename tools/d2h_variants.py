"""A/B of the drop-in's D2H pipeline knobs on the cached (SamePattern_SameRowPerm)
pdgstrf at 100^3, in one process: the D2H stream priority (SLU_D2H_PRIO) and
the push kernel's workgroups (SLU_D2H_WG), read by the engine at every call.
usage: python tools/d2h_variants.py [nx]   (one line per variant and repetition)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superlu_dist_amd import capi  # noqa: E402
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order  # noqa: E402


def main():
    nx = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx, dtype=0)
    S = Symbolic(A, nd_order(nx, nx, nx), 60, 256, reference=True)
    lu = S.distribute()
    L0, U0 = lu.Lval.copy(), lu.Uval.copy()
    opt = capi.default_options()

    def call(fact):
        lu.Lval[:] = L0
        lu.Uval[:] = U0
        opt.Fact = fact
        t = time.perf_counter()
        rv, info, _ = capi.pxgstrf(lu, 12.0, options=opt)
        assert rv == 0 and info == 0
        return (time.perf_counter() - t) * 1e3

    print("first call %.1f ms" % call(0), flush=True)
    for rep in range(2):
        for prio in ("lo", "hi"):
            for wg in ("32", "128"):
                os.environ["SLU_D2H_PRIO"] = prio
                os.environ["SLU_D2H_WG"] = wg
                print("rep %d prio %s wg %s: %.1f ms" % (rep, prio, wg, call(2)), file=sys.stderr,
                      flush=True)


if __name__ == "__main__":
    main()
