"""Diagnostics: the 2D-grid device solve of one refdump fixture against the
host simulation of the same algorithm (tests/lusolve.solve_grid_sim), forward
sweep only (SLU_SV_FWD_ONLY) and full; prints the first supernodes that differ.
usage: python tools/dbg_grid_solve.py NAME"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from gridrun import run_grid  # noqa: E402
from lusolve import solve_grid_sim, to_lu_coords  # noqa: E402
from refdump import Fixture  # noqa: E402


def main():
    name = sys.argv[1]
    fx = Fixture(name)
    b, R, C, perm_r, perm_c, _, _ = fx.full_rhs()
    bl = to_lu_coords(b, perm_r, perm_c, R)
    xs = fx.arr(0, "xsup")
    for fwd in (True, False):
        if fwd:
            os.environ["SLU_SV_FWD_ONLY"] = "1"
        else:
            os.environ.pop("SLU_SV_FWD_ONLY", None)
        ref = solve_grid_sim(fx.lus("post"), fx.pr, fx.pc, bl, fwd_only=fwd)
        with tempfile.TemporaryDirectory() as d:
            out = run_grid(f"refdump:{name}", fx.pr, fx.pc, d, device=0, solve=True)
        # undo the test's from_lu_coords: x = C * y[perm_c]
        for p, o in enumerate(out):
            y = np.empty_like(ref)
            y[perm_c] = o["x"] / (C if C is not None else 1.0)
            bad = [k for k in range(len(xs) - 1)
                   if np.abs(y[xs[k]:xs[k + 1]] - ref[xs[k]:xs[k + 1]]).max() > 1e-8 * np.abs(ref).max()]
            print(f"{'fwd' if fwd else 'full'} rank {p}: {len(bad)} wrong supernodes, first {bad[:8]}, "
                  f"owners {[((k % fx.pr), (k % fx.pc)) for k in bad[:8]]}", flush=True)


if __name__ == "__main__":
    main()
