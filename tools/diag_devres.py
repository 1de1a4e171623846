"""GPU diagnostic (not a test): the device-resident drop-in sequence of
bench.py's leg at a small size, with the factors written back
(SUPERLU_MI355X_HOST_FACTORS=1) and compared per block with the oracle's
factors of the same LUstruct built by the front-end (reference symbolic)."""
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from superlu_dist_amd import capi  # noqa: E402
from superlu_dist_amd import symbolic as SY  # noqa: E402
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order  # noqa: E402

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 12
os.environ["SUPERLU_MI355X_TIMING"] = "1"
A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
n = A.n
cp, ri, v = A.arrays()
co = SY.sp_colorder(n, n, cp, ri, nd_order(nx, nx, nx), SY.MY_PERMC)
sb = SY.symbfact(n, n, co.colbeg, co.colend, SY.relabel_rows(ri, co.perm_c), co.etree, 60, 256)
xt = np.random.default_rng(0).standard_normal(n)
b = sp.csc_matrix((v, ri, cp), shape=(n, n)) @ xt
import ctypes as C  # noqa: E402
from superlu_dist_amd.engine import factor_lustruct  # noqa: E402
from superlu_dist_amd.lib import SluLuView, lib  # noqa: E402


def values(s):
    vw = SluLuView()
    lib().slu_lu_get_view(C.addressof(s.lu), 0, C.byref(vw))
    Lv = np.frombuffer((C.c_char * (vw.Lval_cnt * 8)).from_address(vw.Lval), dtype=np.float64).copy()
    Uv = np.frombuffer((C.c_char * (vw.Uval_cnt * 8)).from_address(vw.Uval), dtype=np.float64).copy()
    return Lv, Uv


S = Symbolic(A, nd_order(nx, nx, nx), 60, 256, reference=True)
lu = S.distribute(1, 1, 0, 0)
L0, U0 = lu.Lval.copy(), lu.Uval.copy()
info, tiny, st = factor_lustruct(lu, anorm=12.0)
print("engine on the front-end LUstruct: info", info, flush=True)
for host_factors in ("0", "1"):
    os.environ["SUPERLU_MI355X_HOST_FACTORS"] = host_factors
    s = capi.DeviceResidentSystem(n, cp, co.perm_c[ri], v, co.perm_c, co.etree, sb.xsup, sb.supno,
                                  sb.xlsub, sb.lsub, sb.xusub, sb.usub, 12.0)
    s.distribute(0)
    Lv, Uv = values(s)
    print(f"after pddistribute: sizes {len(Lv)}/{len(L0)} {len(Uv)}/{len(U0)}; max |d| vs front-end "
          f"L {np.abs(Lv - L0).max() if len(Lv) == len(L0) else -1:.3e} "
          f"U {np.abs(Uv - U0).max() if len(Uv) == len(U0) else -1:.3e}", flush=True)
    rv, info, ops = s.factor()
    if host_factors == "1":
        Lv, Uv = values(s)
        print(f"factors vs engine on the front-end LUstruct: L {np.abs(Lv - lu.Lval).max():.3e} "
              f"U {np.abs(Uv - lu.Uval).max():.3e}", flush=True)
    x = s.solve(b)
    print(f"host_factors={host_factors}: rv {rv} info {info} ops {ops:.3e} fwd err "
          f"{np.abs(x - xt).max() / np.abs(xt).max():.3e}", flush=True)
