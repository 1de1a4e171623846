"""Times the restated symbfact at k^3 (3D 7-point Laplacian, nested
dissection) and hashes its arrays: run with SLU_SYMB_TASKS=0 / 1 to compare
the column-order search with the subtree tasks.  usage: python tools/symb_tasks_timing.py k"""
import os, sys, time, hashlib
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from superlu_dist_amd import symbolic as SY
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, nd_order
k = int(sys.argv[1])
A = Csc.stencil(STENCIL_3D7, k, k, k)
cp, ri, _ = A.arrays()
co = SY.sp_colorder(A.n, A.n, cp, ri, nd_order(k, k, k), SY.MY_PERMC)
rr = SY.relabel_rows(ri, co.perm_c)
t = time.perf_counter()
sb = SY.symbfact(A.n, A.n, co.colbeg, co.colend, rr, co.etree, 60, 256)
dt = time.perf_counter() - t
h = hashlib.sha1()
for f in ("xsup", "supno", "xlsub", "lsub", "xusub", "usub"):
    h.update(np.ascontiguousarray(getattr(sb, f)).tobytes())
print("symbfact %.3f s" % dt, h.hexdigest(), sb.ret, sb.nnzLU)
