import sys, numpy as np
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/oracle"]
import cases, pyoracle
from superlu_dist_amd.engine import Plan, factor_lustruct
from superlu_dist_amd.frontend import STENCIL_3D27, STENCIL_3D7, Csc, Symbolic, nd_order
for kind, d, dt in [(STENCIL_3D27, 10, 1), (STENCIL_3D27, 12, 1), (STENCIL_3D7, 10, 1), (STENCIL_3D27, 10, 0)]:
    A = Csc.stencil(kind, d, d, d, dtype=dt)
    S = Symbolic(A, nd_order(d, d, d), 60, 256)
    gpu, ref = S.distribute(), S.distribute()
    info, tiny, st = factor_lustruct(gpu, anorm=12.0)
    o = pyoracle.oracle_factor([ref], 1, 1, A.n, False, 12.0)
    print(kind, d, dt, "info", info, o["info"], "nan gpu", np.isnan(gpu.Lval).sum(), np.isnan(gpu.Uval).sum(),
          "nan ref", np.isnan(ref.Lval).sum(), np.isnan(ref.Uval).sum(),
          "err", cases.factor_error([gpu], [(ref.Lval, ref.Uval)]), flush=True)
