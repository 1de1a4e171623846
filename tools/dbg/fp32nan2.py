import sys, numpy as np
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/oracle"]
import cases, pyoracle
from superlu_dist_amd.engine import Plan, factor_lustruct
from superlu_dist_amd.frontend import STENCIL_3D27, STENCIL_3D7, Csc, Symbolic, nd_order
for kind, d, dt in [(STENCIL_3D27, 10, 1), (STENCIL_3D7, 10, 1), (STENCIL_3D7, 6, 1)]:
    A = Csc.stencil(kind, d, d, d, dtype=dt)
    S = Symbolic(A, nd_order(d, d, d), 60, 256)
    gpu, ref = S.distribute(), S.distribute()
    info, tiny, st = factor_lustruct(gpu, anorm=12.0)
    o = pyoracle.oracle_factor([ref], 1, 1, A.n, False, 12.0)
    xs = S.xsup
    print("case", kind, d, "nsupers", S.nsupers, "nanL", np.isnan(gpu.Lval).sum(), len(gpu.Lval), "nanU", np.isnan(gpu.Uval).sum(), len(gpu.Uval), "Lvoff", gpu.Lvoff[:S.nsupers+1][-3:], flush=True)
    bad = 0
    for k in range(S.nsupers):
        w = xs[k+1]-xs[k]
        ld = gpu.Lidx[gpu.Loff[k]+1]
        a = gpu.Lval[gpu.Lvoff[k]:gpu.Lvoff[k]+ld*w].reshape(w, ld).T
        r = ref.Lval[ref.Lvoff[k]:ref.Lvoff[k]+ld*w].reshape(w, ld).T
        e = np.abs(a-r)
        if not np.isfinite(a).all() or e.max() > 1e-4*np.abs(r).max():
            nanr = np.argwhere(~np.isfinite(a))
            print(f" sn {k} w {w} ld {ld} nan {(~np.isfinite(a)).sum()} diag-nan {(~np.isfinite(a[:w])).sum()} maxerr(finite) {np.nanmax(np.where(np.isfinite(e), e, 0)):.3e} first nan {nanr[:3].tolist()}", flush=True)
            if not np.isfinite(a[:w]).all() or True:
                print("  gpu diag\n", a[:min(w,6), :min(w,6)], "\n  ref\n", r[:min(w,6), :min(w,6)], flush=True)
            bad += 1
            if bad > 3: break
