"""Drop-in path on the amalgamated plan (reference structure, 1x1): where the
time of upload / factor / download goes, with and without the overlapped
D2H.  Diagnostics only (not the bench)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from superlu_dist_amd.engine import Plan  # noqa: E402
from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order  # noqa: E402

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 100
A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
S = Symbolic(A, nd_order(nx, nx, nx), 60, 256, reference=True)
lu = S.distribute(1, 1, 0, 0)
L0, U0 = lu.Lval.copy(), lu.Uval.copy()
out = {}
modes = (False, True, True) if len(sys.argv) < 3 else tuple(m == "1" for m in sys.argv[2].split(","))
for overlap in modes:
    lu.Lval[:] = L0
    lu.Uval[:] = U0
    t0 = time.perf_counter()
    p = Plan(lu, overlap_upload=overlap, overlap_download=overlap)
    t1 = time.perf_counter()
    p.upload()
    t2 = time.perf_counter()
    p.factor(12.0)
    t3 = time.perf_counter()
    p.download()
    t4 = time.perf_counter()
    st = p.stats()
    out[f"overlap={overlap}"] = {k: round(v, 1) for k, v in {
        "plan_ms": (t1 - t0) * 1e3, "upload_ms": (t2 - t1) * 1e3, "factor_ms": (t3 - t2) * 1e3,
        "download_ms": (t4 - t3) * 1e3, "t_amalg_ms": st["t_amalg_ms"],
        "t_expand_ms": st["t_expand_ms"], "t_compress_ms": st["t_compress_ms"],
        "t_upload_ms": st["t_upload_ms"], "t_d2h_ms": st["t_d2h_ms"],
        "t_d2h_tail_ms": st["t_d2h_tail_ms"], "n_d2h_copies": st["n_d2h_copies"]}.items()}
    print(json.dumps(out[f"overlap={overlap}"]), flush=True)
    del p
