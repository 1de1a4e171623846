"""Generates tests/golden/refdump_<case>.npz: LUstructs built by the
REFERENCE's own front-end (p?gssvx: equilibration, MC64, MMD ordering,
symbfact, pddistribute) before and after the REFERENCE factorization, plus
the reference's solve / refinement results, dumped by oracle/_ref/ref_dump
(gen/ref_dump_main.c).

Run here (needs /root/reference, conda MPICH and MKL; `make -C oracle ref`):
    python oracle/gen/make_refdump.py [case ...]
TEST INFRASTRUCTURE.  Each fixture holds, per rank p, arrays "r{p}_<name>"
(xsup, supno, Lidx/Loff/Lvoff, Uidx/Uoff/Uvoff, pre_/post_ L/U values,
ToRecv/ToSendD/ToSendR, bufmax, perm_r, perm_c, R, C, b, x, x_norefine,
xtrue, berr, A_rowptr/A_colind/A_val) and "meta" (JSON list, one per rank).
"""
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
MATRICES = os.path.join(GOLDEN, "matrices")
DUMP = os.path.join(REPO, "oracle", "_ref", "ref_dump")
CONDA = "/opt/conda"
sys.path.insert(0, REPO)


def write_mtx(path, n, rows, cols, vals):
    cplx = np.iscomplexobj(vals)
    with open(path, "w") as fh:
        fh.write(f"%%MatrixMarket matrix coordinate {'complex' if cplx else 'real'} general\n")
        fh.write(f"{n} {n} {len(vals)}\n")
        for r, c, v in zip(rows, cols, vals):
            if cplx:
                fh.write(f"{r + 1} {c + 1} {v.real:.17g} {v.imag:.17g}\n")
            else:
                fh.write(f"{r + 1} {c + 1} {v:.17g}\n")


def convdiff2d(nx, beta=2.0, seed=7):
    """Upwind convection-diffusion on an nx x nx grid with a second-order
    upwind term on the west side only (structurally unsymmetric), rows
    scrambled by a fixed random permutation: MC64 (RowPerm = LargeDiag_MC64)
    must find a non-identity perm_r to put the large entries back on the
    diagonal."""
    n = nx * nx
    R, Cc, V = [], [], []
    for i in range(nx):
        for j in range(nx):
            r = i * nx + j
            ent = {r: 4.0 + beta}
            if j > 0:
                ent[r - 1] = -1.0 - beta
            if j > 1:
                ent[r - 2] = 0.25 * beta
            if j < nx - 1:
                ent[r + 1] = -1.0
            if i > 0:
                ent[r - nx] = -1.0
            if i < nx - 1:
                ent[r + nx] = -1.0 + 0.1 * beta
            for c, v in ent.items():
                R.append(r)
                Cc.append(c)
                V.append(v)
    p = np.random.default_rng(seed).permutation(n)
    return n, p[np.array(R)], np.array(Cc), np.array(V)


def isolated_zero_pivots(nx):
    """2D 5-point Laplacian (nx x nx) plus two isolated unknowns whose only
    entry is an explicit zero on the diagonal: two exactly zero pivots in
    supernodes that do not depend on each other (or on the Laplacian), so
    which of them pdgstrf reports in *info depends on the elimination order
    (SRC/pdgstrf2.c:246-247 overwrite, SRC/pdgstrf.c:1927-1931 MIN)."""
    m = nx * nx
    R, Cc, V = [0], [0], [0.0]  # unknown 0: isolated, explicit zero diagonal
    for i in range(nx):
        for j in range(nx):
            r = i * nx + j
            for c, v in ((r, 4.0), (r - 1 if j else -1, -1.0), (r + 1 if j < nx - 1 else -1, -1.0),
                         (r - nx, -1.0), (r + nx if i < nx - 1 else -1, -1.0)):
                if 0 <= c < m:
                    R.append(r + 1)
                    Cc.append(c + 1)
                    V.append(v)
    R.append(m + 1)  # unknown m+1: isolated, explicit zero diagonal
    Cc.append(m + 1)
    V.append(0.0)
    return m + 2, np.array(R), np.array(Cc), np.array(V)


def tiny_pivot(nx):
    """2D Laplacian whose (0,0) entry is 1e-14: with ReplaceTinyPivot the
    reference replaces it by sqrt(eps)*anorm-level thresh (SRC/pdgstrf2.c:217-
    232) and counts it in stat->TinyPivots."""
    n, R, Cc, V = isolated_zero_pivots(nx)
    keep = (R != 0) & (R != n - 1)
    R, Cc, V = R[keep] - 1, Cc[keep] - 1, V[keep]
    V = V.copy()
    V[(R == 0) & (Cc == 0)] = 1e-14
    return nx * nx, R, Cc, V


def stencil_mtx(kind, dims, dtype):
    from superlu_dist_amd.frontend import Csc
    kw = dict(diag=6 - 0.25, diag_im=-0.0025) if dtype == 2 else {}
    A = Csc.stencil(kind, *dims, dtype=dtype, **kw)
    cp, ri, v = A.arrays()
    cols = np.repeat(np.arange(A.n), np.diff(cp))
    return A.n, ri, cols, v


def nd_perm(dims):
    from superlu_dist_amd.frontend import nd_order
    return nd_order(*dims)


# name: (matrix source, dtype char, grid, ref_dump options)
#   matrix source: "file:<name>" in tests/golden/matrices, or a callable
#   returning (n, rows, cols, vals) written as .mtx
CASES = {
    # the reference's own test matrices with pddrive's defaults
    # (Equil, LargeDiag_MC64, MMD_AT_PLUS_A: METIS is not in the image)
    "big_1x1_d": ("file:big.rua", "d", (1, 1), {}),
    "big_2x2_d": ("file:big.rua", "d", (2, 2), {}),
    "big_1x2_s": ("file:big.rua", "s", (1, 2), {}),
    # TEST/CMakeLists.txt: relax 8, maxsup 20 on g20, grids up to 5x3
    "g20_2x3_small_d": ("file:g20.rua", "d", (2, 3), {"-x": 8, "-m": 20}),
    "g20_1x1_d": ("file:g20.rua", "d", (1, 1), {}),
    "g20_2x2_s": ("file:g20.rua", "s", (2, 2), {}),
    "cg20_2x2_z": ("file:cg20.cua", "z", (2, 2), {}),
    "cg20_1x1_z": ("file:cg20.cua", "z", (1, 1), {}),
    # structurally unsymmetric, rows scrambled: MC64 perm_r != identity
    "cd2d_24_1x1_d": (lambda: convdiff2d(24), "d", (1, 1), {}),
    "cd2d_24_2x2_d": (lambda: convdiff2d(24), "d", (2, 2), {"-x": 8, "-m": 24}),
    "cd2d_20_2x1_z": (lambda: convdiff2d(20), "z", (2, 1), {}),
    # BASELINE stencils through the reference front-end with our ND order
    # (ColPerm = MY_PERMC, the METIS stand-in of SURVEY 7 hard part 7)
    "lap3d_12_2x2_d": (lambda: stencil_mtx(1, (12, 12, 12), 0), "d", (2, 2),
                       {"perm": (12, 12, 12)}),
    "lap3d_10_1x1_mmd_d": (lambda: stencil_mtx(1, (10, 10, 10), 0), "d", (1, 1), {}),
    # pivot edge cases: no row permutation, no equilibration
    "zeropiv2_1x1_d": (lambda: isolated_zero_pivots(8), "d", (1, 1), {"-p": 0, "-e": 0}),
    "zeropiv2_2x2_d": (lambda: isolated_zero_pivots(8), "d", (2, 2), {"-p": 0, "-e": 0}),
    "tinypiv_1x1_d": (lambda: tiny_pivot(8), "d", (1, 1), {"-p": 0, "-e": 0, "-y": 1}),
}


def make(name):
    src, dt, (pr, pc), opts = CASES[name]
    tmp = tempfile.mkdtemp(prefix="slu_refdump_")
    try:
        if isinstance(src, str):
            mfile = os.path.join(MATRICES, src[5:])
        else:
            n, R, Cc, V = src()
            if dt == "z":
                V = V.astype(np.complex128) * (1.0 + 0.05j)
            mfile = os.path.join(tmp, "A.mtx")
            write_mtx(mfile, n, R, Cc, V)
        out = os.path.join(tmp, "out")
        os.makedirs(out)
        cmd = [os.path.join(CONDA, "bin", "mpiexec"), "-n", str(pr * pc), DUMP, "-t", dt,
               "-o", out, "-r", str(pr), "-c", str(pc)]
        for k, v in opts.items():
            if k == "perm":
                pf = os.path.join(tmp, "perm.bin")
                nd_perm(v).astype(np.int64).tofile(pf)
                cmd += ["-P", pf]
            else:
                cmd += [k, str(v)]
        cmd.append(mfile)
        env = dict(os.environ)
        env.update({"MPICH_CC": "gcc", "OMP_NUM_THREADS": "1", "MKL_NUM_THREADS": "1",
                    "MKL_THREADING_LAYER": "SEQUENTIAL",
                    "LD_LIBRARY_PATH": CONDA + "/lib:" + env.get("LD_LIBRARY_PATH", "")})
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"ref_dump failed for {name}:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
        metas, arrs = [], {}
        for p in range(pr * pc):
            with open(os.path.join(out, f"meta_{p}.json")) as fh:
                metas.append(json.load(fh))
            for f in glob.glob(os.path.join(out, f"r{p}_*.npy")):
                arrs[os.path.basename(f)[:-4]] = np.load(f)
        # global arrays are identical on every rank: keep rank 0's only
        for key in ("xsup", "supno", "perm_r", "perm_c", "R", "C"):
            for p in range(1, pr * pc):
                arrs.pop(f"r{p}_{key}", None)
        meta = {"case": name, "grid": [pr, pc], "dtype": dt, "options": {k: str(v) for k, v in opts.items()},
                "matrix": src if isinstance(src, str) else "generated (oracle/gen/make_refdump.py)",
                "generator": "oracle/gen/make_refdump.py via oracle/_ref/ref_dump", "ranks": metas}
        dst = os.path.join(GOLDEN, f"refdump_{name}.npz")
        np.savez_compressed(dst, meta=json.dumps(meta), **arrs)
        m0 = metas[0]
        print(f"{name}: nsupers={m0.get('nsupers')} info={m0.get('info')} tiny={m0.get('tiny')} "
              f"gssvx_info={m0.get('gssvx_info')} steps={m0.get('refine_steps')} "
              f"-> {os.path.getsize(dst) / 1024:.0f} KiB")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    for nm in sys.argv[1:] or list(CASES):
        make(nm)
