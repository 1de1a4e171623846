"""Parity cases shared by the golden-fixture generator (oracle/gen/make_golden.py)
and the tests.  Each case is a deterministic recipe: matrix, ordering,
supernode parameters, process grid, value type and pdgstrf options.

The matrices are the reference's own test inputs (EXAMPLE/g4.rua, g20.rua,
cg20.cua; TEST/CMakeLists.txt uses g20 with relax 8 / maxsup 20 on grids up
to 5x3) and the BASELINE stencils (3D 7-point, 2D 5-point, 27-point, complex
Helmholtz) at small sizes, plus two pivot edge cases.
"""
import os

import numpy as np

from superlu_dist_amd.frontend import (STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Csc,
                                       Symbolic, nd_order)
from superlu_dist_amd.hbio import read_hb
from superlu_dist_amd.lib import SLU_D, SLU_S, SLU_Z

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MATRICES = os.path.join(GOLDEN, "matrices")

DT = {"d": SLU_D, "s": SLU_S, "z": SLU_Z}


def _hb(name, dtype):
    n, cp, ri, v, cplx = read_hb(os.path.join(MATRICES, name))
    if dtype == SLU_Z:
        v = v.astype(np.complex128)
    elif dtype == SLU_S:
        v = v.real.astype(np.float32)
    else:
        v = v.real.astype(np.float64)
    return Csc.from_arrays(n, cp, ri, v, dtype), None


def _stencil(kind, nx, ny, nz, dtype, diag=None, diag_im=0.0):
    A = Csc.stencil(kind, nx, ny, nz, diag=diag, diag_im=diag_im, dtype=dtype)
    return A, nd_order(nx, ny, nz if kind != STENCIL_2D5 else 1)


def _zero_pivot(dtype):
    """2D 5-point 8x8 Laplacian with A(0,0) = 0: node 0 is the first column of
    the first leaf supernode, so its pivot is exactly zero."""
    A = Csc.stencil(STENCIL_2D5, 8, 8, 1, dtype=dtype)
    cp, ri, v = A.arrays()
    for p in range(cp[0], cp[1]):
        if ri[p] == 0:
            v[p] = 0
    return Csc.from_arrays(A.n, cp, ri, v, dtype), nd_order(8, 8, 1)


CASES = {
    # name: (builder, dtype, grid, relax, maxsup, replace_tiny)
    "g4_1x1_d": (lambda d: _hb("g4.rua", d), "d", (1, 1), 60, 256, False),
    "g20_1x1_d": (lambda d: _hb("g20.rua", d), "d", (1, 1), 60, 256, False),
    "g20_1x1_small_d": (lambda d: _hb("g20.rua", d), "d", (1, 1), 8, 20, False),
    "g20_2x3_small_d": (lambda d: _hb("g20.rua", d), "d", (2, 3), 8, 20, False),
    "g20_1x1_s": (lambda d: _hb("g20.rua", d), "s", (1, 1), 60, 256, False),
    "cg20_1x1_z": (lambda d: _hb("cg20.cua", d), "z", (1, 1), 60, 256, False),
    "cg20_2x2_small_z": (lambda d: _hb("cg20.cua", d), "z", (2, 2), 8, 20, False),
    "lap3d_8_1x1_d": (lambda d: _stencil(STENCIL_3D7, 8, 8, 8, d), "d", (1, 1), 60, 256, False),
    "lap3d_8_2x2_d": (lambda d: _stencil(STENCIL_3D7, 8, 8, 8, d), "d", (2, 2), 60, 256, False),
    "lap3d_10_2x4_small_d": (lambda d: _stencil(STENCIL_3D7, 10, 10, 10, d), "d", (2, 4), 4, 10,
                             False),
    "lap3d_14_1x1_d": (lambda d: _stencil(STENCIL_3D7, 14, 14, 14, d), "d", (1, 1), 60, 256, False),
    "lap2d_32_1x1_d": (lambda d: _stencil(STENCIL_2D5, 32, 32, 1, d), "d", (1, 1), 60, 256, False),
    "lap2d_32_2x1_d": (lambda d: _stencil(STENCIL_2D5, 32, 32, 1, d), "d", (2, 1), 60, 256, False),
    "helm3d_6_2x2_z": (lambda d: _stencil(STENCIL_3D7, 6, 6, 6, d, diag=6 - 0.25, diag_im=-0.0025),
                       "z", (2, 2), 60, 256, False),
    "helm3d_8_1x1_z": (lambda d: _stencil(STENCIL_3D7, 8, 8, 8, d, diag=6 - 0.25, diag_im=-0.0025),
                       "z", (1, 1), 60, 256, False),
    "st27_8_1x1_s": (lambda d: _stencil(STENCIL_3D27, 8, 8, 8, d), "s", (1, 1), 60, 256, False),
    "st27_8_2x2_s": (lambda d: _stencil(STENCIL_3D27, 8, 8, 8, d), "s", (2, 2), 60, 256, False),
    "zeropiv_1x1_d": (_zero_pivot, "d", (1, 1), 60, 256, False),
    "tinypiv_1x1_d": (_zero_pivot, "d", (1, 1), 60, 256, True),
}


def build(name):
    """Returns (A, perm_c_or_None, dtype_code, (Pr, Pc), relax, maxsup, replace_tiny)."""
    fn, dch, grid, relax, maxsup, tiny = CASES[name]
    dtype = DT[dch]
    A, perm = fn(dtype)
    return A, perm, dtype, grid, relax, maxsup, tiny


def distribute(name):
    """Symbolic factorization + all ranks' LUstructs (rank order row*Pc+col)."""
    A, perm, dtype, (pr, pc), relax, maxsup, tiny = build(name)
    S = Symbolic(A, perm, relax, maxsup)
    lus = [S.distribute(pr, pc, r, c) for r in range(pr) for c in range(pc)]
    return A, S, lus


def anorm(A):
    """||A||_1 as pdlangs("1") (SRC/pdlangs.c), modulus for complex."""
    cp, ri, v = A.arrays()
    s = np.add.reduceat(np.abs(v).astype(np.float64), cp[:-1]) if len(v) else np.zeros(1)
    return float(s.max())


def structure_digest(lus):
    """Fingerprint of the pre-factor index arrays (guards fixture/front-end drift)."""
    import hashlib
    h = hashlib.sha256()
    for lu in lus:
        h.update(np.ascontiguousarray(lu.Lidx).tobytes())
        h.update(np.ascontiguousarray(lu.Uidx).tobytes())
    return h.hexdigest()[:16]


def factor_error(lus, ref):
    """max over ranks and over L/U of ||mine - ref||_max / ||ref||_max."""
    worst = 0.0
    for lu, (Lr, Ur) in zip(lus, ref):
        for mine, r in ((lu.Lval, Lr), (lu.Uval, Ur)):
            if len(r) == 0:
                continue
            mine = mine[:len(r)]  # library-built *_dat arrays carry one spare element
            if not np.isfinite(mine).all():
                return float("inf")  # max() below would drop a NaN
            d = np.abs(mine.astype(np.complex128) - r.astype(np.complex128)).max()
            worst = max(worst, d / max(np.abs(r).max(), 1e-300))
    return worst


def stencil_case(kind, dims, dtype, grid, relax, maxsup, reference=False):
    """cases.build()-style recipe for a seeded stencil (picklable via partial);
    reference: the LUstruct pdgssvx builds (reference symbfact + pddistribute)
    instead of the front-end's."""
    kw = {}
    if dtype == SLU_Z:
        kw = dict(diag=6 - 0.25, diag_im=-0.0025)
    A, perm = _stencil(kind, *dims, dtype, **kw)
    return (A, perm, dtype, grid, relax, maxsup, False) + ((True,) if reference else ())
