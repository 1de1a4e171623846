"""ctypes mirror of the reference types that cross the pdgstrf boundary
(include/slu_abi.h: superlu_dist_options_t SRC/superlu_defs.h:716-755,
gridinfo_t :385-399, SuperLUStat_t SRC/util_dist.h:101-134) and a caller of
the drop-in entry points pdgstrf / psgstrf / pzgstrf exactly as pdgssvx calls
them (SRC/pdgssvx.c:1174-1180).

Used by the tests to exercise the exported symbols themselves (argument
checks, in-place factors, stat side effects, info) on a 1x1 grid, where the
entry points touch no MPI.  Multi-rank grids go through the reference's own
drivers linked against libslu_mi355x.so (oracle/_ref/p?drive_mi355x).
"""
import ctypes as C

import numpy as np

from .lib import DROPIN_PATH, SLU_D, SLU_S, SLU_Z

_dropin = None


def dropin():
    """The drop-in library itself (libslu_mi355x.so: only the p[dsz]gstrf /
    [dsz]scatter_* symbols of the reference's p?gstrf.c.o)."""
    global _dropin
    if _dropin is None:
        import os
        if not os.path.exists(DROPIN_PATH):
            raise RuntimeError(f"{DROPIN_PATH} missing: build with make -C superlu_dist_amd/csrc")
        _dropin = C.CDLL(DROPIN_PATH)
    return _dropin

MPI_Comm = C.c_int  # conda MPICH: MPI_Comm is an int (SURVEY 8b ABI layout)
NPHASES = 22        # PhaseType (SRC/superlu_enum_consts.h)
FACT = 7
YES, NO = 1, 0


class ScopeT(C.Structure):
    _fields_ = [("comm", MPI_Comm), ("Np", C.c_int), ("Iam", C.c_int)]


class GridInfo(C.Structure):
    _fields_ = [("comm", MPI_Comm), ("rscp", ScopeT), ("cscp", ScopeT), ("iam", C.c_int),
                ("nprow", C.c_int64), ("npcol", C.c_int64)]


class Options(C.Structure):
    _fields_ = [(nm, C.c_int) for nm in ("Fact", "Equil", "DiagInv", "ColPerm", "Trans",
                                         "IterRefine")] + \
               [("DiagPivotThresh", C.c_double)] + \
               [(nm, C.c_int) for nm in ("SymmetricMode", "PivotGrowth", "ConditionNumber",
                                         "RowPerm", "ILU_DropRule")] + \
               [("ILU_DropTol", C.c_double), ("ILU_FillFactor", C.c_double),
                ("ILU_Norm", C.c_int), ("ILU_FillTol", C.c_double), ("ILU_MILU", C.c_int),
                ("ILU_MILU_Dim", C.c_double)] + \
               [(nm, C.c_int) for nm in ("ParSymbFact", "ReplaceTinyPivot", "SolveInitialized",
                                         "RefineInitialized", "PrintStat", "lookahead_etree",
                                         "num_lookaheads", "superlu_relax", "superlu_maxsup")] + \
               [("superlu_rankorder", C.c_char * 4), ("superlu_lbs", C.c_char * 4)] + \
               [(nm, C.c_int) for nm in ("superlu_n_gemm", "superlu_max_buffer_size",
                                         "superlu_num_gpu_streams", "superlu_acc_offload",
                                         "SymPattern", "Use_TensorCore", "Algo3d")]


class SuperMatrix(C.Structure):
    """SRC/supermatrix.h:54-63."""
    _fields_ = [("Stype", C.c_int), ("Dtype", C.c_int), ("Mtype", C.c_int),
                ("nrow", C.c_int64), ("ncol", C.c_int64), ("Store", C.c_void_p)]


class NCformat(C.Structure):
    _fields_ = [("nnz", C.c_int64), ("nzval", C.c_void_p), ("rowind", C.POINTER(C.c_int64)),
                ("colptr", C.POINTER(C.c_int64))]


class NCPformat(C.Structure):
    _fields_ = [("nnz", C.c_int64), ("nzval", C.c_void_p), ("rowind", C.POINTER(C.c_int64)),
                ("colbeg", C.POINTER(C.c_int64)), ("colend", C.POINTER(C.c_int64))]


class GluPersist(C.Structure):
    _fields_ = [("xsup", C.POINTER(C.c_int64)), ("supno", C.POINTER(C.c_int64))]


class GluFreeable(C.Structure):
    """SRC/superlu_defs.h:494-505."""
    _fields_ = [("lsub", C.POINTER(C.c_int64)), ("xlsub", C.POINTER(C.c_int64)),
                ("usub", C.POINTER(C.c_int64)), ("xusub", C.POINTER(C.c_int64)),
                ("nzlmax", C.c_int64), ("nzumax", C.c_int64), ("MemModel", C.c_int),
                ("nnzLU", C.c_int64)]


class Stat(C.Structure):
    _fields_ = [("panel_histo", C.POINTER(C.c_int)), ("utime", C.POINTER(C.c_double)),
                ("ops", C.POINTER(C.c_float)), ("TinyPivots", C.c_int), ("RefineSteps", C.c_int),
                ("num_look_aheads", C.c_int), ("current_buffer", C.c_float),
                ("peak_buffer", C.c_float), ("gpu_buffer", C.c_float),
                ("MaxActiveBTrees", C.c_int64), ("MaxActiveRTrees", C.c_int64)]


def default_options():
    """set_default_options_dist (SRC/util.c:203-238), the fields pdgstrf reads."""
    o = Options()
    o.Equil = YES
    o.ColPerm = 2          # MMD_AT_PLUS_A (no METIS in the image)
    o.IterRefine = 2       # SLU_DOUBLE
    o.RowPerm = 1          # LargeDiag_MC64
    o.ReplaceTinyPivot = NO
    o.PrintStat = YES
    o.num_lookaheads = 10
    o.superlu_relax = 60
    o.superlu_maxsup = 256
    o.superlu_rankorder = b"ROW"
    o.superlu_lbs = b"GD"
    o.superlu_n_gemm = 5000
    o.superlu_max_buffer_size = 256000000
    o.superlu_num_gpu_streams = 8
    o.superlu_acc_offload = 1
    o.SymPattern = NO
    return o


def grid_1x1(comm=0x44000000):
    """A 1x1 gridinfo_t (MPICH's MPI_COMM_WORLD handle by default; a 1x1
    pdgstrf never calls MPI)."""
    g = GridInfo()
    g.comm = comm
    g.rscp.comm = g.cscp.comm = comm
    g.rscp.Np = g.cscp.Np = 1
    g.iam = 0
    g.nprow = g.npcol = 1
    return g


def pxgstrf(lu, anorm, options=None, grid=None, m=None, n=None):
    """Call pdgstrf / psgstrf / pzgstrf on the LUStruct ``lu`` in place, as
    pdgssvx does.  Returns (return value, info, stat dict)."""
    L = dropin()
    fn = {SLU_D: L.pdgstrf, SLU_S: L.psgstrf, SLU_Z: L.pzgstrf}[lu.dtype]
    fn.restype = C.c_int64
    anorm_t = C.c_float if lu.dtype == SLU_S else C.c_double
    fn.argtypes = [C.POINTER(Options), C.c_int, C.c_int, anorm_t, C.c_void_p,
                   C.POINTER(GridInfo), C.POINTER(Stat), C.POINTER(C.c_int)]
    o = options if options is not None else default_options()
    g = grid if grid is not None else grid_1x1()
    utime = (C.c_double * NPHASES)()
    ops = (C.c_float * NPHASES)()
    st = Stat()
    st.utime = C.cast(utime, C.POINTER(C.c_double))
    st.ops = C.cast(ops, C.POINTER(C.c_float))
    info = C.c_int(-999)
    n = lu.n if n is None else n
    m = n if m is None else m
    rv = fn(C.byref(o), m, n, anorm, C.c_void_p(lu.ptr), C.byref(g), C.byref(st), C.byref(info))
    return int(rv), info.value, {"ops_fact": float(ops[FACT]), "TinyPivots": st.TinyPivots,
                                 "num_look_aheads": st.num_look_aheads,
                                 "gpu_buffer": float(st.gpu_buffer)}


# ---- the device-resident drop-in: libslu_mi355x_solve.so also exports
# p[dsz]distribute (SRC/pddistribute.c:327) and p[dsz]gstrs (SRC/pdgstrs.c),
# so that pdgssvx's DISTRIBUTE keeps A for a device-side fill, pdgstrf leaves
# the factors in HBM and SOLVE runs on them.

_solve = None


def solve_lib():
    """libslu_mi355x_solve.so: the 12 drop-in symbols + p[dsz]distribute,
    p[dsz]gstrs (opt-in superset, csrc/dropin_solve.map)."""
    global _solve
    if _solve is None:
        import os
        path = os.path.join(os.path.dirname(DROPIN_PATH), "libslu_mi355x_solve.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: build with make -C superlu_dist_amd/csrc")
        _solve = C.CDLL(path)
    return _solve


SLU_NR_LOC, SLU_GE, NOEQUIL = 7, 0, 0  # Stype_t / Mtype_t / DiagScale_t (SRC/supermatrix.h, superlu_enum_consts.h)
SAMEPATTERN_SAMEROWPERM = 2


class NRformatLoc(C.Structure):
    """SRC/supermatrix.h NRformat_loc."""
    _fields_ = [("nnz_loc", C.c_int64), ("m_loc", C.c_int64), ("fst_row", C.c_int64),
                ("nzval", C.c_void_p), ("rowptr", C.POINTER(C.c_int64)),
                ("colind", C.POINTER(C.c_int64))]


class ScalePermstruct(C.Structure):
    """SRC/superlu_ddefs.h:60-66."""
    _fields_ = [("DiagScale", C.c_int), ("R", C.c_void_p), ("C", C.c_void_p),
                ("perm_r", C.POINTER(C.c_int64)), ("perm_c", C.POINTER(C.c_int64))]


class LUstruct(C.Structure):
    """SRC/superlu_ddefs.h dLUstruct_t (Llu: a calloc'ed dLocalLU_t, 2352
    bytes, include/slu_abi.h)."""
    _fields_ = [("etree", C.POINTER(C.c_int64)), ("Glu_persist", C.POINTER(GluPersist)),
                ("Llu", C.c_void_p), ("dt", C.c_char)]


def _p64(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


class DeviceResidentSystem:
    """One fp64 system through the reference's pdgssvx sequence on a 1x1
    grid, driven from here: A (NRformat_loc, column indices already mapped
    by perm_c as SRC/pdgssvx.c:1140 leaves them), ScalePermstruct (no
    equilibration, perm_r = identity), the symbolic factorization's
    Glu_persist / Glu_freeable, then pddistribute -> pdgstrf -> pdgstrs of
    libslu_mi355x_solve.so.  The arrays stay referenced for the lifetime of
    the object (the library keeps pointers to A's copy and to the
    LUstruct).

    One-shot use only, in a child process that exits afterwards (bench.py's
    device-resident leg runs it so): nothing frees the calloc'ed Llu, the
    arrays pddistribute allocates into it, or the library's cached plan and
    its device factors -- the reference's Destroy_LU / LUstructFree live in
    the reference library, which this process does not load.  Process exit
    releases them."""

    def __init__(self, n, rowptr, colind, nzval, perm_c, etree, xsup, supno, xlsub, lsub, xusub,
                 usub, anorm):
        self.L = solve_lib()
        self.n, self.anorm = n, anorm
        # Glu_persist's xsup as symbfact leaves it: n + 1 entries (the
        # supernode bounds, then the last one repeated)
        xs = np.full(n + 2, int(xsup[-1]), np.int64)
        xs[:len(xsup)] = xsup
        self.keep = [np.ascontiguousarray(x, np.int64) for x in
                     (rowptr, colind, perm_c, etree, xs, supno, xlsub, lsub, xusub, usub)]
        (self.rowptr, self.colind, self.perm_c, self.etree, self.xsup, self.supno, self.xlsub,
         self.lsub, self.xusub, self.usub) = self.keep
        self.nzval = np.ascontiguousarray(nzval, np.float64)
        self.perm_r = np.arange(n, dtype=np.int64)
        self.store = NRformatLoc(len(self.nzval), n, 0, self.nzval.ctypes.data, _p64(self.rowptr),
                                 _p64(self.colind))
        self.A = SuperMatrix(SLU_NR_LOC, SLU_D, SLU_GE, n, n, C.addressof(self.store))
        self.sp = ScalePermstruct(NOEQUIL, None, None, _p64(self.perm_r), _p64(self.perm_c))
        self.glu = GluFreeable(_p64(self.lsub), _p64(self.xlsub), _p64(self.usub), _p64(self.xusub),
                               len(self.lsub), len(self.usub), 0, 0)
        self.gp = GluPersist(_p64(self.xsup), _p64(self.supno))
        libc = C.CDLL(None)
        libc.calloc.restype = C.c_void_p
        libc.calloc.argtypes = [C.c_size_t, C.c_size_t]
        self.lu = LUstruct(_p64(self.etree), C.pointer(self.gp), libc.calloc(1, 2352), b"d")
        self.grid = grid_1x1()
        self.opt = default_options()
        self.opt.Equil = NO
        self.opt.RowPerm = 0  # NOROWPERM
        self.opt.ColPerm = 7  # MY_PERMC
        L = self.L
        L.pddistribute.restype = C.c_float
        L.pddistribute.argtypes = [C.POINTER(Options), C.c_int64, C.POINTER(SuperMatrix),
                                   C.POINTER(ScalePermstruct), C.POINTER(GluFreeable),
                                   C.POINTER(LUstruct), C.POINTER(GridInfo)]
        L.pdgstrf.restype = C.c_int64
        L.pdgstrf.argtypes = [C.POINTER(Options), C.c_int, C.c_int, C.c_double,
                              C.POINTER(LUstruct), C.POINTER(GridInfo), C.POINTER(Stat),
                              C.POINTER(C.c_int)]
        L.pdgstrs.restype = None
        L.pdgstrs.argtypes = [C.POINTER(Options), C.c_int64, C.POINTER(LUstruct),
                              C.POINTER(ScalePermstruct), C.POINTER(GridInfo),
                              C.POINTER(C.c_double), C.c_int64, C.c_int64, C.c_int64, C.c_int,
                              C.c_void_p, C.POINTER(Stat), C.POINTER(C.c_int)]

    def _stat(self):
        self._ut = (C.c_double * NPHASES)()
        self._ops = (C.c_float * NPHASES)()
        st = Stat()
        st.utime = C.cast(self._ut, C.POINTER(C.c_double))
        st.ops = C.cast(self._ops, C.POINTER(C.c_float))
        return st

    def distribute(self, fact):
        self.opt.Fact = fact
        return float(self.L.pddistribute(C.byref(self.opt), self.n, C.byref(self.A), C.byref(self.sp),
                                         C.byref(self.glu), C.byref(self.lu), C.byref(self.grid)))

    def factor(self):
        st = self._stat()
        info = C.c_int(-999)
        rv = self.L.pdgstrf(C.byref(self.opt), self.n, self.n, self.anorm, C.byref(self.lu),
                            C.byref(self.grid), C.byref(st), C.byref(info))
        return int(rv), info.value, float(self._ops[FACT])

    def solve(self, b):
        """b in A's original row order (m_loc = n on 1x1); returns x in A's
        original column order: pdgstrs leaves the solution of the column-
        permuted system, and pdgssvx maps it back with pdPermute_Dense_Matrix
        by inv_perm_c (SRC/pdgssvx.c, SOLVE phase), i.e. x[j] = X[perm_c[j]]."""
        x = np.ascontiguousarray(b, np.float64).copy()
        st = self._stat()
        info = C.c_int(-999)
        self.L.pdgstrs(C.byref(self.opt), self.n, C.byref(self.lu), C.byref(self.sp),
                       C.byref(self.grid), x.ctypes.data_as(C.POINTER(C.c_double)), self.n, 0,
                       self.n, 1, None, C.byref(st), C.byref(info))
        if info.value:
            raise RuntimeError(f"pdgstrs info {info.value}")
        return x[self.perm_c]


def layout():
    """Sizes / offsets of the mirror, in the keys of tests/golden/abi_layout.json."""
    return {"sizeof(gridinfo_t)": C.sizeof(GridInfo), "sizeof(superlu_scope_t)": C.sizeof(ScopeT),
            "sizeof(superlu_dist_options_t)": C.sizeof(Options),
            "sizeof(SuperLUStat_t)": C.sizeof(Stat),
            "gridinfo_t.nprow": GridInfo.nprow.offset, "gridinfo_t.iam": GridInfo.iam.offset,
            "superlu_dist_options_t.ReplaceTinyPivot": Options.ReplaceTinyPivot.offset,
            "superlu_dist_options_t.num_lookaheads": Options.num_lookaheads.offset,
            "superlu_dist_options_t.superlu_maxsup": Options.superlu_maxsup.offset,
            "superlu_dist_options_t.SymPattern": Options.SymPattern.offset,
            "superlu_dist_options_t.Algo3d": Options.Algo3d.offset,
            "SuperLUStat_t.ops": Stat.ops.offset, "SuperLUStat_t.TinyPivots": Stat.TinyPivots.offset,
            "SuperLUStat_t.num_look_aheads": Stat.num_look_aheads.offset}


__all__ = ["Options", "GridInfo", "Stat", "default_options", "grid_1x1", "pxgstrf", "layout",
           "np"]
