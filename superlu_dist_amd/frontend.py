"""Python side of the front-end helpers (matrix generation, ordering,
symbolic factorization, distribution).  Thin wrappers over the C++ code in
``csrc/frontend.cpp``; they build LUstructs in the reference layout
(SRC/pddistribute.c) for the tests and the benchmark."""
import ctypes as C

import numpy as np

from .lib import (DTYPES, SLU_D, SLU_S, SLU_Z, SluLuView, as_i64p, c_i64p, lib)

STENCIL_2D5, STENCIL_3D7, STENCIL_3D27 = 0, 1, 2


class Csc:
    """Owning handle of a library slu_csc."""

    def __init__(self, ptr):
        self.ptr = ptr

    @classmethod
    def stencil(cls, kind, nx, ny, nz=1, diag=None, diag_im=0.0, off=-1.0, dtype=SLU_D):
        if diag is None:
            diag = {STENCIL_2D5: 4.0, STENCIL_3D7: 6.0, STENCIL_3D27: 26.0}[kind]
        return cls(lib().slu_gen_stencil(kind, nx, ny, nz, diag, diag_im, off, dtype))

    @classmethod
    def from_arrays(cls, n, colptr, rowind, val, dtype):
        colptr = np.ascontiguousarray(colptr, dtype=np.int64)
        rowind = np.ascontiguousarray(rowind, dtype=np.int64)
        val = np.ascontiguousarray(val, dtype=DTYPES[dtype])
        return cls(lib().slu_csc_create(n, len(rowind), as_i64p(colptr), as_i64p(rowind),
                                        val.ctypes.data_as(C.c_void_p), dtype))

    @property
    def n(self):
        return self.ptr.contents.n

    @property
    def dtype(self):
        return self.ptr.contents.dtype

    def arrays(self):
        s = self.ptr.contents
        colptr = np.ctypeslib.as_array(s.colptr, shape=(s.n + 1,)).copy()
        rowind = np.ctypeslib.as_array(s.rowind, shape=(s.nnz,)).copy()
        npt = DTYPES[s.dtype]
        buf = (C.c_char * (s.nnz * np.dtype(npt).itemsize)).from_address(s.val)
        val = np.frombuffer(buf, dtype=npt).copy()
        return colptr, rowind, val

    def to_dense(self):
        colptr, rowind, val = self.arrays()
        n = self.n
        A = np.zeros((n, n), dtype=val.dtype)
        for j in range(n):
            A[rowind[colptr[j]:colptr[j + 1]], j] = val[colptr[j]:colptr[j + 1]]
        return A

    def permuted(self, perm):
        perm = np.ascontiguousarray(perm, dtype=np.int64)
        return Csc(lib().slu_permute(self.ptr, as_i64p(perm)))

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().slu_csc_free(self.ptr)
            self.ptr = None


def nd_order(nx, ny, nz=1):
    perm = np.empty(nx * ny * nz, dtype=np.int64)
    if lib().slu_order_nd_grid(nx, ny, nz, as_i64p(perm)) != 0:
        raise RuntimeError("nested dissection failed")
    return perm


SLU_SYMB_MULTICHILD, SLU_SYMB_REFERENCE, SLU_SYMB_COARSE = 1, 2, 4


class Symbolic:
    def __init__(self, A, perm_c=None, relax=60, maxsup=256, multichild=False, reference=False,
                 coarse=False):
        """multichild: chain supernodes continue through columns with several
        etree children (csrc/frontend.cpp; shortens the supernodal tree of
        level-set nested dissections such as the library's METIS_NodeND).
        reference: pdgssvx's own symbolic stage instead (sp_colorder +
        symbfact, SRC/pdgssvx.c:1046-1076, bit-exact restatements in
        csrc/symbolic.cpp), distributed by the reference's pddistribute
        (csrc/distribute.cpp): the supernodes and L/U structure the reference
        hands pdgstrf for this perm_c.
        coarse (with reference): the engine's coarse partition of that
        structure (csrc/amalg.h, what a 1x1 plan factors internally), laid out
        by the same pddistribute rules on any grid; ref_flops() is still the
        reference partition's work."""
        self.A = A
        pc = None
        if perm_c is not None:
            self._perm_in = np.ascontiguousarray(perm_c, dtype=np.int64)
            pc = as_i64p(self._perm_in)
        self.reference = reference
        self.ptr = lib().slu_symbolic(A.ptr, pc, relax, maxsup,
                                      (SLU_SYMB_MULTICHILD if multichild else 0) |
                                      (SLU_SYMB_REFERENCE if reference else 0) |
                                      (SLU_SYMB_COARSE if coarse else 0))
        if not self.ptr:
            raise RuntimeError("slu_symbolic: " + lib().slu_last_error().decode())
        self.n = A.n
        self.nsupers = lib().slu_symb_nsupers(self.ptr)
        self.xsup = np.empty(self.nsupers + 1, dtype=np.int64)
        self.supno = np.empty(self.n, dtype=np.int64)
        self.perm_c = np.empty(self.n, dtype=np.int64)
        lib().slu_symb_arrays(self.ptr, as_i64p(self.xsup), as_i64p(self.supno),
                              as_i64p(self.perm_c))
        a, b = C.c_double(), C.c_double()
        lib().slu_symb_counts(self.ptr, C.byref(a), C.byref(b))
        self.nnzL, self.nnzU = a.value, b.value
        self.struct_sizes = np.empty(self.nsupers, dtype=np.int64)
        lib().slu_symb_struct_sizes(self.ptr, as_i64p(self.struct_sizes))

    def flops(self):
        """Algorithmic flops of the factorization with full U segments
        (SURVEY §8d): diag LU + L TRSM + U TRSV + Schur, fp64 counting."""
        w = np.diff(self.xsup).astype(np.float64)
        b = self.struct_sizes - w
        j = None
        diag = np.array([sum((wi - jj - 1) + 2.0 * (wi - jj - 1) ** 2 for jj in range(int(wi)))
                         for wi in w]) if len(w) < 0 else (w * (w - 1) / 2 + 2 * (w - 1) * w * (2 * w - 1) / 6)
        trsm = w * (w + 1) * b
        trsv = b * w * (w + 1)
        schur = 2.0 * b * b * w
        return {"schur": schur.sum(), "panel": (diag + trsm + trsv).sum(),
                "total": (schur + diag + trsm + trsv).sum()}

    def ref_flops(self):
        """reference symbolic: algorithmic flops of the reference's partition
        (SURVEY 8d accounting, as the plan reports them; for coarse=True the
        partition before the engine's amalgamation) and its supernode count"""
        out = (C.c_double * 7)()
        lib().slu_symb_ref_info(self.ptr, out)
        cp = self.A.dtype == SLU_Z
        schur, trsm, trsv, s1, s2, w = out[1:]
        m = 4.0 if cp else 1.0
        panel = (6 * s1 + 10 * w + 8 * s2 if cp else s1 + 2 * s2) + m * trsm + trsv
        return {"schur": m * schur, "panel": panel, "total": m * schur + panel,
                "nsupers": int(out[0])}

    def distribute(self, nprow=1, npcol=1, myrow=0, mycol=0):
        return LUStruct(self, nprow, npcol, myrow, mycol)

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().slu_symb_free(self.ptr)
            self.ptr = None


class LUStruct:
    """One rank's LUstruct (dLUstruct_t / sLUstruct_t / zLUstruct_t) owned by
    the library; exposes its flat arrays as numpy views.  Built either by our
    front-end (``Symbolic.distribute``) or from given arrays (``from_arrays``,
    e.g. the reference's own pddistribute output in tests/golden/refdump_*)."""

    def __init__(self, symb, nprow, npcol, myrow, mycol):
        self.symb = symb
        ptr = lib().slu_distribute(symb.ptr, symb.A.ptr, nprow, npcol, myrow, mycol)
        if not ptr:
            raise RuntimeError("slu_distribute failed")
        self._wrap(ptr, symb.A.dtype, symb.n, symb.nsupers, nprow, npcol, myrow, mycol)

    @classmethod
    def from_arrays(cls, dtype, n, xsup, supno, nprow, npcol, myrow, mycol, Lidx, Loff, Lval,
                    Lvoff, Uidx, Uoff, Uval, Uvoff, ToRecv=None, ToSendD=None, ToSendR=None,
                    bufmax=None):
        self = cls.__new__(cls)
        self.symb = None
        npt = DTYPES[dtype]
        i64 = lambda a: np.ascontiguousarray(a, dtype=np.int64)  # noqa: E731
        i32 = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
        xsup, supno = i64(xsup), i64(supno)
        Lidx, Loff, Lvoff, Uidx, Uoff, Uvoff = map(i64, (Lidx, Loff, Lvoff, Uidx, Uoff, Uvoff))
        Lval = np.ascontiguousarray(Lval, dtype=npt)
        Uval = np.ascontiguousarray(Uval, dtype=npt)
        ToRecv, ToSendD, ToSendR = i32(ToRecv), i32(ToSendD), i32(ToSendR)
        bufmax = i64(bufmax if bufmax is not None else np.zeros(5))
        ns = len(xsup) - 1
        ip = lambda a: None if a is None else a.ctypes.data_as(C.POINTER(C.c_int))  # noqa: E731
        ptr = lib().slu_lustruct_build(dtype, n, ns, as_i64p(xsup), as_i64p(supno), nprow, npcol,
                                       as_i64p(Lidx), len(Lidx), as_i64p(Loff),
                                       Lval.ctypes.data_as(C.c_void_p), len(Lval), as_i64p(Lvoff),
                                       as_i64p(Uidx), len(Uidx), as_i64p(Uoff),
                                       Uval.ctypes.data_as(C.c_void_p), len(Uval), as_i64p(Uvoff),
                                       ip(ToRecv), ip(ToSendD), ip(ToSendR), as_i64p(bufmax))
        if not ptr:
            raise RuntimeError("slu_lustruct_build failed")
        self._wrap(ptr, dtype, n, ns, nprow, npcol, myrow, mycol)
        return self

    @classmethod
    def from_glu(cls, symb, colptr, rowind, values, dtype, nprow=1, npcol=1, myrow=0, mycol=0):
        """This rank's LUstruct as the reference's pddistribute builds it
        (csrc/distribute.cpp) from a reference-exact symbolic factorization
        ``symb`` (superlu_dist_amd.symbolic.Symb) and A in the LUstruct's
        coordinates (CSC colptr / rowind / values of Pc Pr A Pc^T)."""
        self = cls.__new__(cls)
        self.symb = None
        i64 = lambda a: np.ascontiguousarray(a, dtype=np.int64)  # noqa: E731
        xsup, supno = i64(symb.xsup), i64(symb.supno)
        xl, ls, xu, us = i64(symb.xlsub), i64(symb.lsub), i64(symb.xusub), i64(symb.usub)
        cp, ri = i64(colptr), i64(rowind)
        v = np.ascontiguousarray(values, dtype=DTYPES[dtype])
        n = len(cp) - 1
        ptr = lib().slu_distribute_glu(dtype, n, as_i64p(xsup), as_i64p(supno), as_i64p(xl),
                                       as_i64p(ls), as_i64p(xu), as_i64p(us), as_i64p(cp),
                                       as_i64p(ri), v.ctypes.data_as(C.c_void_p), nprow, npcol,
                                       myrow, mycol)
        if not ptr:
            raise RuntimeError("slu_distribute_glu: " + lib().slu_last_error().decode())
        self._wrap(ptr, dtype, n, symb.nsupers, nprow, npcol, myrow, mycol)
        return self

    def _wrap(self, ptr, dtype, n, nsupers, nprow, npcol, myrow, mycol):
        self.ptr = ptr
        self.dtype = dtype
        self.n = n
        self.nsupers = nsupers
        self.nprow, self.npcol, self.myrow, self.mycol = nprow, npcol, myrow, mycol
        v = SluLuView()
        lib().slu_lu_get_view(self.ptr, self.dtype, C.byref(v))
        self.view = v
        self.xsup = np.ctypeslib.as_array(v.xsup, shape=(nsupers + 1,))
        npt = DTYPES[self.dtype]
        isz = np.dtype(npt).itemsize
        self.Lidx = np.ctypeslib.as_array(v.Lidx, shape=(v.Lidx_cnt,))
        self.Uidx = np.ctypeslib.as_array(v.Uidx, shape=(v.Uidx_cnt,))
        self.Lval = np.frombuffer((C.c_char * (v.Lval_cnt * isz)).from_address(v.Lval), dtype=npt)
        self.Uval = np.frombuffer((C.c_char * (v.Uval_cnt * isz)).from_address(v.Uval), dtype=npt)
        ns = nsupers
        self.nlc = (ns + npcol - 1) // npcol
        self.nlr = (ns + nprow - 1) // nprow
        self.Loff = np.ctypeslib.as_array(v.Lidx_off, shape=(self.nlc,))
        self.Lvoff = np.ctypeslib.as_array(v.Lval_off, shape=(self.nlc,))
        self.Uoff = np.ctypeslib.as_array(v.Uidx_off, shape=(self.nlr,))
        self.Uvoff = np.ctypeslib.as_array(v.Uval_off, shape=(self.nlr,))
        self.ToRecv = np.ctypeslib.as_array(v.ToRecv, shape=(ns,))
        self.ToSendD = np.ctypeslib.as_array(v.ToSendD, shape=(self.nlr,))
        self.bufmax = np.array(list(v.bufmax), dtype=np.int64)

    def to_sendr(self):
        out = np.empty((self.nlc, self.npcol), dtype=np.int32)
        for i in range(self.nlc):
            out[i] = np.ctypeslib.as_array(self.view.ToSendR[i], shape=(self.npcol,))
        return out

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().slu_lustruct_free(self.ptr, self.dtype)
            self.ptr = None


class Amalgamation:
    """The engine's supernode amalgamation of a 1x1 LUStruct (csrc/amalg.h):
    the coarse partition the plan factors, as an LUStruct of its own
    (``merged``, values zero until ``expand``), and the host versions of the
    device expand / compress programs.  For tests: the plan applies the same
    programs on the device."""

    def __init__(self, lu, zero_frac=0.10, maxw=256):
        self.lu = lu
        self.h = lib().slu_amalg_create(lu.dtype, lu.ptr, lu.n, zero_frac, maxw)
        if not self.h:
            raise RuntimeError(lib().slu_last_error().decode())
        sz = np.zeros(8, np.int64)
        lib().slu_amalg_sizes(self.h, as_i64p(sz))
        self.ns1, self.ns2, nli, nui, self.lval2, self.uval2, self.groups, self.zeros = map(int, sz)
        n = lu.n
        xs, sn = np.zeros(self.ns2 + 1, np.int64), np.zeros(n, np.int64)
        Li, Ui = np.zeros(max(nli, 1), np.int64), np.zeros(max(nui, 1), np.int64)
        Lo, Lv, Uo, Uv = (np.zeros(self.ns2, np.int64) for _ in range(4))
        lib().slu_amalg_arrays(self.h, as_i64p(xs), as_i64p(sn), as_i64p(Li), as_i64p(Lo),
                               as_i64p(Lv), as_i64p(Ui), as_i64p(Uo), as_i64p(Uv))
        npt = DTYPES[lu.dtype]
        self.merged = LUStruct.from_arrays(lu.dtype, n, xs, sn, 1, 1, 0, 0, Li[:nli], Lo,
                                           np.zeros(self.lval2 + 1, npt), Lv, Ui[:nui], Uo,
                                           np.zeros(self.uval2 + 1, npt), Uv)

    def flops(self):
        """the ORIGINAL partition's algorithmic flops, as the plan reports them"""
        out = (C.c_double * 2)()
        lib().slu_amalg_flops(self.h, self.lu.dtype, out)
        return out[0] + out[1]

    def apply(self, oL, oU, mL, mU, direction):
        arrs = [np.ascontiguousarray(a) for a in (oL, oU, mL, mU)]
        rc = lib().slu_amalg_apply(self.h, self.lu.dtype, *[a.ctypes.data_as(C.c_void_p)
                                                            for a in arrs], direction)
        if rc:
            raise RuntimeError("slu_amalg_apply")

    def expand(self):
        """merged := the original LUStruct's values (structural zeros elsewhere)"""
        self.merged.Lval[:] = 0
        self.merged.Uval[:] = 0
        self.apply(self.lu.Lval, self.lu.Uval, self.merged.Lval, self.merged.Uval, 0)

    def compress(self, oL, oU):
        """oL / oU (the original layout) := the merged values at their positions"""
        self.apply(oL, oU, self.merged.Lval, self.merged.Uval, 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().slu_amalg_free(self.h)
            self.h = None


class GridAmalgamation:
    """The engine's amalgamation of a Pr x Pc grid's LUStructs (csrc/amalg.h,
    "grids"): every rank's coarse LUStruct (``merged[k]``, values zero until
    ``expand``) and the host versions of the relayout -- pack, all-to-all,
    unpack -- that the grid plan runs on the device with its transport.  All
    ranks in one process, for tests."""

    def __init__(self, lus, nprow, npcol, zero_frac=0.10, maxw=256):
        self.lus = list(lus)
        P = nprow * npcol
        assert len(self.lus) == P
        self.nprow, self.npcol = nprow, npcol
        dt, n = self.lus[0].dtype, self.lus[0].n
        ptrs = (C.c_void_p * P)(*[lu.ptr for lu in self.lus])
        self.h = lib().slu_gamalg_create(dt, P, ptrs, n, nprow, npcol, zero_frac, maxw)
        if not self.h:
            raise RuntimeError(lib().slu_last_error().decode())
        npt = DTYPES[dt]
        self.merged = []
        for k in range(P):
            sz = np.zeros(8, np.int64)
            lib().slu_gamalg_sizes(self.h, k, as_i64p(sz))
            self.ns1, self.ns2, nli, nui, lval2, uval2, nlc2, nlr2 = map(int, sz)
            xs, sn = np.zeros(self.ns2 + 1, np.int64), np.zeros(n, np.int64)
            Li, Ui = np.zeros(max(nli, 1), np.int64), np.zeros(max(nui, 1), np.int64)
            Lo, Lv = np.zeros(max(nlc2, 1), np.int64), np.zeros(max(nlc2, 1), np.int64)
            Uo, Uv = np.zeros(max(nlr2, 1), np.int64), np.zeros(max(nlr2, 1), np.int64)
            lib().slu_gamalg_arrays(self.h, k, as_i64p(xs), as_i64p(sn), as_i64p(Li), as_i64p(Lo),
                                    as_i64p(Lv), as_i64p(Ui), as_i64p(Uo), as_i64p(Uv))
            self.merged.append(LUStruct.from_arrays(
                dt, n, xs, sn, nprow, npcol, k // npcol, k % npcol, Li[:nli], Lo[:nlc2],
                np.zeros(lval2 + 1, npt), Lv[:nlc2], Ui[:nui], Uo[:nlr2], np.zeros(uval2 + 1, npt),
                Uv[:nlr2]))

    def flops(self):
        """the ORIGINAL partition's algorithmic flops (summed over the ranks'
        analysis ranges, as the grid plans report them)"""
        out = (C.c_double * 2)()
        lib().slu_gamalg_flops(self.h, self.lus[0].dtype, out)
        return out[0] + out[1]

    def _apply(self, o, m, direction):
        P = len(self.lus)
        arr = lambda xs: (C.c_void_p * P)(*[x.ctypes.data for x in xs])  # noqa: E731
        rc = lib().slu_gamalg_apply(self.h, self.lus[0].dtype, arr([a for a, _ in o]), arr([b for _, b in o]),
                                    arr([a for a, _ in m]), arr([b for _, b in m]), direction)
        if rc:
            raise RuntimeError("slu_gamalg_apply")

    def expand(self):
        """every rank's merged := the caller values routed to it (zeros elsewhere)"""
        for m in self.merged:
            m.Lval[:] = 0
            m.Uval[:] = 0
        self._apply([(lu.Lval, lu.Uval) for lu in self.lus], [(m.Lval, m.Uval) for m in self.merged], 0)

    def compress(self, outs):
        """outs[k] = (L, U) arrays in rank k's caller layout := the merged values"""
        self._apply(outs, [(m.Lval, m.Uval) for m in self.merged], 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().slu_gamalg_free(self.h)
            self.h = None
