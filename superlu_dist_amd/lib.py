"""ctypes binding of libslu_mi355x_full.so (include/slu_mi355x.h).

Two libraries are built in-tree by ``make -C superlu_dist_amd/csrc``
(``__graft_entry__.build()``) from the same objects: libslu_mi355x.so, the
drop-in with exactly the reference pdgstrf.c.o symbol set (bound by
``capi.dropin()``), and libslu_mi355x_full.so, which also exports the engine
API, the front-end helpers and the opt-in reference-prototype extras.  This
module binds the latter.  Nothing here falls back to Python or the CPU: a
missing library raises immediately.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SLU_LIB overrides the in-tree library (A/B comparisons of engine builds)
LIB_PATH = os.environ.get("SLU_LIB") or os.path.join(_HERE, "lib", "libslu_mi355x_full.so")
DROPIN_PATH = os.path.join(os.path.dirname(LIB_PATH), "libslu_mi355x.so")

SLU_D, SLU_S, SLU_Z = 0, 1, 2
DTYPES = {SLU_D: np.float64, SLU_S: np.float32, SLU_Z: np.complex128}
DTYPE_CODE = {"d": SLU_D, "s": SLU_S, "z": SLU_Z}

c_i64p = C.POINTER(C.c_int64)
c_intp = C.POINTER(C.c_int)


# int (*)(void *ctx, int group, int root, void *buf, int64_t bytes)
HOST_BCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int64)


class HostP2POp(C.Structure):
    """slu_host_p2p_op: one send / receive of an exchange phase."""
    _fields_ = [("group", C.c_int), ("peer", C.c_int), ("send", C.c_int), ("reserved", C.c_int),
                ("buf", C.c_void_p), ("bytes", C.c_int64)]


# int (*)(void *ctx, int nops, const slu_host_p2p_op *ops)
HOST_P2P_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(HostP2POp))


class SluCsc(C.Structure):
    _fields_ = [("n", C.c_int64), ("nnz", C.c_int64), ("colptr", c_i64p),
                ("rowind", c_i64p), ("val", C.c_void_p), ("dtype", C.c_int)]


class SluLuView(C.Structure):
    _fields_ = [("nsupers", C.c_int64), ("xsup", c_i64p), ("supno", c_i64p),
                ("Lidx", c_i64p), ("Lidx_cnt", C.c_int64), ("Lidx_off", C.POINTER(C.c_long)),
                ("Lval", C.c_void_p), ("Lval_cnt", C.c_int64), ("Lval_off", C.POINTER(C.c_long)),
                ("Uidx", c_i64p), ("Uidx_cnt", C.c_int64), ("Uidx_off", C.POINTER(C.c_long)),
                ("Uval", C.c_void_p), ("Uval_cnt", C.c_int64), ("Uval_off", C.POINTER(C.c_long)),
                ("ToRecv", c_intp), ("ToSendD", c_intp), ("ToSendR", C.POINTER(c_intp)),
                ("bufmax", C.c_int64 * 5)]


class EngineOpts(C.Structure):
    _fields_ = [("replace_tiny_pivot", C.c_int), ("timing", C.c_int), ("serial", C.c_int),
                ("overlap_upload", C.c_int), ("overlap_download", C.c_int),
                ("schedule_only", C.c_int), ("forest_map", C.c_void_p)]


class PlanStats(C.Structure):
    _fields_ = [("nsupers", C.c_int64), ("nlevels", C.c_int64),
                ("n_schur_tiles", C.c_int64), ("n_diag", C.c_int64),
                ("n_trsm_items", C.c_int64),
                ("schur_flops", C.c_double), ("schur_flops_padded", C.c_double),
                ("panel_flops", C.c_double), ("scatter_bytes", C.c_double),
                ("lu_bytes", C.c_double), ("index_bytes", C.c_double),
                ("t_total_ms", C.c_double), ("t_diag_ms", C.c_double),
                ("t_trsm_ms", C.c_double), ("t_schur_ms", C.c_double),
                ("t_comm_ms", C.c_double), ("t_schur_big_ms", C.c_double),
                ("schur_big_flops", C.c_double), ("n_schur_launches", C.c_int64),
                ("n_schur_big_launches", C.c_int64), ("comm_bytes", C.c_double),
                ("t_solve_ms", C.c_double), ("t_fill_ms", C.c_double),
                ("t_refine_ms", C.c_double), ("t_plan_ms", C.c_double),
                ("t_upload_ms", C.c_double), ("t_upload_wait_ms", C.c_double),
                ("t_d2h_ms", C.c_double), ("t_d2h_tail_ms", C.c_double),
                ("h2d_bytes", C.c_double), ("d2h_bytes", C.c_double),
                ("n_d2h_copies", C.c_int64), ("comm_buf_bytes", C.c_double),
                ("nsupers_in", C.c_int64), ("amalg_groups", C.c_int64),
                ("amalg_zeros", C.c_double), ("t_amalg_ms", C.c_double),
                ("t_expand_ms", C.c_double), ("t_compress_ms", C.c_double),
                ("t_phase_ms", C.c_double * 8), ("t_zreduce_ms", C.c_double),
                ("zred_bytes", C.c_double * 8),
                ("npdep", C.c_int64), ("zlayer", C.c_int64), ("phase_last", C.c_int64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["t_phase_ms"] = list(d["t_phase_ms"])
        d["zred_bytes"] = list(d["zred_bytes"])
        return d


_lib = None


def lib():
    """Load the in-tree shared library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    P = C.c_void_p
    sig = {
        "slu_gen_stencil": (C.POINTER(SluCsc), [C.c_int, C.c_int, C.c_int, C.c_int,
                                                C.c_double, C.c_double, C.c_double, C.c_int]),
        "slu_csc_create": (C.POINTER(SluCsc), [C.c_int64, C.c_int64, c_i64p, c_i64p, P, C.c_int]),
        "slu_csc_free": (None, [C.POINTER(SluCsc)]),
        "slu_order_nd_grid": (C.c_int, [C.c_int, C.c_int, C.c_int, c_i64p]),
        "slu_colorder": (C.c_int, [C.c_int64, C.c_int64, c_i64p, c_i64p, C.c_int, C.c_int,
                                   c_i64p, c_i64p, c_i64p, c_i64p]),
        "slu_symbfact": (P, [C.c_int64, C.c_int64, c_i64p, c_i64p, c_i64p, c_i64p, C.c_int64,
                             C.c_int64]),
        "slu_symbfact_sizes": (None, [P, c_i64p]),
        "slu_symbfact_arrays": (None, [P, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p]),
        "slu_symbfact_views": (None, [P, C.POINTER(C.c_void_p)]),
        "slu_symbfact_free": (None, [P]),
        "slu_symbfact_last_epilogue_device": (C.c_int, []),
        "METIS_NodeND": (C.c_int, [c_i64p, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p]),
        "slu_symbolic": (P, [C.POINTER(SluCsc), c_i64p, C.c_int, C.c_int, C.c_int]),
        "slu_symb_free": (None, [P]),
        "slu_symb_nsupers": (C.c_int64, [P]),
        "slu_symb_arrays": (None, [P, c_i64p, c_i64p, c_i64p]),
        "slu_symb_counts": (None, [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "slu_symb_struct_sizes": (None, [P, c_i64p]),
        "slu_distribute": (P, [P, C.POINTER(SluCsc), C.c_int, C.c_int, C.c_int, C.c_int]),
        "slu_lustruct_free": (None, [P, C.c_int]),
        "slu_amalg_create": (P, [C.c_int, P, C.c_int64, C.c_double, C.c_int]),
        "slu_amalg_sizes": (None, [P, c_i64p]),
        "slu_amalg_arrays": (None, [P] + [c_i64p] * 8),
        "slu_amalg_apply": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int]),
        "slu_amalg_free": (None, [P]),
        "slu_symb_ref_info": (None, [P, C.POINTER(C.c_double)]),
        "slu_amalg_flops": (None, [P, C.c_int, C.POINTER(C.c_double)]),
        "slu_gamalg_create": (P, [C.c_int, C.c_int, C.POINTER(P), C.c_int64, C.c_int, C.c_int,
                                  C.c_double, C.c_int]),
        "slu_gamalg_sizes": (None, [P, C.c_int, c_i64p]),
        "slu_gamalg_arrays": (None, [P, C.c_int] + [c_i64p] * 8),
        "slu_gamalg_flops": (None, [P, C.c_int, C.POINTER(C.c_double)]),
        "slu_gamalg_apply": (C.c_int, [P, C.c_int] + [C.POINTER(P)] * 4 + [C.c_int]),
        "slu_gamalg_free": (None, [P]),
        "slu_distribute_glu": (P, [C.c_int, C.c_int64, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p,
                                   c_i64p, c_i64p, c_i64p, P, C.c_int, C.c_int, C.c_int, C.c_int]),
        "slu_lustruct_build": (P, [C.c_int, C.c_int64, C.c_int64, c_i64p, c_i64p, C.c_int,
                                   C.c_int, c_i64p, C.c_int64, c_i64p, P, C.c_int64, c_i64p,
                                   c_i64p, C.c_int64, c_i64p, P, C.c_int64, c_i64p, c_intp,
                                   c_intp, c_intp, c_i64p]),
        "slu_permute": (C.POINTER(SluCsc), [C.POINTER(SluCsc), c_i64p]),
        "slu_lu_get_view": (C.c_int, [P, C.c_int, C.POINTER(SluLuView)]),
        "slu_comm_unique_id": (C.c_int, [P]),
        "slu_comm_create": (P, [P, C.c_int, C.c_int, C.c_int, C.c_int]),
        "slu_comm_create_host": (P, [HOST_BCAST_FN, P, C.c_int, C.c_int, C.c_int, C.c_int]),
        "slu_comm_create_host_p2p": (P, [HOST_P2P_FN, P, C.c_int, C.c_int, C.c_int, C.c_int]),
        "slu_comm_create3d": (P, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
        "slu_comm_create_host_p2p3d": (P, [HOST_P2P_FN, P, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_int]),
        "slu_comm_size": (C.c_int, [P, C.c_int]),
        "slu_comm_destroy": (None, [P]),
        "slu_plan_create": (P, [C.c_int, P, C.c_int, C.c_int, C.c_int, C.c_int, P,
                                C.POINTER(EngineOpts), C.c_char_p, C.c_int]),
        "slu_plan_upload": (C.c_int, [P]),
        "slu_plan_factor": (C.c_int, [P, C.c_double, c_intp, c_intp]),
        "slu_plan_download": (C.c_int, [P]),
        "slu_plan_solve": (C.c_int, [P, P, C.c_int64, C.c_int]),
        "slu_plan_set_a_pattern": (C.c_int, [P, C.c_int64, c_i64p, c_i64p]),
        "slu_plan_fill_a": (C.c_int, [P, P, C.c_int]),
        "slu_plan_refine": (C.c_int, [P, P, P, C.c_int64, C.c_int, C.POINTER(C.c_double), c_intp]),
        "slu_plan_snapshot": (C.c_int, [P]),
        "slu_plan_restore": (C.c_int, [P]),
        "slu_plan_sync": (C.c_int, [P]),
        "slu_plan_set_timing": (C.c_int, [P, C.c_int, C.c_int]),
        "slu_plan_check_exchange": (C.c_int, [P, c_i64p, c_i64p]),
        "slu_plan_gather3d": (C.c_int, [P]),
        "slu_plan_destroy": (None, [P]),
        "slu_plan_get_stats": (C.c_int, [P, C.POINTER(PlanStats)]),
        "slu_last_error": (C.c_char_p, []),
        "slu_debug_poison_lds": (C.c_int, [C.c_int]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):
            raise RuntimeError(f"{LIB_PATH} does not export {name}: rebuild it")
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def as_i64p(a):
    return a.ctypes.data_as(c_i64p)
