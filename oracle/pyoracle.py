"""Python access to the checker (TEST INFRASTRUCTURE ONLY).

* ``oracle_factor`` runs our plain-C restatement (oracle.c -> _build/liboracle.so)
  over the LUstructs of a simulated Pr x Pc grid.
* ``run_reference`` runs the reference pdgstrf harness (_ref/ref_pdgstrf) under
  mpiexec on the same front-end input and returns its per-rank factors.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBORACLE = os.path.join(HERE, "_build", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_pdgstrf")
CONDA = "/opt/conda"

_lib = None


def build():
    """Compile the C restatement (and the reference harness when the
    reference sources are present)."""
    subprocess.run(["make", "-C", HERE, "all"], check=True, capture_output=True)
    if os.path.isdir("/root/reference/SRC"):
        subprocess.run(["make", "-C", HERE, "-j8", "ref"], check=True, capture_output=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBORACLE):
            build()
        _lib = C.CDLL(LIBORACLE)
        for nm in ("oracle_dfactor", "oracle_sfactor", "oracle_zfactor"):
            f = getattr(_lib, nm)
            f.restype = C.c_int
            f.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_int, C.c_int,
                          C.c_double, C.POINTER(C.c_int), C.POINTER(C.c_int),
                          C.POINTER(C.c_double)]
    return _lib


def oracle_factor(lus, nprow, npcol, n, replace_tiny=False, anorm=1.0):
    """Factor in place the LUStruct objects ``lus`` (rank order row*npcol+col)."""
    L = _load()
    arr = (C.c_void_p * len(lus))(*[lu.ptr for lu in lus])
    info, tiny, flops = C.c_int(), C.c_int(), C.c_double()
    fn = {0: L.oracle_dfactor, 1: L.oracle_sfactor, 2: L.oracle_zfactor}[lus[0].dtype]
    rc = fn(nprow, npcol, arr, n, int(replace_tiny), anorm, C.byref(info), C.byref(tiny),
            C.byref(flops))
    if rc != 0:
        raise RuntimeError("oracle failed")
    return {"info": info.value, "tiny": tiny.value, "flops": flops.value}


class BlockSum(C.Structure):
    """blocksum.h's record: per-block fingerprint keyed by global (ib, jb)."""
    _fields_ = [("kind", C.c_int64), ("ib", C.c_int64), ("jb", C.c_int64), ("cnt", C.c_int64),
                ("maxabs", C.c_double), ("wre", C.c_double), ("wim", C.c_double)]


BLOCKSUM_DT = np.dtype([("kind", "<i8"), ("ib", "<i8"), ("jb", "<i8"), ("cnt", "<i8"),
                        ("maxabs", "<f8"), ("wre", "<f8"), ("wim", "<f8")])


def blocksums(lu, Lval=None, Uval=None):
    """Per-block fingerprints (oracle/blocksum.h) of one rank's LUStruct, with
    its own value arrays or the given ones (e.g. a copy of the factors)."""
    L = _load()
    f = L.oracle_blocksums
    f.restype = C.c_int64
    Lv = lu.Lval if Lval is None else Lval
    Uv = lu.Uval if Uval is None else Uval
    v = lu.view
    args = [lu.dtype, lu.nsupers, lu.xsup.ctypes.data_as(C.c_void_p),
            C.cast(v.Lidx, C.c_void_p), C.cast(v.Lidx_off, C.c_void_p),
            Lv.ctypes.data_as(C.c_void_p), C.cast(v.Lval_off, C.c_void_p),
            C.cast(v.Uidx, C.c_void_p), C.cast(v.Uidx_off, C.c_void_p),
            Uv.ctypes.data_as(C.c_void_p), C.cast(v.Uval_off, C.c_void_p),
            C.c_int(lu.nprow), C.c_int(lu.npcol), C.c_int(lu.myrow), C.c_int(lu.mycol)]
    f.argtypes = [C.c_int, C.c_int64] + [C.c_void_p] * 9 + [C.c_int] * 4 + [C.c_void_p]
    n = f(*args, None)
    out = np.zeros(max(n, 1), BLOCKSUM_DT)
    f(*args, out.ctypes.data_as(C.c_void_p))
    return out[:n]


def read_blocksums(path):
    with open(path, "rb") as fh:
        n = int(np.fromfile(fh, np.int64, 1)[0])
        return np.fromfile(fh, BLOCKSUM_DT, n)


def compare_blocksums(mine, ref):
    """Factor parity from per-block fingerprints of two factorizations of the
    same LUstruct (any two process grids): every block present in both, and
    rel_err = max over blocks of max(|d maxabs|, |d wsum| / sqrt(cnt)) / max|ref|
    (|d wsum| / sqrt(cnt) estimates the block's RMS elementwise error: w is a
    fixed pseudo-random projection)."""
    key = lambda a: (a["kind"] * (1 << 42) + a["ib"]) * (1 << 21) + a["jb"]  # noqa: E731
    a = np.sort(mine, order=["kind", "ib", "jb"])
    b = np.sort(ref, order=["kind", "ib", "jb"])
    if len(a) != len(b) or not np.array_equal(key(a), key(b)) or not np.array_equal(a["cnt"], b["cnt"]):
        return {"blocks": int(len(b)), "blocks_mine": int(len(a)), "match": False, "rel_err": None}
    scale = max(float(b["maxabs"].max()), 1e-300)
    dmax = np.abs(a["maxabs"] - b["maxabs"])
    dw = np.hypot(a["wre"] - b["wre"], a["wim"] - b["wim"]) / np.sqrt(np.maximum(b["cnt"], 1))
    return {"blocks": int(len(b)), "values": int(b["cnt"].sum()), "match": True,
            "rel_err": float(max(dmax.max(), dw.max()) / scale),
            "rel_err_maxabs": float(dmax.max() / scale), "rel_err_proj": float(dw.max() / scale)}


def write_matrix_bin(path, A, perm_c=None):
    colptr, rowind, val = A.arrays()
    with open(path, "wb") as fh:
        np.array([A.n, len(rowind), A.dtype, 0 if perm_c is None else 1],
                 dtype=np.int64).tofile(fh)
        colptr.astype(np.int64).tofile(fh)
        rowind.astype(np.int64).tofile(fh)
        val.tofile(fh)
        if perm_c is not None:
            np.asarray(perm_c, dtype=np.int64).tofile(fh)


def have_reference_harness():
    return os.path.exists(REF_BIN) and os.path.exists(os.path.join(CONDA, "bin", "mpiexec"))


def run_reference(A, perm_c, nprow, npcol, relax=60, maxsup=256, lookahead=10,
                  replace_tiny=False, reps=1, want_factors=True, omp_threads=1,
                  timeout=3600, symb_flags=0, want_blocksums=False):
    """Run the reference factorization on nprow*npcol MPI ranks.
    symb_flags: slu_symbolic flags for the LUstruct the harness builds
    (2 = the reference's own sp_colorder + symbfact + pddistribute).
    Returns (stats_dict, [(Lval, Uval) per rank] or None); with
    want_blocksums, stats_dict["blocksums"] holds every rank's per-block
    fingerprints (blocksum.h), concatenated."""
    from superlu_dist_amd.lib import DTYPES, LIB_PATH
    tmp = tempfile.mkdtemp(prefix="slu_ref_")
    try:
        mfile = os.path.join(tmp, "A.bin")
        write_matrix_bin(mfile, A, perm_c)
        outp = os.path.join(tmp, "out") if want_factors else None
        env = dict(os.environ)
        # SLU_SYMB_DEVICE=0: the harness's symbolic stage stays on the host
        # (its ranks must not open the GPU: the box allows 16 processes per
        # GPU, and a 16-rank reference run beside the bench would be 17)
        env.update({"MPICH_CC": "gcc", "OMP_NUM_THREADS": str(omp_threads),
                    "MKL_NUM_THREADS": "1", "MKL_THREADING_LAYER": "SEQUENTIAL", "SLU_SYMB_DEVICE": "0",
                    "LD_LIBRARY_PATH": "/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:" + CONDA + "/lib:" + env.get("LD_LIBRARY_PATH", "")})
        cmd = [os.path.join(CONDA, "bin", "mpiexec"), "-n", str(nprow * npcol), REF_BIN,
               "-lib", LIB_PATH, "-f", mfile, "-r", str(nprow), "-c", str(npcol),
               "-x", str(relax), "-m", str(maxsup), "-l", str(lookahead),
               "-t", str(int(replace_tiny)), "-n", str(reps), "-s", str(symb_flags)]
        if outp:
            cmd += ["-o", outp]
        sums = os.path.join(tmp, "sums") if want_blocksums else None
        if sums:
            cmd += ["-k", sums]
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"reference harness failed: {r.stderr[-2000:]}")
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        stats = json.loads(line)
        if sums:
            stats["blocksums"] = np.concatenate([read_blocksums(f"{sums}.rank{p}.bin")
                                                 for p in range(nprow * npcol)])
        facs = None
        if want_factors:
            npt = DTYPES[A.dtype]
            facs = []
            for p in range(nprow * npcol):
                Lv = np.fromfile(f"{outp}.rank{p}.L.bin", dtype=npt)
                Uv = np.fromfile(f"{outp}.rank{p}.U.bin", dtype=npt)
                facs.append((Lv, Uv))
        return stats, facs
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
