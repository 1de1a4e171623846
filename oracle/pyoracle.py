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
                  timeout=3600):
    """Run the reference factorization on nprow*npcol MPI ranks.
    Returns (stats_dict, [(Lval, Uval) per rank] or None)."""
    from superlu_dist_amd.lib import DTYPES, LIB_PATH
    tmp = tempfile.mkdtemp(prefix="slu_ref_")
    try:
        mfile = os.path.join(tmp, "A.bin")
        write_matrix_bin(mfile, A, perm_c)
        outp = os.path.join(tmp, "out") if want_factors else None
        env = dict(os.environ)
        env.update({"MPICH_CC": "gcc", "OMP_NUM_THREADS": str(omp_threads),
                    "MKL_NUM_THREADS": "1", "MKL_THREADING_LAYER": "SEQUENTIAL",
                    "LD_LIBRARY_PATH": "/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:" + CONDA + "/lib:" + env.get("LD_LIBRARY_PATH", "")})
        cmd = [os.path.join(CONDA, "bin", "mpiexec"), "-n", str(nprow * npcol), REF_BIN,
               "-lib", LIB_PATH, "-f", mfile, "-r", str(nprow), "-c", str(npcol),
               "-x", str(relax), "-m", str(maxsup), "-l", str(lookahead),
               "-t", str(int(replace_tiny)), "-n", str(reps)]
        if outp:
            cmd += ["-o", outp]
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"reference harness failed: {r.stderr[-2000:]}")
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        stats = json.loads(line)
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
