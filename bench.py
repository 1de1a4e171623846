"""Benchmark: pdgstrf fp64 GFLOP/s + factor time, 3D 7-point Laplacian n = 1M.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--nx 100]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
ranks itself (spawn_ranks); a WORLD_SIZE that differs from --gpus, fewer
visible GPUs than ranks, or communicators that see a different number of ranks
end the run with a non-zero status instead of measuring another grid.

One process per GPU; N GPUs form the near-square 2D process grid of the
reference (1x1, 1x2, 2x2, 2x4).  A step is one numeric factorization
(the hot path, SRC/pdgstrf.c) of the 100^3 7-point Laplacian (diag 6, off -1,
nested-dissection ordering, relax 60 / maxsup 256) with the LU storage already
resident in HBM.  Before each step the original values are restored from a
pristine device copy (outside the timed bracket; the factorization is in place).
Each step is bracketed by a barrier + device synchronize; the reported time is
the max over ranks.  value = algorithmic flops of the whole factorization
(all ranks) / time.

Extra fields: roofline of the dominant kernel (k_schur, fp64 MFMA bound) from
HIP events recorded on the engine's stream during the timed steps, and the
reference CPU pdgstrf (oracle/_ref, MPI + MKL) timed on a bounded sample on
this host.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix (MI355X_MICROARCH.md / SURVEY §8d)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X dense FP32 matrix (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0

# BASELINE.json configs.  The default, lap3d at nx=100, is the
# headline metric's workload (C3 on one GPU); the others are extra
# measurements of the same path in fp64 2D (C2), complex (C4) and fp32 (C5).
WORKLOADS = {
    # name: (stencil kind, dims(nx), dtype, diag, diag_im, metric, routine, dtype label, default nx)
    "lap3d": ("3d7", lambda n: (n, n, n), 0, None, 0.0,
              "pdgstrf fp64 GFLOP/s + factor time, 3D Laplacian n~1M", "pdgstrf", "f64", 100),
    "lap2d": ("2d5", lambda n: (n, n, 1), 0, None, 0.0,
              "pdgstrf fp64 GFLOP/s + factor time, 2D 5-point Laplacian", "pdgstrf", "f64", 1000),
    "helm3d": ("3d7", lambda n: (n, n, n), 2, 6.0 - 0.25, -0.0025,
               "pzgstrf complex fp64 GFLOP/s + factor time, 3D Helmholtz (kh=0.5)", "pzgstrf",
               "c128", 80),
    "st27": ("3d27", lambda n: (n, n, n), 1, None, 0.0,
             "psgstrf fp32 GFLOP/s + factor time, 3D 27-point stencil", "psgstrf", "f32", 120),
}


def log(msg):
    """Progress on stderr (a long GPU job must keep writing, gpurun kills silent ones)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class _StdoutToStderr:
    """Route fd 1 to fd 2 for the duration (gloo prints its connection
    messages to stdout; the driver reads rank 0's stdout for the one JSON
    line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def grid_shape(n):
    return {1: (1, 1), 2: (1, 2), 4: (2, 2), 8: (2, 4), 16: (4, 4)}.get(n, (1, n))


def build_lu(workload, nx, pr, pc, myrow, mycol, ordering="grid", symbolic="reference",
             coarse=None):
    from superlu_dist_amd.frontend import STENCIL_2D5, STENCIL_3D7, STENCIL_3D27, Csc, Symbolic, nd_order
    kind, dims, dtype, diag, diag_im = WORKLOADS[workload][:5]
    kind = {"2d5": STENCIL_2D5, "3d7": STENCIL_3D7, "3d27": STENCIL_3D27}[kind]
    d = dims(nx)
    A = Csc.stencil(kind, *d, diag=diag, diag_im=diag_im, dtype=dtype)
    if ordering == "graph":
        # the library's METIS_NodeND on A'+A (csrc/ordering.cpp), as
        # get_perm_c_dist's METIS_AT_PLUS_A would call it
        from superlu_dist_amd.symbolic import at_plus_a, metis_nodend
        cp, ri, _ = A.arrays()
        perm = metis_nodend(A.n, *at_plus_a(A.n, cp, ri))[0]
    else:
        perm = nd_order(*d)
    if symbolic == "reference":
        # what pdgssvx hands pdgstrf for this perm_c (ColPerm = MY_PERMC):
        # the reference's sp_colorder + symbfact, laid out by its pddistribute
        # (bit-exact restatements, csrc/symbolic.cpp, csrc/distribute.cpp), on
        # every grid as is: the plan amalgamates it (1x1: csrc/amalg.h; 2D
        # grids: the grid relayout of the same header).  3D grids factor the
        # caller's partition, so --grid3d lays the coarse partition out with
        # pddistribute's rules instead (coarse=True, SLU_SYMB_COARSE); the
        # rate always counts the reference partition's work.
        S = Symbolic(A, perm, 60, 256, reference=True, coarse=bool(coarse))
    else:
        # the library front-end's amalgamated partition (chains with <= 10 %
        # explicit zeros; graph ordering: chains through multi-child columns,
        # DESIGN §11)
        S = Symbolic(A, perm, 60, 256, multichild=ordering == "graph")
    lu = S.distribute(pr, pc, myrow, mycol)
    return A, S, lu, perm


def next_rows(plan, A, S, anorm, one_step):
    """SURVEY 8(f) rows 1-2 on the same workload, untimed for value:
    device refill of the factor storage from A (SamePattern_SameRowPerm,
    instead of the PCIe upload of L and U), the triangular solve on the
    device-resident factors with its backward error, and the iterative
    refinement (pdgsrfs) of that solution."""
    import scipy.sparse as sp
    cp, ri, v = A.permuted(S.perm_c).arrays()
    t0 = time.time()
    plan.set_a_pattern(cp, ri)
    t_pat = time.time() - t0
    fills = []
    for _ in range(3):
        plan.fill_a(v)
        fills.append(plan.stats()["t_fill_ms"])
    st = plan.stats()
    lu_bytes = st["lu_bytes"]
    info, _ = plan.factor(anorm)
    plan.sync()
    B = sp.csc_matrix((v, ri, cp), shape=(A.n, A.n))
    xt = np.random.default_rng(1).standard_normal(A.n).astype(v.dtype)
    b = B @ xt
    solves = []
    for _ in range(3):
        x = plan.solve(b)
        solves.append(plan.stats()["t_solve_ms"])
    r = B @ x - b
    berr = float(np.abs(r).max() / (abs(B).sum(axis=1).max() * np.abs(x).max()))
    xb = plan.solve(np.repeat(b[:, None], 8, axis=1))
    t8 = plan.stats()["t_solve_ms"]
    # the panel sums meet through atomics: batch and single solves agree to rounding
    assert np.abs(xb - x[:, None]).max() <= (1e-4 if x.dtype == np.float32 else 1e-12) * np.abs(x).max()
    xr, rberr, rsteps = plan.refine(b, x)
    t_ref = plan.stats()["t_refine_ms"]
    fill_ms = min(fills)
    return {"fill": {"kernel": "memset L/U + k_fill_a (nnz(A) scatter)",
                     "device_ms": round(fill_ms, 3),
                     "hbm_gbps": round((lu_bytes + len(v) * (8 + v.itemsize * 2)) / fill_ms / 1e6, 1),
                     "pattern_setup_s": round(t_pat, 3), "nnz_A": int(len(v)),
                     "lu_bytes": lu_bytes, "factor_info_after_fill": int(info)},
            "solve": {"device_ms": round(min(solves), 3), "nrhs": 1, "berr": berr,
                      "device_ms_8rhs": round(t8, 3),
                      "fwd_err": float(np.abs(x - xt).max() / np.abs(xt).max())},
            "refine": {"device_ms": round(t_ref, 3), "steps": int(rsteps[0]),
                       "berr_componentwise": float(rberr[0]),
                       "fwd_err": float(np.abs(xr - xt).max() / np.abs(xt).max())}}


def abi_leg(lu, anorm, factor_ms, fingerprint=None):
    """utime[FACT] of the drop-in path: pdgstrf called through the C ABI the
    way pdgssvx calls it (SRC/pdgssvx.c:1174-1180) -- plan build, H2D of the
    host LUstruct's values, factorization and D2H of the factors into the
    same host arrays, wall-clocked around the call -- and the same sequence
    through the engine API for the breakdown.  The H2D overlaps the plan
    build and each level's factors go back while later levels run."""
    from superlu_dist_amd import capi
    from superlu_dist_amd.engine import Plan
    L0, U0 = lu.Lval.copy(), lu.Uval.copy()
    walls = []
    if os.environ.get("SLU_ABI_BREAKDOWN_ONLY"):
        walls = [0.0, 0.0, 0.0]
    # first call of the process (Fact = DOFACT: plan build, HIP / pinned-pool
    # set-up), then the refactorization as pdgssvx calls it (Fact =
    # SamePattern_SameRowPerm: the cached plan, shallow structure digest),
    # then a DOFACT call on the same arrays (cached plan, full digest)
    opt = capi.default_options()
    for fact in ([] if walls else [0, 2, 0]):
        lu.Lval[:] = L0
        lu.Uval[:] = U0
        opt.Fact = fact
        t = time.perf_counter()
        rv, info, st = capi.pxgstrf(lu, anorm, options=opt)
        walls.append((time.perf_counter() - t) * 1e3)
        assert rv == 0 and info == 0, (rv, info)
    # the drop-in's factors, fingerprinted for the parity check of the
    # cpu_baseline leg (oracle/blocksum.h) while they are in the host arrays
    sums = fingerprint(lu) if fingerprint else None
    Lf = lu.Lval.copy()
    lu.Lval[:] = L0
    lu.Uval[:] = U0
    t = time.perf_counter()
    p = Plan(lu, overlap_upload=True, overlap_download=True)
    p.upload()
    t_fact = time.perf_counter()
    p.factor(anorm)
    t_end = time.perf_counter()
    p.download()
    st = p.stats()
    del p
    # atomics order the sums differently run to run: compare, do not demand bits
    same = float(np.abs(Lf[:-1] - lu.Lval[:-1]).max() / max(np.abs(Lf[:-1]).max(), 1e-300))
    lu.Lval[:] = L0
    lu.Uval[:] = U0
    h2d = st["t_upload_ms"]
    pcie = 56.0  # GB/s, registered H2D / D2H on the box (profiles/r02_pcie_micro.json)
    return {"utime_fact_ms": round(walls[1], 1), "utime_fact_ms_first_call": round(walls[0], 1),
            "utime_fact_ms_cached_dofact": round(walls[2], 1),
            "bar_ms": round(1.2 * (h2d + factor_ms), 1),
            "breakdown_ms": {"plan_build": round(st["t_plan_ms"], 1),
                             "h2d_values": round(h2d, 1),
                             "h2d_wait_after_plan": round(st["t_upload_wait_ms"], 1),
                             "factor_with_overlapped_d2h": round((t_end - t_fact) * 1e3, 1),
                             "d2h_span": round(st["t_d2h_ms"], 1),
                             "d2h_after_factor": round(st["t_d2h_tail_ms"], 1),
                             "total": round((t_end - t) * 1e3, 1)},
            "h2d_gbs": round(st["h2d_bytes"] / h2d / 1e6, 1) if h2d else None,
            "d2h_copies": int(st["n_d2h_copies"]),
            "pcie_floor_ms": round((st["h2d_bytes"] + st["d2h_bytes"]) / pcie / 1e6, 1),
            "factors_rel_diff_abi_vs_engine": same,
            "note": "factor_ms in bar_ms = ms_per_step (HBM-resident); h2d = staged H2D of the "
                    "L/U values (hostio.h); D2H rides under the factorization"}, sums


def device_resident_child(nx):
    """Child process of the N=1 bench (``--device-resident-child``): the
    device-resident drop-in (libslu_mi355x_solve.so) as
    pdgssvx drives it (SRC/pdgssvx.c:1146-1180 and its SOLVE phase) on the
    headline workload: this library's pddistribute keeps A, pdgstrf fills the
    factor storage on the device and leaves the factors in HBM, pdgstrs solves
    on them.  Then the refactorization pddrive3.c does (Fact =
    SamePattern_SameRowPerm: pddistribute refills the values, pdgstrf reuses
    the cached plan).  Each call wall-clocked as pdgssvx's utime does.  A
    fresh process, HIP initialised before the first call (reported apart)."""
    import ctypes as C
    from superlu_dist_amd import capi
    from superlu_dist_amd import symbolic as SY
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, nd_order
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    n = A.n
    cp, ri, v = A.arrays()
    t0 = time.perf_counter()
    co = SY.sp_colorder(n, n, cp, ri, nd_order(nx, nx, nx), SY.MY_PERMC)
    sb = SY.symbfact(n, n, co.colbeg, co.colend, SY.relabel_rows(ri, co.perm_c), co.etree, 60, 256)
    t_symb = time.perf_counter() - t0
    # the 7-point Laplacian is symmetric: A's CSR arrays are its CSC arrays;
    # pdgssvx maps the column indices by perm_c before pddistribute
    s = capi.DeviceResidentSystem(n, cp, co.perm_c[ri], v, co.perm_c, co.etree, sb.xsup, sb.supno,
                                  sb.xlsub, sb.lsub, sb.xusub, sb.usub, one_norm(A))
    xt = np.random.default_rng(3).standard_normal(n)
    import scipy.sparse as sp
    b = sp.csc_matrix((v, ri, cp), shape=(n, n)) @ xt
    t0 = time.perf_counter()
    hip = C.CDLL("libamdhip64.so")
    hip.hipFree(None)
    t_hip = time.perf_counter() - t0
    rec = {"symbolic_s": round(t_symb, 2), "hip_init_ms": round(t_hip * 1e3, 1), "calls": []}
    for i, fact in enumerate([0, capi.SAMEPATTERN_SAMEROWPERM, capi.SAMEPATTERN_SAMEROWPERM]):
        t0 = time.perf_counter()
        s.distribute(fact)
        t1 = time.perf_counter()
        rv, info, ops = s.factor()
        t2 = time.perf_counter()
        x = s.solve(b)
        t3 = time.perf_counter()
        assert rv == 0 and info == 0, (rv, info)
        rec["calls"].append({"fact": ["DOFACT", "", "SamePattern_SameRowPerm"][fact],
                             "distribute_ms": round((t1 - t0) * 1e3, 1),
                             "utime_fact_ms": round((t2 - t1) * 1e3, 1),
                             "solve_ms": round((t3 - t2) * 1e3, 1),
                             "fwd_err": float(np.abs(x - xt).max() / np.abs(xt).max()),
                             "ops_fact": ops})
    c = rec["calls"]
    rec.update({"utime_fact_ms_first_call": c[0]["utime_fact_ms"],
                "utime_fact_ms_refactor": min(x["utime_fact_ms"] for x in c[1:]),
                "solve_ms": min(x["solve_ms"] for x in c),
                "note": "libslu_mi355x_solve.so: pddistribute keeps A, pdgstrf fills L/U on the "
                        "device and keeps the factors in HBM, pdgstrs solves on them (1 rhs); "
                        "refactor = Fact SamePattern_SameRowPerm (refill + cached plan)"})
    print(json.dumps(rec), flush=True)


def device_resident_leg(nx):
    """Runs device_resident_child in a fresh process (its LUstruct and HBM
    plan are freed with it); returns its record or an error note."""
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--device-resident-child",
                            "--nx", str(nx)], capture_output=True, text=True, timeout=900)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if os.environ.get("SLU_BENCH_CHILD_ERR"):  # diagnostics: the child's stderr
            with open(os.environ["SLU_BENCH_CHILD_ERR"], "w") as f:
                f.write(r.stderr)
        if r.returncode != 0 or not line:
            return {"error": f"exit {r.returncode}: {r.stderr[-1500:]}"}
        return json.loads(line[-1])
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}


def one_norm(A):
    """||A||_1 (max column sum of |a_ij|), the anorm pdgssvx passes to pdgstrf."""
    colptr, _, val = A.arrays()
    return float(np.add.reduceat(np.abs(val).astype(np.float64), colptr[:-1]).max())


def gpu_fingerprints(lu):
    """cpu_baseline leg, the checker: per-block fingerprints (max |v| and a
    fixed random projection, oracle/blocksum.h) of the factors in ``lu``'s
    host arrays, keyed by global block, to compare with the reference's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    return pyoracle.blocksums(lu)


def cpu_baseline(A, perm, nx, nranks, timeout, flops, symbolic="reference", gpu_sums=None):
    """Reference pdgstrf (oracle/_ref/ref_pdgstrf: /root/reference sources,
    MPICH + sequential MKL, one rank per core) on the same matrix, ordering
    and LUstruct (the reference's own symbolic stage for symbolic ==
    "reference"), and -- given the GPU factors' fingerprints -- the parity of
    the full-size factors: the reference's per-block fingerprints from its
    own grid against the GPU's (oracle/pyoracle.compare_blocksums)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    if not pyoracle.have_reference_harness():
        return None, None
    pr, pc = grid_shape(nranks)
    import threading
    done = threading.Event()

    def heartbeat():  # a silent GPU job is taken for hung: say the CPU run is alive
        t0 = time.time()
        while not done.wait(30):
            log(f"  reference pdgstrf running ({time.time() - t0:.0f} s)")
    threading.Thread(target=heartbeat, daemon=True).start()
    try:
        st, _ = pyoracle.run_reference(A, perm, pr, pc, relax=60, maxsup=256, lookahead=10,
                                       want_factors=False, timeout=timeout,
                                       symb_flags=2 if symbolic == "reference" else 0,
                                       want_blocksums=gpu_sums is not None)
    except Exception as e:  # noqa: BLE001
        print(f"[bench] cpu baseline failed: {e}", file=sys.stderr)
        return None, None
    finally:
        done.set()
    t = st["time_best"]
    parity = None
    if gpu_sums is not None:
        parity = pyoracle.compare_blocksums(gpu_sums, st["blocksums"])
        parity.update({"tolerance": 1e-12, "ok": bool(parity["match"] and parity["rel_err"] <= 1e-12),
                       "against": f"reference pdgstrf on a {pr}x{pc} grid (oracle/_ref/ref_pdgstrf)",
                       "gpu_factors": "drop-in pdgstrf (C ABI) factors, 1x1",
                       "method": "per-block fingerprints keyed by global (ib, jb): max|v| and a "
                                 "fixed pseudo-random projection (oracle/blocksum.h); rel_err = "
                                 "max over blocks of max(|d maxabs|, |d proj|/sqrt(cnt)) / max|ref|"})
    return ({"value": round(flops / t / 1e9, 2), "unit": "GFLOP/s", "cores": pr * pc,
             "kind": "reference",
             "sample": f"reference pdgstrf (oracle/_ref) on the same 3D 7-pt Laplacian {nx}^3 "
                       f"and LUstruct (n={nx**3}, {flops:.3e} flops), {pr}x{pc} MPI ranks x 1 "
                       f"thread, MKL sequential; factor time {t:.2f} s"}, parity)


def preflight_parity(args, comm, pr, pc, myrow, mycol, rank, dist):
    """Multi-rank runs, the checker (the reference checks
    every grid run, TEST/pdtest.c:372-393): before the timed run, factor the
    same workload at a small size (--preflight-nx, default 40) through the
    same transport and grid, gather every rank's per-block fingerprints of
    its factors (oracle/blocksum.h) to rank 0 and compare them with the
    reference pdgstrf's on the same grid (oracle/_ref/ref_pdgstrf, CPU).
    Returns the parity record on rank 0 (None elsewhere)."""
    from superlu_dist_amd.engine import Plan
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    nx = args.preflight_nx
    t0 = time.time()
    A, S, lu, perm = build_lu(args.workload, nx, pr, pc, myrow, mycol, args.ordering, args.symbolic)
    p = Plan(lu, comm=comm)
    p.upload()
    info, _ = p.factor(one_norm(A))
    p.download()
    nsup = int(p.stats()["nsupers"])
    del p
    mine = pyoracle.blocksums(lu)
    allsums = [None] * (pr * pc)
    dist.all_gather_object(allsums, mine)
    infos = [None] * (pr * pc)
    dist.all_gather_object(infos, int(info))
    t_gpu = time.time() - t0
    if rank != 0:
        return None
    rec = {"preflight": f"{args.workload} nx={nx} (n={A.n}), {pr}x{pc} grid, factored on the "
                        f"GPUs through the same transport before the timed run",
           "against": f"reference pdgstrf on a {pr}x{pc} grid (oracle/_ref/ref_pdgstrf)",
           "tolerance": 1e-12 if lu.Lval.dtype.itemsize >= 8 else 1e-5,
           "info": infos, "nsupers_factored_rank0": nsup, "gpu_s": round(t_gpu, 2),
           "method": "per-block fingerprints keyed by global (ib, jb), all ranks "
                     "(oracle/blocksum.h; pyoracle.compare_blocksums)"}
    if not pyoracle.have_reference_harness():
        rec.update(ok=None, note="oracle/_ref not built: parity unchecked")
        return rec
    try:
        st, _ = pyoracle.run_reference(A, perm, pr, pc, relax=60, maxsup=256, lookahead=10,
                                       want_factors=False, timeout=600,
                                       symb_flags=2 if args.symbolic == "reference" else 0,
                                       want_blocksums=True)
    except Exception as e:  # noqa: BLE001
        rec.update(ok=False, error=f"reference run failed: {e}")
        return rec
    c = pyoracle.compare_blocksums(np.concatenate(allsums), st["blocksums"])
    rec.update({k: (float(v) if isinstance(v, (float, np.floating)) else v) for k, v in c.items()})
    rec["ok"] = bool(c["match"] and c["rel_err"] <= rec["tolerance"] and max(infos) == 0)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="lap3d",
                    help="lap3d = C3 (headline), lap2d = C2, helm3d = C4 (complex), st27 = C5 (fp32)")
    ap.add_argument("--nx", type=int, default=None, help="grid points per dimension")
    ap.add_argument("--ordering", choices=["grid", "graph"], default="grid",
                    help="grid: geometric nested dissection of the stencil grid (the headline "
                         "configuration); graph: the library's METIS_NodeND on A'+A")
    ap.add_argument("--symbolic", choices=["reference", "frontend"], default="reference",
                    help="reference: pdgssvx's own sp_colorder + symbfact + pddistribute (the "
                         "LUstruct the reference hands pdgstrf for this perm_c; headline); "
                         "frontend: the library front-end's amalgamated supernodes")
    ap.add_argument("--cpu-ranks", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-next", action="store_true",
                    help="skip the device fill / solve measurements (SURVEY 8(f) rows 1-2)")
    ap.add_argument("--no-abi", action="store_true",
                    help="skip the drop-in pdgstrf leg (utime[FACT] incl. host copies)")
    ap.add_argument("--level-log", action="store_true",
                    help="per-level phase breakdown of the last step on stderr")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the serialized (single-stream) profiling step: for rocprofv3 runs")
    ap.add_argument("--grid3d", default=None, metavar="PRxPCxPZ",
                    help="3D process grid (pdgstrf3d): PZ layers of a PR x PC grid, PR*PC*PZ = "
                         "--gpus; the layers factor the etree's forests and reduce the "
                         "ancestors between them (default: the 2D grid of --gpus ranks)")
    ap.add_argument("--preflight-nx", type=int, default=40,
                    help="multi-rank runs: grid points per dimension of the parity preflight "
                         "(0 skips it)")
    ap.add_argument("--rank-timeout", type=float, default=float(os.environ.get("SLU_BENCH_TIMEOUT_S", 1500)),
                    help="--gpus N without a launcher: seconds before the spawned ranks are killed")
    ap.add_argument("--device-resident-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-device-resident", action="store_true",
                    help="skip the device-resident drop-in leg (libslu_mi355x_solve.so)")
    ap.add_argument("--host-transport", action="store_true",
                    help="REHEARSAL ONLY: several ranks on one GPU through the host-staged "
                         "point-to-point test transport (the RCCL send / receive pairs over "
                         "gloo; RCCL refuses duplicate devices); not a measurement")
    args = ap.parse_args()
    W = WORKLOADS[args.workload]
    if args.nx is None:
        args.nx = W[8]
    if args.device_resident_child:
        device_resident_child(args.nx)
        return
    if args.workload != "lap3d":
        args.no_cpu = True  # the CPU baseline is the reference on the headline workload

    # the library's exchange watchdog is opt-in: armed for the bench's ranks
    # (a hung exchange then ends with a diagnosis and exit 86, csrc/watchdog.h)
    os.environ.setdefault("SLU_WATCHDOG_S", "300")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` without a launcher: start the N ranks here,
        # before anything touches the GPU (torch.distributed.run does the same)
        sys.exit(spawn_ranks(args.gpus, args.rank_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus {args.gpus}: refusing to measure a different grid")
        sys.exit(2)
    pz = 1
    if args.grid3d:
        pr, pc, pz = (int(x) for x in args.grid3d.lower().split("x"))
        if pr * pc * pz != world or pz & (pz - 1):
            log(f"--grid3d {args.grid3d} does not make {world} ranks with a power-of-two depth")
            sys.exit(2)
    else:
        pr, pc = grid_shape(world)
    layer, r2 = rank // (pr * pc), rank % (pr * pc)
    myrow, mycol = r2 // pc, r2 % pc

    from superlu_dist_amd.engine import Comm, Plan
    dist = None
    uid = None
    grid = None
    if world > 1:
        # torch first: it bundles a ROCm runtime with the same sonames as the
        # system one libslu_mi355x.so links; the first loaded is shared.
        import torch
        import torch.distributed as dist
        with _StdoutToStderr():
            dist.init_process_group("gloo")
        if args.host_transport:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            from gridrun import GlooGrid
            with _StdoutToStderr():
                grid = GlooGrid(rank, pr, pc, pz)
            local = 0
        else:
            ndev = torch.cuda.device_count()
            if ndev < world:
                log(f"{world} ranks but {ndev} visible GPUs: RCCL needs one GPU per rank "
                    f"(--host-transport rehearses several ranks on one GPU)")
                sys.exit(2)
            buf = torch.zeros(128, dtype=torch.uint8)
            if rank == 0:
                buf[:] = torch.tensor(list(Comm.unique_id()), dtype=torch.uint8)
            dist.broadcast(buf, 0)
            uid = bytes(buf.tolist())

    def barrier():
        if dist is not None:
            dist.barrier()

    t0 = time.time()
    gname = f"{pr}x{pc}" + (f"x{pz}" if pz > 1 else "")
    log(f"front-end {args.workload} nx={args.nx} grid {gname}")
    A, S, lu, perm = build_lu(args.workload, args.nx, pr, pc, myrow, mycol, args.ordering,
                              args.symbolic, coarse=pz > 1)
    t_front = time.time() - t0
    log(f"front-end {t_front:.1f} s, {S.nsupers} supernodes")
    if world == 1:
        comm = None
    elif grid is not None:
        # the RCCL transport's send / receive pairs, host-staged over gloo
        comm = (Comm.host_p2p3d(pr, pc, pz, rank, 0, grid.p2p) if pz > 1 else
                Comm.host_p2p(pr, pc, rank, 0, grid.p2p))
    else:
        comm = (Comm.grid3d(pr, pc, pz, rank, device=local, uid=uid) if pz > 1 else
                Comm(pr, pc, rank, device=local, uid=uid))
    if comm is not None:
        sizes = (comm.size(0), comm.size(1), comm.size(2), comm.size(3) if pz > 1 else 1)
        if sizes != (pr * pc, pc, pr, pz):
            log(f"the communicators see {sizes} ranks (layer, row, column, layers), expected "
                f"{(pr * pc, pc, pr, pz)}")
            sys.exit(3)
        log(f"communicators: layer {sizes[0]}, row {sizes[1]}, column {sizes[2]}, "
            f"{sizes[3]} layers")
    parity_pre = None
    if world > 1 and pz == 1 and args.preflight_nx > 0 and not args.roofline_only:
        log(f"parity preflight nx={args.preflight_nx} on the {gname} grid")
        parity_pre = preflight_parity(args, comm, pr, pc, myrow, mycol, rank, dist)
        if rank == 0:
            log(f"parity preflight: ok={parity_pre.get('ok')} rel_err={parity_pre.get('rel_err')}")
    t0 = time.time()
    plan = Plan(lu, comm=comm, timing=2 if args.level_log else 1)
    t_plan = time.time() - t0
    t0 = time.time()
    plan.upload()
    t_upload = time.time() - t0
    plan.snapshot()
    anorm = one_norm(A)  # 12 for the 7-point Laplacian (diag 6, six -1 neighbours)

    st0 = plan.stats()
    my_flops = st0["schur_flops"] + st0["panel_flops"]

    def one_step():
        plan.restore()
        barrier()
        plan.sync()
        t = time.perf_counter()
        info, tiny = plan.factor(anorm)
        plan.sync()
        dt = time.perf_counter() - t
        barrier()
        return dt, info

    log("plan + upload done; warmup")
    for _ in range(args.warmup):
        one_step()
    log(f"timed steps: {args.steps}")
    if args.roofline_only:
        args.steps = 0
    times = []
    acc = {k: 0.0 for k in ("t_schur_ms", "t_schur_big_ms", "t_diag_ms", "t_trsm_ms",
                            "t_comm_ms", "t_total_ms")}
    for _ in range(args.steps):
        dt, info = one_step()
        times.append(dt)
        st = plan.stats()
        for k in acc:
            acc[k] += st[k]
    # kernel-level roofline: one more factorization with every launch on one
    # stream, so k_schur_big launch durations are not stretched by the
    # look-ahead kernels running beside them (not part of the timed steps)
    plan.set_timing(2 if args.level_log else 1, serial=True)  # level log: serialized kernel times
    one_step()
    sst = plan.stats()
    plan.set_timing(2 if args.level_log else 1, serial=False)
    st = plan.stats()
    nxt = None
    if world == 1 and not args.no_next and not args.roofline_only:
        log("next rows (fill / solve / refine)")
        nxt = next_rows(plan, A, S, anorm, one_step)
    abi = gpu_sums = None
    want_cpu = rank == 0 and world == 1 and not args.no_cpu and not args.roofline_only
    if world == 1 and not args.no_abi and not args.roofline_only:
        t_step_local = float(np.mean(times)) * 1e3
        del plan
        log("drop-in pdgstrf leg (utime[FACT])")
        abi, gpu_sums = abi_leg(lu, anorm, t_step_local,
                                fingerprint=gpu_fingerprints if want_cpu else None)
        # (a fresh process's first drop-in call, after the headline: on a box
        # whose HBM no process has mapped yet, the first 16.8 GB allocation
        # alone takes ~0.5 s instead of ~0.06 s -- DESIGN section 16)
        if args.workload == "lap3d" and args.ordering == "grid" and not args.no_device_resident:
            log("device-resident drop-in leg (libslu_mi355x_solve.so, child process)")
            abi["device_resident"] = device_resident_leg(args.nx)
            abi["device_resident"]["refactor_vs_ms_per_step"] = (
                round(abi["device_resident"]["utime_fact_ms_refactor"] / t_step_local, 3)
                if "utime_fact_ms_refactor" in abi["device_resident"] else None)
    if args.roofline_only:
        if rank == 0:
            print(json.dumps({"roofline_only": True, "t_schur_big_ms": sst["t_schur_big_ms"],
                              "n_schur_big_launches": sst["n_schur_big_launches"],
                              "t_total_ms": sst["t_total_ms"]}), flush=True)
        return
    t_step = float(np.mean(times))
    flops_all = my_flops
    ref_work = S.ref_flops() if args.symbolic == "reference" else None
    if dist is not None:
        import torch
        tt = torch.tensor([t_step], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step = float(tt.item())
        ff = torch.tensor([my_flops], dtype=torch.float64)
        dist.all_reduce(ff, op=dist.ReduceOp.SUM)
        flops_all = float(ff.item())
    layers3d = None
    if pz > 1:
        # per-layer phase times of the last timed step (rank 0 of each layer)
        import torch.distributed as tdist
        mine = {"layer": layer, "factored": int(st["nsupers"]), "phase_last": int(st["phase_last"]),
                "phase_ms": [round(x, 3) for x in st["t_phase_ms"][:int(st["phase_last"]) + 1]],
                "zreduce_ms": round(st["t_zreduce_ms"], 3),
                "flops": my_flops, "comm_gb": round(st["comm_bytes"] / 1e9, 3)}
        allm = [None] * world
        tdist.all_gather_object(allm, mine)
        layers3d = [m for i, m in enumerate(allm) if i % (pr * pc) == 0]
    if ref_work is not None:
        # the reference partition's algorithmic work (what pdgstrf does on the
        # LUstruct pdgssvx builds; the coarse partition adds explicit zeros)
        flops_all = ref_work["total"]

    if rank == 0:
        K = args.steps
        dtype = W[2]
        peak = FP32_MFMA_PEAK_TFLOPS if dtype == 1 else FP64_MFMA_PEAK_TFLOPS
        if dtype == 2:
            # complex tiles are 128 rows x 64 columns (4 real MFMAs per complex
            # multiply-add, kernels.h BigCfg<zc>)
            kname = "k_schur_big<zc> (128x64 complex fp64 MFMA GEMM + fused scatter)"
            tkey = "k_schur_big<zc>"
        else:
            tn = "double" if dtype == 0 else "float"
            kname = f"k_schur_big<{tn}> (128x128 {W[7]} MFMA GEMM + fused scatter)"
            tkey = f"k_schur_big<{tn}>"
        ker_ms, ker_flops = sst["t_schur_big_ms"], sst["schur_big_flops"]
        launches = max(int(sst["n_schur_big_launches"]), 1)
        achieved = ker_flops / (ker_ms / 1e3) / 1e12 if ker_ms > 0 else 0.0
        roof = {"bound": "mfma", "achieved": round(achieved, 3),
                "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4),
                "traffic": pmc_traffic(args.workload, args.nx, pr, pc, tkey),
                "kernel": kname,
                "launches_per_step": launches,
                "flops_per_launch": ker_flops / launches,
                "avg_launch_ms": round(ker_ms / launches, 4),
                "timer": "HIP events around each launch of the kernel, in one extra "
                         "factorization with all launches on one stream (untimed for value)",
                "serial_factor_ms": round(sst["t_total_ms"], 3),
                "all_schur_tflops": round(st["schur_flops"] / (acc["t_schur_ms"] / 1e3 / K) / 1e12,
                                          3) if acc["t_schur_ms"] else None}
        cpu = parity = None
        if want_cpu:
            log(f"cpu baseline (reference pdgstrf, {args.nx}^3, {args.cpu_ranks} ranks)")
            cpu, parity = cpu_baseline(A, perm, args.nx, args.cpu_ranks, 900, flops_all,
                                       args.symbolic, gpu_sums)
        out = {
            "metric": W[5],
            "value": round(flops_all / t_step / 1e9, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": W[7],
            "data": f"synthetic (generated {W[0]} stencil matrix, ||A||_1 = {anorm:g})",
            "config": {"workload": f"{args.workload}: {W[0]} stencil {'x'.join(map(str, W[1](args.nx)))} "
                                   f"(n={A.n}), {'graph nested dissection (METIS_NodeND)' if args.ordering == 'graph' else 'nested dissection'}, relax 60, maxsup 256, {W[6]}",
                       "symbolic": ("reference sp_colorder + symbfact + pddistribute (ColPerm = MY_PERMC)"
                                    if args.symbolic == "reference" else "library front-end (amalgamated)"),
                       "grid": gname,
                       "nsupers": ref_work["nsupers"] if ref_work else int(S.nsupers),
                       "nsupers_factored": int(st0["nsupers"]),
                       "flops_per_factorization": flops_all,
                       "nnz_L": S.nnzL,
                       "parallelism": (f"3D: {pz} layers (etree forests, ancestor reductions "
                                       f"between layers) of 2D block-cyclic {pr}x{pc}" if pz > 1
                                       else f"2D block-cyclic {pr}x{pc}"),
                       "transport": ("host-staged gloo point-to-point (REHEARSAL, not a measurement)"
                                     if grid is not None else
                                     (f"rccl ({world} ranks, row/column"
                                      f"{'/layer' if pz > 1 else ''} communicators)"
                                      if world > 1 else "none")),
                       "hbm_gb_rank0": round((st0["lu_bytes"] + st0["index_bytes"] +
                                              st0["comm_buf_bytes"]) / 1e9, 2),
                       "comm_ring_gb_rank0": round(st0["comm_buf_bytes"] / 1e9, 3),
                       "comm_volume_gb_rank0": round(st0["comm_bytes"] / 1e9, 3)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity if parity is not None else parity_pre,
            "next_rows": nxt,
            "abi_pdgstrf": abi,
            "phases_ms_per_step_rank0": {k[2:-3]: round(v / K, 3) for k, v in acc.items()},
            "layers3d": layers3d,
            "setup_s": {"frontend": round(t_front, 2), "plan": round(t_plan, 2),
                        "h2d_upload_pcie": round(t_upload, 2)},
            "info": info,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def spawn_ranks(n, timeout_s=1500.0):
    """One child process per rank with the torch.distributed.run environment
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT); rank 0's
    stdout is ours (the one JSON line), the others' goes to stderr.  When a
    rank fails, or the ranks are still running after timeout_s seconds, the
    others are terminated (killed 15 s later) instead of waiting for a peer
    that is gone: a rank whose exchange never completes ends through the
    engine's watchdog (exit 86, csrc/watchdog.h), its peers through this.
    Returns the first non-zero exit status (0 if all ranks succeeded)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + sys.argv, env=env,
                                      stdout=None if r == 0 else sys.stderr))
    deadline = time.time() + timeout_s
    codes = [None] * n
    why = None
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        failed = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
        if failed and any(c is None for c in codes):
            why = f"rank {failed[0][0]} exited with {failed[0][1]}"
        elif time.time() > deadline and any(c is None for c in codes):
            why = f"ranks still running after {timeout_s:.0f} s"
        if why:
            log(f"{why}: terminating the other ranks")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            t_kill = time.time() + 15
            for i, p in enumerate(procs):
                try:
                    codes[i] = p.wait(max(0.1, t_kill - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    codes[i] = p.wait()
            break
        time.sleep(0.2)
    log(f"ranks exited with {codes}")
    if why and all(c == 0 or c < 0 for c in codes):
        return 124
    return next((c for c in codes if c not in (0, None) and c > 0), next((c for c in codes if c), 0))


def pmc_traffic(workload, nx, pr, pc, kernel):
    """HBM bytes per launch of the roofline kernel from the committed
    rocprofv3 PMC passes (profiles/traffic.json, written by
    tools/pmc_traffic.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) for
    this exact workload, else None."""
    f = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    return d.get(f"{workload}_{nx}_{pr}x{pc}", {}).get(kernel)


if __name__ == "__main__":
    main()
