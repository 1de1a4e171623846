"""Benchmark: pdgstrf fp64 GFLOP/s + factor time, 3D 7-point Laplacian n = 1M.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 100]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

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
HBM_PEAK_GBS = 8000.0


def grid_shape(n):
    return {1: (1, 1), 2: (1, 2), 4: (2, 2), 8: (2, 4), 16: (4, 4)}.get(n, (1, n))


def build_lu(nx, pr, pc, myrow, mycol):
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    S = Symbolic(A, nd_order(nx, nx, nx), 60, 256)
    lu = S.distribute(pr, pc, myrow, mycol)
    return A, S, lu


def cpu_baseline(nx_sample, nranks, timeout):
    """Reference pdgstrf (oracle/_ref/ref_pdgstrf: /root/reference sources,
    MPICH + sequential MKL, one rank per core) on the sample problem."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    if not pyoracle.have_reference_harness():
        return None
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order
    pr, pc = grid_shape(nranks)
    A = Csc.stencil(STENCIL_3D7, nx_sample, nx_sample, nx_sample)
    perm = nd_order(nx_sample, nx_sample, nx_sample)
    S = Symbolic(A, perm, 60, 256)
    flops = S.flops()["total"]
    try:
        st, _ = pyoracle.run_reference(A, perm, pr, pc, relax=60, maxsup=256, lookahead=10,
                                       want_factors=False, timeout=timeout)
    except Exception as e:  # noqa: BLE001
        print(f"[bench] cpu baseline failed: {e}", file=sys.stderr)
        return None
    t = st["time_best"]
    return {"value": round(flops / t / 1e9, 2), "unit": "GFLOP/s", "cores": pr * pc,
            "kind": "reference",
            "sample": f"reference pdgstrf (oracle/_ref) on 3D 7-pt Laplacian {nx_sample}^3 "
                      f"(n={nx_sample**3}, {flops:.3e} flops), {pr}x{pc} MPI ranks x 1 thread, "
                      f"MKL sequential; factor time {t:.2f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=100, help="grid points per dimension")
    ap.add_argument("--cpu-sample", type=int, default=80)
    ap.add_argument("--cpu-ranks", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = max(world, 1)
    pr, pc = grid_shape(world)
    myrow, mycol = rank // pc, rank % pc

    from superlu_dist_amd.engine import Comm, Plan
    dist = None
    uid = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        buf = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf[:] = torch.tensor(list(Comm.unique_id()), dtype=torch.uint8)
        dist.broadcast(buf, 0)
        uid = bytes(buf.tolist())

    def barrier():
        if dist is not None:
            dist.barrier()

    t0 = time.time()
    A, S, lu = build_lu(args.n, pr, pc, myrow, mycol)
    t_front = time.time() - t0
    comm = Comm(pr, pc, rank, device=local, uid=uid) if world > 1 else None
    t0 = time.time()
    plan = Plan(lu, comm=comm, timing=True)
    t_plan = time.time() - t0
    t0 = time.time()
    plan.upload()
    t_upload = time.time() - t0
    plan.snapshot()
    anorm = 12.0  # ||A||_1 of the 7-point Laplacian (diag 6, six -1 neighbours)

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

    for _ in range(args.warmup):
        one_step()
    times, schur_ms, schur_big_ms, tot_ms = [], 0.0, 0.0, 0.0
    diag_ms = trsm_ms = 0.0
    for _ in range(args.steps):
        dt, info = one_step()
        times.append(dt)
        st = plan.stats()
        schur_ms += st["t_schur_ms"]
        schur_big_ms += st["t_schur_big_ms"]
        diag_ms += st["t_diag_ms"]
        trsm_ms += st["t_trsm_ms"]
        tot_ms += st["t_total_ms"]
    st = plan.stats()
    t_step = float(np.mean(times))
    flops_all = my_flops
    if dist is not None:
        import torch
        tt = torch.tensor([t_step], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step = float(tt.item())
        ff = torch.tensor([my_flops], dtype=torch.float64)
        dist.all_reduce(ff, op=dist.ReduceOp.SUM)
        flops_all = float(ff.item())

    if rank == 0:
        K = args.steps
        sch_s = schur_ms / 1e3 / K
        achieved = st["schur_flops"] / sch_s / 1e12 if sch_s > 0 else 0.0
        roof = {"bound": "mfma", "achieved": round(achieved, 3),
                "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP64_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                "kernel": "k_schur<double> (fp64 MFMA GEMM + fused scatter)",
                "launches_per_step": st["n_schur_launches"],
                "schur_flops_per_step": st["schur_flops"],
                "kernel_ms_per_step": round(schur_ms / K, 3)}
        big_s = schur_big_ms / 1e3 / K
        if big_s > 0:
            roof["achieved_big_levels"] = round(st["schur_big_flops"] / big_s / 1e12, 3)
        cpu = None
        if not args.no_cpu:
            cpu = cpu_baseline(args.cpu_sample, args.cpu_ranks, timeout=600)
        out = {
            "metric": "pdgstrf fp64 GFLOP/s + factor time, 3D Laplacian n~1M",
            "value": round(flops_all / t_step / 1e9, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (generated 7-point stencil, diag 6 / off -1)",
            "config": {"workload": f"3D 7-point Laplacian {args.n}^3 (n={args.n**3}), nested "
                                   f"dissection, relax 60, maxsup 256",
                       "grid": f"{pr}x{pc}", "nsupers": int(S.nsupers),
                       "flops_per_factorization": flops_all,
                       "nnz_L": S.nnzL, "parallelism": f"2D block-cyclic {pr}x{pc}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "phases_ms_per_step": {"diag_lu": round(diag_ms / K, 3), "trsm": round(trsm_ms / K, 3),
                                   "schur": round(schur_ms / K, 3),
                                   "events_total": round(tot_ms / K, 3)},
            "setup_s": {"frontend": round(t_front, 2), "plan": round(t_plan, 2),
                        "h2d_upload": round(t_upload, 2)},
            "info": info,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
