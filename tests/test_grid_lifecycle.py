"""Several plans, LUstructs and communicators in one process per rank (the
life cycle of a long-running pdgssvx caller: gridinit / factor / gridexit
repeated).  Every factorization must match the oracle's, whatever the
process did before.  GPU (host-staged broadcast transport, ranks sharing the
box's GPU, as the drop-in's MPI transport)."""
import functools
import os
import traceback

import numpy as np
import pytest

import cases
import pyoracle
from gridrun import GlooGrid, free_port
from superlu_dist_amd.frontend import STENCIL_3D7, Symbolic
from test_oracle import TOL


def _recipe(nx, pr, pc, reference):
    return cases.stencil_case(STENCIL_3D7, (nx, nx, nx), 0, (pr, pc), 60, 256, reference)


def _worker(rank, world, port, pr, pc, nx, reference, schedule, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from superlu_dist_amd.engine import Comm, Plan
        A, perm, dtype, _, relax, maxsup, tiny = _recipe(nx, pr, pc, reference)[:7]
        gg = GlooGrid(rank, pr, pc)
        res = {}
        comm = None
        for it, what in enumerate(schedule):
            if comm is None or "comm" in what:
                comm = Comm.host(pr, pc, rank, 0, gg.bcast)
            S = Symbolic(A, perm, relax, maxsup, reference=reference)
            lu = S.distribute(pr, pc, gg.myrow, gg.mycol)
            p = Plan(lu, comm=comm, replace_tiny=tiny)
            p.upload()
            info, _ = p.factor(cases.anorm(A))
            p.download()
            del p
            # (copies: lu's arrays are freed with it on the next iteration)
            res[f"L{it}"], res[f"U{it}"], res[f"info{it}"] = lu.Lval.copy(), lu.Uval.copy(), info
            if "drop" in what:
                del comm
                comm = None
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        with open(os.path.join(out_dir, f"rank{rank}.err"), "w") as fh:
            fh.write(traceback.format_exc())
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("reference", [False, True])
@pytest.mark.parametrize("schedule", [("same", "same", "same"), ("comm", "comm+drop", "comm")])
def test_repeated_factorizations_in_one_process(reference, schedule, tmp_path):
    """Three factorizations per rank in one process on a 2x2 grid: the same
    communicator each time, or a new one each time (the previous one dropped
    as superlu_gridexit drops it); reference = the structure pdgssvx builds
    (fine partition, grid amalgamation in the plan)."""
    import multiprocessing as mp
    pr, pc, nx = 2, 2, 16
    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 4, port, pr, pc, nx, reference, schedule, str(tmp_path)))
             for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(400)
    bad = []
    for r, p in enumerate(procs):
        if p.is_alive():
            p.kill()
            p.join()
            bad.append(f"rank {r}: timed out")
        elif p.exitcode != 0:
            err = tmp_path / f"rank{r}.err"
            bad.append(f"rank {r}: exit {p.exitcode}\n" + (err.read_text() if err.exists() else ""))
    assert not bad, "\n".join(bad)
    A, perm, _, _, relax, maxsup, _ = _recipe(nx, pr, pc, reference)[:7]
    S = Symbolic(A, perm, relax, maxsup, reference=reference)
    lus = [S.distribute(pr, pc, k // pc, k % pc) for k in range(4)]
    o = pyoracle.oracle_factor(lus, pr, pc, A.n, False, cases.anorm(A))
    outs = [np.load(tmp_path / f"rank{r}.npz") for r in range(4)]
    errs = []
    for it in range(len(schedule)):
        worst = 0.0
        for z, lu in zip(outs, lus):
            for mine, ref in ((z[f"L{it}"], lu.Lval), (z[f"U{it}"], lu.Uval)):
                if len(ref):
                    worst = max(worst, float(np.abs(mine - ref).max() / max(np.abs(ref).max(), 1e-300)))
        errs.append(worst)
    assert all(e < TOL[0] for e in errs), errs
