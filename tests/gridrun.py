"""Multi-rank (2D process grid) runs of the engine for the tests.

``run_grid`` spawns Pr*Pc processes.  Each is one rank of the grid: it builds
its own LUstruct with the front-end, factors it with the MI355X engine and
returns its factors.  The ranks exchange panels either through RCCL (one GPU
per rank) or, where the box has fewer GPUs than ranks, through the engine's
host-staged test transport over torch.distributed gloo (RCCL refuses two ranks
on one GPU).  The CPU-only variant (``device=None``) exercises the same gloo
group plumbing without the engine.
"""
import os
import socket
import traceback

import numpy as np


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class GlooGrid:
    """torch.distributed gloo groups of a Pr x Pc grid (world / rows /
    columns), or of pz such layers (3D: global rank = layer * Pr * Pc + rank in
    the layer; group 3 = my (row, column) position in every layer)."""

    def __init__(self, rank, pr, pc, pz=1):
        import torch.distributed as dist
        self.dist = dist
        P = pr * pc
        self.rank, self.pr, self.pc, self.pz = rank, pr, pc, pz
        self.layer, r2 = rank // P, rank % P
        self.base = self.layer * P
        self.myrow, self.mycol = r2 // pc, r2 % pc
        self.row = self.col = None
        # test hook: SLU_TEST_DROP_SEND="r:k" makes global rank r skip its
        # k-th send (counted over the whole run) and every later send to the
        # same peer (sections pair in order: with only the one dropped, the
        # next message would land in its place) -- the receiver must then end
        # through the engine's exchange watchdog, not hang
        self.sends = []  # (peer global rank, bytes) of every send of this rank
        drop = os.environ.get("SLU_TEST_DROP_SEND")
        self.drop = int(drop.split(":")[1]) if drop and int(drop.split(":")[0]) == rank else -1
        self.dropped_peer = None
        if pz == 1:  # (the 3D runs use the point-to-point transport only)
            rows = [dist.new_group([r * pc + c for c in range(pc)]) for r in range(pr)]
            cols = [dist.new_group([r * pc + c for r in range(pr)]) for c in range(pc)]
            self.row, self.col = rows[self.myrow], cols[self.mycol]

    def global_root(self, group, root):
        if group == 0:
            return self.base + root
        if group == 1:
            return self.base + self.myrow * self.pc + root
        if group == 2:
            return self.base + root * self.pc + self.mycol
        return root * self.pr * self.pc + self.myrow * self.pc + self.mycol

    def bcast(self, group, root, arr):
        import torch
        t = torch.from_numpy(arr)
        g = None if group == 0 else (self.row if group == 1 else self.col)
        self.dist.broadcast(t, src=self.global_root(group, root), group=g)

    def p2p(self, ops):
        """One exchange phase of the point-to-point transport: post every
        send / receive (global ranks, one tag: pairs match in order, as
        ncclSend / ncclRecv inside a group), then wait for all of them."""
        import torch
        works = []
        for group, peer, send, arr in ops:
            t = torch.from_numpy(arr)
            other = self.global_root(group, peer)
            if other == self.rank:
                raise RuntimeError(f"p2p op with myself (group {group}, peer {peer})")
            if send:
                self.sends.append((other, arr.nbytes))
                if len(self.sends) - 1 == self.drop:
                    self.dropped_peer = other
                if other == self.dropped_peer:
                    continue
            works.append(self.dist.isend(t, other) if send else self.dist.irecv(t, other))
        for w in works:
            w.wait()


def _worker(rank, world, port, recipe, out_dir, device, fill=False, solve=False,
            transport="bcast", pz=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("SLU_WATCHDOG_S", "120")  # the library's watchdog is opt-in
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import cases
        from superlu_dist_amd.engine import Comm, Plan
        from superlu_dist_amd.frontend import Symbolic
        if isinstance(recipe, str):  # "refdump:<case>": the reference's own LUstruct
            from refdump import Fixture
            fx = Fixture(recipe.split(":", 1)[1])
            pr, pc, tiny, anorm = fx.pr, fx.pc, fx.replace_tiny, fx.anorm
            gg = GlooGrid(rank, pr, pc, pz)
            lu = fx.lu(rank % (pr * pc))
            A = S = None
        else:
            rc = recipe()
            A, perm, dtype, (pr, pc), relax, maxsup, tiny = rc[:7]
            reference = len(rc) > 7 and rc[7]  # the structure pdgssvx builds (symbfact + pddistribute)
            anorm = cases.anorm(A)
            gg = GlooGrid(rank, pr, pc, pz)
            S = Symbolic(A, perm, relax, maxsup, reference=reference)
            lu = S.distribute(pr, pc, gg.myrow, gg.mycol)
        res = {}
        if pz > 1:  # 3D grid: every layer holds the LUstruct; p2p transport
            comm = Comm.host_p2p3d(pr, pc, pz, rank, -1 if device is None else device, gg.p2p)
            assert comm.size(3) == pz and comm.size(0) == pr * pc
            if transport == "schedule":
                p = Plan(lu, comm=comm, schedule_only=True)
                res["nsec"], res["nbytes"] = p.check_exchange()
                res["nlevels"] = p.stats()["nlevels"]
                res["nsupers"] = p.stats()["nsupers"]
            else:
                p = Plan(lu, comm=comm, replace_tiny=tiny)
                p.upload()
                info, ntiny = p.factor(anorm)
                st = p.stats()
                res.update(info=info, tiny=ntiny, flops=st["schur_flops"] + st["panel_flops"],
                           comm_bytes=st["comm_bytes"], nsupers=st["nsupers"])
                p.gather3d()
                p.download()
            del p
        elif transport == "schedule":  # no GPU: the exchange schedule over the p2p transport
            comm = Comm.host_p2p(pr, pc, rank, -1, gg.p2p)
            p = Plan(lu, comm=comm, schedule_only=True)
            res["nsec"], res["nbytes"] = p.check_exchange()
            res["sends"] = np.array(gg.sends, dtype=np.int64).reshape(-1, 2)
            st = p.stats()
            res["nlevels"] = st["nlevels"]
            res["nsupers"], res["nsupers_in"] = st["nsupers"], st["nsupers_in"]
            res["flops"] = st["schur_flops"] + st["panel_flops"]
            del p
        elif device is not None:
            if transport == "p2p":
                comm = Comm.host_p2p(pr, pc, rank, device, gg.p2p)
            else:
                comm = Comm.host(pr, pc, rank, device, gg.bcast)
            assert comm.size(0) == pr * pc and comm.size(1) == pc and comm.size(2) == pr
            p = Plan(lu, comm=comm, replace_tiny=tiny)
            if fill and A is not None:  # values from A on the device (no LU upload), SamePattern refill
                cp, ri, v = A.permuted(S.perm_c).arrays()
                p.set_a_pattern(cp, ri)
                p.fill_a(v)
            elif solve:  # the fixture's A in the LUstruct's coordinates, filled on the device
                from lusolve import lu_coords_matrix_from_lus
                cp, ri, v = lu_coords_matrix_from_lus(fx.lus("pre"), pr, pc)
                p.set_a_pattern(cp, ri)
                p.fill_a(v)
            else:
                p.upload()
            info, ntiny = p.factor(anorm)
            if solve:  # the 2D-grid device solve and refinement of the fixture's right-hand side
                from lusolve import from_lu_coords, to_lu_coords
                b, R, C, perm_r, perm_c, _, _ = fx.full_rhs()
                bl = to_lu_coords(b, perm_r, perm_c, R).astype(lu.Lval.dtype)
                y = p.solve(bl)
                res["x"] = from_lu_coords(y, perm_c, C)
                res["t_solve_ms"] = p.stats()["t_solve_ms"]
                yr, berr, steps = p.refine(bl, y)
                res["xr"] = from_lu_coords(yr, perm_c, C)
                res["berr"], res["steps"] = float(berr[0]), int(steps[0])
            p.download()
            st = p.stats()
            res.update(info=info, tiny=ntiny, flops=st["schur_flops"] + st["panel_flops"],
                       comm_bytes=st["comm_bytes"], nsupers=st["nsupers"], nsupers_in=st["nsupers_in"])
            del p
        else:  # group plumbing only
            buf = np.full(16, rank, dtype=np.uint8)
            gg.bcast(1, 0, buf)
            res["row_root"] = int(buf[0])
            buf = np.full(16, rank, dtype=np.uint8)
            gg.bcast(2, pr - 1, buf)
            res["col_root"] = int(buf[0])
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), L=lu.Lval, U=lu.Uval,
                 **{k: np.asarray(v) for k, v in res.items()})
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        with open(os.path.join(out_dir, f"rank{rank}.err"), "w") as fh:
            fh.write(traceback.format_exc())
        raise


def run_grid(recipe, pr, pc, out_dir, device=0, timeout=240, fill=False, solve=False,
             transport="bcast", pz=1):
    """Run ``recipe`` (picklable callable returning cases.build()-style
    tuples, or "refdump:<case>" for the per-rank LUstructs of a reference
    dump fixture) on a pr x pc grid; returns the per-rank result dicts.
    transport: "bcast" (host-staged broadcasts, the drop-in's MPI path when
    ranks share a GPU) or "p2p" (the RCCL transport's send / receive pairs,
    host-staged over gloo isend / irecv).

    The parent never imports torch: torch bundles its own ROCm runtime, and a
    process that loads libslu_mi355x.so (system ROCm) before torch ends up
    with two HIP runtimes.  Each worker imports torch.distributed first."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    world = pr * pc * pz
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, recipe, str(out_dir), device, fill,
                                                solve, transport, pz))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    bad = []
    for r, p in enumerate(procs):
        if p.is_alive():
            p.kill()
            p.join()
            bad.append(f"rank {r}: timed out")
        elif p.exitcode != 0:
            err = os.path.join(out_dir, f"rank{r}.err")
            msg = open(err).read() if os.path.exists(err) else ""
            bad.append(f"rank {r}: exit {p.exitcode}\n{msg}")
    if bad:
        raise RuntimeError("grid run failed:\n" + "\n".join(bad))
    out = []
    for r in range(world):
        z = np.load(os.path.join(out_dir, f"rank{r}.npz"))
        out.append({k: z[k] for k in z.files})
    return out
