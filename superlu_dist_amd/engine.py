"""Python driver of the MI355X engine (csrc/engine.hip) through its C ABI.

A ``Plan`` is built once per LU structure: it copies the factor storage of a
host LUstruct into HBM, levels the supernodal dependency DAG and uploads every
index table the kernels need.  ``factor()`` then runs the numeric
factorization entirely on the device; ``download()`` writes the factors back
into the host LUstruct (the in-place contract of SRC/pdgstrf.c).
"""
import ctypes as C

import numpy as np

from .lib import HOST_BCAST_FN, HOST_P2P_FN, EngineOpts, PlanStats, as_i64p, lib

SMACH_EPS = 5.9604644775390625e-08  # smach_dist("Epsilon"), SRC/smach_dist.c:64


class Comm:
    """RCCL communicators of one 2D grid (one rank per GPU)."""

    def __init__(self, nprow, npcol, iam, device=0, uid=None):
        self.nprow, self.npcol, self.iam = nprow, npcol, iam
        buf = None
        if nprow * npcol > 1:
            if uid is None:
                raise ValueError("multi-rank grids need the RCCL unique id")
            buf = C.create_string_buffer(bytes(uid), 128)
        self.ptr = lib().slu_comm_create(buf, nprow, npcol, iam, device)
        if not self.ptr:
            raise RuntimeError(lib().slu_last_error().decode())

    @classmethod
    def host(cls, nprow, npcol, iam, device, bcast):
        """Test transport: ``bcast(group, root, buf)`` broadcasts the uint8
        numpy array ``buf`` in place within group 0 (grid), 1 (my process
        row) or 2 (my process column) from the group-local rank ``root``.
        For several ranks on one GPU (RCCL refuses duplicate devices); the
        device kernels are the same as with RCCL."""
        self = cls.__new__(cls)
        self.nprow, self.npcol, self.iam = nprow, npcol, iam

        def _cb(_ctx, group, root, buf, nbytes):
            try:
                arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(buf))
                bcast(group, root, arr)
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the C status
                import sys
                print(f"host broadcast failed: {e!r}", file=sys.stderr)
                return 1

        self._cb = HOST_BCAST_FN(_cb)  # keep alive as long as the comm
        self.ptr = lib().slu_comm_create_host(self._cb, None, nprow, npcol, iam, device)
        if not self.ptr:
            raise RuntimeError(lib().slu_last_error().decode())
        return self

    @classmethod
    def host_p2p(cls, nprow, npcol, iam, device, p2p, _npdep=1, _iam3d=None):
        """Point-to-point test transport: ``p2p(ops)`` receives the list of
        (group, peer, is_send, uint8 numpy buffer) of one exchange phase --
        exactly the ncclSend / ncclRecv pairs the RCCL transport issues, in
        its order -- and must post them all before waiting for any."""
        self = cls.__new__(cls)
        self.nprow, self.npcol, self.iam = nprow, npcol, iam

        def _cb(_ctx, nops, ops):
            try:
                lst = []
                for i in range(nops):
                    o = ops[i]
                    arr = np.ctypeslib.as_array((C.c_uint8 * o.bytes).from_address(o.buf))
                    lst.append((o.group, o.peer, bool(o.send), arr))
                p2p(lst)
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the C status
                import sys
                print(f"host p2p group failed: {e!r}", file=sys.stderr)
                return 1

        self._cb = HOST_P2P_FN(_cb)
        if _npdep > 1:
            self.ptr = lib().slu_comm_create_host_p2p3d(self._cb, None, nprow, npcol, _npdep,
                                                        _iam3d, device)
        else:
            self.ptr = lib().slu_comm_create_host_p2p(self._cb, None, nprow, npcol, iam, device)
        if not self.ptr:
            raise RuntimeError(lib().slu_last_error().decode())
        return self

    @classmethod
    def grid3d(cls, nprow, npcol, npdep, iam3d, device=0, uid=None):
        """RCCL communicators of a 3D grid (npdep layers of nprow x npcol;
        iam3d = layer * nprow * npcol + row * npcol + column)."""
        self = cls.__new__(cls)
        self.nprow, self.npcol, self.npdep = nprow, npcol, npdep
        self.iam = iam3d % (nprow * npcol)
        buf = None
        if nprow * npcol * npdep > 1:
            if uid is None:
                raise ValueError("multi-rank grids need the RCCL unique id")
            buf = C.create_string_buffer(bytes(uid), 128)
        self.ptr = lib().slu_comm_create3d(buf, nprow, npcol, npdep, iam3d, device)
        if not self.ptr:
            raise RuntimeError(lib().slu_last_error().decode())
        return self

    @classmethod
    def host_p2p3d(cls, nprow, npcol, npdep, iam3d, device, p2p):
        """host_p2p for a 3D grid: group 3 = the ranks at my (row, column)
        of every layer, peer = layer."""
        self = cls.host_p2p(nprow, npcol, iam3d % (nprow * npcol), device, p2p, _npdep=npdep,
                            _iam3d=iam3d)
        self.npdep = npdep
        return self

    def size(self, group=0):
        """Ranks in the grid (0), my process row (1) or column (2), the
        layers of a 3D grid (3); for RCCL what ncclCommCount reports."""
        return lib().slu_comm_size(self.ptr, group)

    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(128)
        if lib().slu_comm_unique_id(buf) != 0:
            raise RuntimeError(lib().slu_last_error().decode())
        return buf.raw

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().slu_comm_destroy(self.ptr)
            self.ptr = None


class Plan:
    def __init__(self, lu, comm=None, replace_tiny=False, timing=False, overlap_upload=False,
                 overlap_download=False, schedule_only=False):
        """overlap_upload: the H2D copy of the values starts inside the
        constructor, beside the plan build (upload() waits for it);
        overlap_download: factor() writes each finished level back into the
        host LUstruct while later levels run (download() is then a no-op);
        schedule_only: host-only plan (no GPU needed) whose exchange schedule
        check_exchange() replays through the communicator."""
        self.lu = lu
        o = EngineOpts()
        o.replace_tiny_pivot = int(bool(replace_tiny))
        o.timing = int(timing)
        o.overlap_upload = int(bool(overlap_upload))
        o.overlap_download = int(bool(overlap_download))
        o.schedule_only = int(bool(schedule_only))
        err = C.create_string_buffer(1024)
        iam = lu.myrow * lu.npcol + lu.mycol
        self.comm = comm
        self.ptr = lib().slu_plan_create(lu.dtype, lu.ptr, lu.n, lu.nprow, lu.npcol, iam,
                                         comm.ptr if comm is not None else None, C.byref(o),
                                         err, len(err))
        if not self.ptr:
            raise RuntimeError("slu_plan_create: " + err.value.decode())

    def _chk(self, rc):
        if rc != 0:
            raise RuntimeError(lib().slu_last_error().decode())

    def upload(self):
        self._chk(lib().slu_plan_upload(self.ptr))

    def factor(self, anorm=1.0):
        info, tiny = C.c_int(), C.c_int()
        self._chk(lib().slu_plan_factor(self.ptr, anorm, C.byref(info), C.byref(tiny)))
        return info.value, tiny.value

    def snapshot(self):
        """Keep a pristine device copy of the uploaded values."""
        self._chk(lib().slu_plan_snapshot(self.ptr))

    def restore(self):
        """Restore the working factor storage from the snapshot (device to device)."""
        self._chk(lib().slu_plan_restore(self.ptr))

    def set_timing(self, timing, serial=False):
        """timing: 0 off, 1 phase events, 2 + per-level log; serial: run every
        launch on one stream (no look-ahead overlap) so kernel durations are
        not inflated by concurrent kernels."""
        self._chk(lib().slu_plan_set_timing(self.ptr, int(timing), int(bool(serial))))

    def sync(self):
        self._chk(lib().slu_plan_sync(self.ptr))

    def download(self):
        self._chk(lib().slu_plan_download(self.ptr))

    def solve(self, b):
        """Solve L U x = b with the device-resident factors (the LUstruct's
        permuted coordinates); b: (n,) or (n, nrhs).  Returns x.  On a 2D grid
        every rank calls it with the same b and receives the whole x."""
        dt = self.lu.Lval.dtype
        x = np.array(b, dtype=dt, order="F", copy=True)
        nrhs = 1 if x.ndim == 1 else x.shape[1]
        n = x.shape[0]
        self._chk(lib().slu_plan_solve(self.ptr, x.ctypes.data_as(C.c_void_p), n, nrhs))
        return x

    def set_a_pattern(self, colptr, rowind):
        """Pattern of A in the LUstruct's permuted coordinates (CSC)."""
        self._xa = np.ascontiguousarray(colptr, dtype=np.int64)
        self._asub = np.ascontiguousarray(rowind, dtype=np.int64)
        self._chk(lib().slu_plan_set_a_pattern(self.ptr, len(self._xa) - 1,
                                               as_i64p(self._xa), as_i64p(self._asub)))

    def fill_a(self, values):
        """Refill the device factor storage from A's values (host array in the
        order of the pattern), SamePattern_SameRowPerm; no LU upload."""
        v = np.ascontiguousarray(values, dtype=self.lu.Lval.dtype)
        if len(v) != len(self._asub):
            raise ValueError(f"{len(v)} values for a pattern of {len(self._asub)} nonzeros")
        self._chk(lib().slu_plan_fill_a(self.ptr, v.ctypes.data_as(C.c_void_p), 0))

    def refine(self, b, x):
        """Iterative refinement of x for A x = b on the device (pdgsrfs), A =
        the values of the last fill_a; returns (x, berr, steps) per column."""
        dt = self.lu.Lval.dtype
        bb = np.array(b, dtype=dt, order="F", copy=True)
        xx = np.array(x, dtype=dt, order="F", copy=True)
        if bb.shape != xx.shape:
            raise ValueError("b and x differ in shape")
        nrhs = 1 if bb.ndim == 1 else bb.shape[1]
        berr = np.zeros(max(nrhs, 1))
        steps = np.zeros(max(nrhs, 1), dtype=np.int32)
        self._chk(lib().slu_plan_refine(self.ptr, bb.ctypes.data_as(C.c_void_p),
                                        xx.ctypes.data_as(C.c_void_p), bb.shape[0], nrhs,
                                        berr.ctypes.data_as(C.POINTER(C.c_double)),
                                        steps.ctypes.data_as(C.POINTER(C.c_int))))
        return xx, berr[:nrhs], steps[:nrhs]

    def check_exchange(self):
        """Schedule-only plans: replay every level's exchange phases of
        factor() through the communicator, each received section checked
        byte for byte (collective).  Returns (sections, bytes) received."""
        ns, nb = C.c_int64(), C.c_int64()
        self._chk(lib().slu_plan_check_exchange(self.ptr, C.byref(ns), C.byref(nb)))
        return ns.value, nb.value

    def gather3d(self):
        """3D plans (collective over the layers): bring the factored forests
        to layer 0, whose ranks then hold the final factors (download())."""
        self._chk(lib().slu_plan_gather3d(self.ptr))

    def stats(self):
        st = PlanStats()
        lib().slu_plan_get_stats(self.ptr, C.byref(st))
        return st.as_dict()

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().slu_plan_destroy(self.ptr)
            self.ptr = None


def factor_lustruct(lu, anorm=1.0, comm=None, replace_tiny=False):
    """Factor one rank's LUstruct in place on the GPU; returns (info, tiny, stats)."""
    p = Plan(lu, comm=comm, replace_tiny=replace_tiny)
    p.upload()
    info, tiny = p.factor(anorm)
    p.download()
    return info, tiny, p.stats()
