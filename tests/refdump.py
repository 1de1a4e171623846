"""Loader for tests/golden/refdump_*.npz: LUstructs built by the REFERENCE's own
front-end (p?gssvx: equilibration, MC64, MMD, symbfact, pddistribute), the
reference's factors of them, and its solve / refinement results
(oracle/gen/make_refdump.py, oracle/gen/ref_dump_main.c)."""
import glob
import json
import os

import numpy as np

from superlu_dist_amd.frontend import LUStruct
from superlu_dist_amd.lib import DTYPE_CODE

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(f)[8:-4] for f in glob.glob(os.path.join(GOLDEN, "refdump_*.npz")))


class Fixture:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, f"refdump_{name}.npz"), allow_pickle=False)
        self.meta = json.loads(str(z["meta"]))
        self.z = {k: z[k] for k in z.files if k != "meta"}
        self.pr, self.pc = self.meta["grid"]
        self.dtype = DTYPE_CODE[self.meta["dtype"]]
        r0 = self.meta["ranks"][0]
        self.n = r0["n"]
        self.anorm = r0["anorm"]
        self.info = r0["info"]                       # after the MIN over ranks
        self.tiny = sum(r["tiny"] for r in self.meta["ranks"])
        self.replace_tiny = bool(r0["replace_tiny"])
        self.nsupers = r0["nsupers"]

    @property
    def nranks(self):
        return self.pr * self.pc

    def arr(self, rank, key):
        return self.z[f"r{rank}_{key}"]

    def lu(self, rank, tag="pre"):
        """The rank's LUstruct as the reference's pddistribute left it
        (tag "pre") or as the reference's pdgstrf left it ("post")."""
        a = lambda k: self.arr(rank, k)  # noqa: E731
        return LUStruct.from_arrays(self.dtype, self.n, self.arr(0, "xsup"), self.arr(0, "supno"),
                                    self.pr, self.pc, rank // self.pc, rank % self.pc,
                                    a("Lidx"), a("Loff"), a(f"{tag}_Lval"), a("Lvoff"),
                                    a("Uidx"), a("Uoff"), a(f"{tag}_Uval"), a("Uvoff"),
                                    a("ToRecv"), a("ToSendD"), a("ToSendR"), a("bufmax"))

    def lus(self, tag="pre"):
        return [self.lu(p, tag) for p in range(self.nranks)]

    def full_rhs(self):
        """b, R, C, perm_r, perm_c, x_norefine, xtrue as full vectors: the
        reference's distributed B / X (NRformat_loc rows fst_row .. fst_row +
        m_loc of each rank) put back together."""
        order = sorted(range(self.nranks), key=lambda p: self.meta["ranks"][p]["fst_row"])
        cat = lambda k: np.concatenate([self.arr(p, k) for p in order])  # noqa: E731
        return (cat("b"), self.z.get("r0_R"), self.z.get("r0_C"), self.arr(0, "perm_r"),
                self.arr(0, "perm_c"), cat("x_norefine"), cat("xtrue"))

    def ref_factors(self):
        return [(self.arr(p, "post_Lval"), self.arr(p, "post_Uval")) for p in range(self.nranks)]
