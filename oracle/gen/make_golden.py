"""Generates tests/golden/ref_<case>.npz: the factors computed by the
REFERENCE pdgstrf / psgstrf / pzgstrf (oracle/_ref/ref_pdgstrf, compiled from
/root/reference/SRC) on the LUstructs of tests/cases.py.

Run here (needs /root/reference, conda MPICH and MKL):
    python oracle/gen/make_golden.py [case ...]
Each fixture stores the per-rank Lnzval/Unzval arrays after factorization,
the reference's info / TinyPivots / ops, the anorm passed, and a digest of the
pre-factor index arrays.  TEST INFRASTRUCTURE.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import cases  # noqa: E402
import pyoracle  # noqa: E402


def make(name):
    A, S, lus = cases.distribute(name)
    _, perm, dtype, (pr, pc), relax, maxsup, tiny = cases.build(name)
    an = cases.anorm(A)
    stats, facs = pyoracle.run_reference(A, perm, pr, pc, relax=relax, maxsup=maxsup,
                                         lookahead=10, replace_tiny=tiny)
    meta = {"case": name, "grid": [pr, pc], "relax": relax, "maxsup": maxsup,
            "replace_tiny": tiny, "dtype": dtype, "ref_info": stats["info"],
            "ref_tiny": stats["tiny"], "ref_ops": stats["ops"], "anorm": stats["anorm"],
            "nsupers": int(S.nsupers), "digest": cases.structure_digest(lus),
            "generator": "oracle/gen/make_golden.py via oracle/_ref/ref_pdgstrf"}
    arrs = {}
    for p, (Lv, Uv) in enumerate(facs):
        arrs[f"L{p}"] = Lv
        arrs[f"U{p}"] = Uv
    out = os.path.join(cases.GOLDEN, f"ref_{name}.npz")
    np.savez_compressed(out, meta=json.dumps(meta), **arrs)
    print(f"{name}: info={stats['info']} tiny={stats['tiny']} ops={stats['ops']:.4e} -> {out}")


if __name__ == "__main__":
    names = sys.argv[1:] or list(cases.CASES)
    for nm in names:
        make(nm)
