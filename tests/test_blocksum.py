"""The full-size parity checker of bench.py (oracle/blocksum.h): per-block
fingerprints of two factorizations, keyed by global block, compared across
process grids.  CPU: the oracle's factors of the reference-structure LUstruct
(the reference's own sp_colorder + symbfact + pddistribute, restated
bit-exact) on 1x1 against the reference pdgstrf's on 2x2 (oracle/_ref), and
the checker must see a perturbation of one value and a different structure."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order  # noqa: E402

needs_ref = pytest.mark.skipif(not pyoracle.have_reference_harness(),
                               reason="reference harness (oracle/_ref) not built")


def _problem(nx=10):
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    return A, nd_order(nx, nx, nx)


def test_blocksums_grid_independent():
    """The same factors distributed on 1x1 and on 2x2 give the same records."""
    A, p = _problem(8)
    S = Symbolic(A, p, 60, 256, reference=True)
    one = S.distribute(1, 1, 0, 0)
    pyoracle.oracle_factor([one], 1, 1, A.n, False, 12.0)
    lus = [S.distribute(2, 2, r // 2, r % 2) for r in range(4)]
    pyoracle.oracle_factor(lus, 2, 2, A.n, False, 12.0)
    grid = np.concatenate([pyoracle.blocksums(lu) for lu in lus])
    c = pyoracle.compare_blocksums(pyoracle.blocksums(one), grid)
    assert c["match"] and c["values"] == len(one.Lval) - 1 + len(one.Uval) - 1
    assert c["rel_err"] <= 1e-13


@needs_ref
def test_reference_structure_factors_match_reference_pdgstrf():
    A, p = _problem(10)
    S = Symbolic(A, p, 60, 256, reference=True)
    lu = S.distribute(1, 1, 0, 0)
    pyoracle.oracle_factor([lu], 1, 1, A.n, False, 12.0)
    mine = pyoracle.blocksums(lu)
    st, _ = pyoracle.run_reference(A, p, 2, 2, symb_flags=2, want_factors=False,
                                   want_blocksums=True, timeout=300)
    c = pyoracle.compare_blocksums(mine, st["blocksums"])
    assert c["match"], c
    assert c["rel_err"] <= 1e-12, c
    # one value off by 1e-8 (relative) is seen
    k = int(np.argmax(np.abs(lu.Lval[:-1])))
    lu.Lval[k] *= 1 + 1e-8
    assert pyoracle.compare_blocksums(pyoracle.blocksums(lu), st["blocksums"])["rel_err"] > 1e-12
    # and the library front-end's (amalgamated) structure is a different LUstruct
    st2, _ = pyoracle.run_reference(A, p, 1, 1, symb_flags=0, want_factors=False,
                                    want_blocksums=True, timeout=300)
    assert not pyoracle.compare_blocksums(mine, st2["blocksums"])["match"]
