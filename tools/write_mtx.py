"""Writes the bench's 3D 7-point Laplacian as a Matrix Market file for the
reference's EXAMPLE/pddrive (dcreate_matrix_postfix "mtx" branch,
EXAMPLE/dcreate_matrix.c:107) -- the CPU baseline with the reference's own
front-end and MMD_AT_PLUS_A ordering.

usage: python tools/write_mtx.py NX OUT.mtx
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superlu_dist_amd.frontend import STENCIL_3D7, Csc  # noqa: E402


def main():
    nx, out = int(sys.argv[1]), sys.argv[2]
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    colptr, rowind, val = A.arrays()
    cols = np.repeat(np.arange(A.n, dtype=np.int64), np.diff(colptr))
    with open(out, "w") as fh:
        fh.write("%%MatrixMarket matrix coordinate real general\n")
        fh.write(f"{A.n} {A.n} {len(rowind)}\n")
        blk = 1 << 20
        for s in range(0, len(rowind), blk):
            e = min(len(rowind), s + blk)
            np.savetxt(fh, np.column_stack([rowind[s:e] + 1, cols[s:e] + 1, val[s:e]]),
                       fmt="%d %d %.17g")
    print(f"wrote {out}: n={A.n} nnz={len(rowind)}")


if __name__ == "__main__":
    main()
