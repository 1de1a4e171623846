"""Write a seeded 3D 7-point stencil as a Harwell-Boeing RUA file (the format
the reference's EXAMPLE drivers read with dreadhb), for the drop-in tests of
pdgstrf3d: a matrix whose elimination tree splits into balanced subtrees.

    python tools/gen_rua.py NX OUT.rua

A = 7-point Laplacian (diag 6, off-diagonal -1) with a small seeded
unsymmetric perturbation of the off-diagonals (so MC64 / equilibration have
work and L != U^T)."""
import sys

import numpy as np


def stencil(nx):
    n = nx ** 3
    rng = np.random.default_rng(12345)
    cols = []
    for z in range(nx):
        for y in range(nx):
            for x in range(nx):
                j = x + nx * (y + nx * z)
                ent = [(j, 6.0)]
                for dx, dy, dz in ((-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)):
                    a, b, c = x + dx, y + dy, z + dz
                    if 0 <= a < nx and 0 <= b < nx and 0 <= c < nx:
                        ent.append((a + nx * (b + nx * c), -1.0 + 0.1 * rng.standard_normal()))
                ent.sort()
                cols.append(ent)
    colptr = np.cumsum([0] + [len(c) for c in cols])
    rows = np.array([r for c in cols for r, _ in c])
    vals = np.array([v for c in cols for _, v in c])
    return n, colptr, rows, vals


def fmt_int(a, per=16, w=5):
    return ["".join(f"{int(v):{w}d}" for v in a[i:i + per]) for i in range(0, len(a), per)]


def fmt_real(a, per=5):
    return ["".join(f"{v:15.8E}" for v in a[i:i + per]) for i in range(0, len(a), per)]


def main(nx, out):
    n, colptr, rows, vals = stencil(nx)
    w = max(5, len(str(len(rows) + 1)) + 1)
    per = 80 // w
    ptr = fmt_int(colptr + 1, per, w)
    ind = fmt_int(rows + 1, per, w)
    val = fmt_real(vals)
    title = f"lap3d_{nx} 7-point stencil, seeded unsymmetric perturbation"
    with open(out, "w") as f:
        f.write(f"{title:<72}{'LAP3D':<8}\n")
        f.write(f"{len(ptr) + len(ind) + len(val):14d}{len(ptr):14d}{len(ind):14d}{len(val):14d}{0:14d}\n")
        f.write(f"{'RUA':<14}{n:14d}{n:14d}{len(rows):14d}{0:14d}\n")
        f.write(f"{f'({per}I{w})':<16}{f'({per}I{w})':<16}{'(5E15.8)':<20}{'(5E15.8)':<20}\n")
        for block in (ptr, ind, val):
            for line in block:
                f.write(line + "\n")


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2])
