"""Generates tests/golden/symb_<case>.npz: the REFERENCE's sp_colorder and
symbfact outputs (perm_c after the etree postorder, etree, A Pc' column
pointers, xsup, supno, xlsub, lsub, xusub, usub, symbfact's return value and
nnzLU) on fixed patterns, dumped by oracle/_ref/symb_dump
(gen/symb_dump_main.c), which runs them as pdgssvx does
(SRC/pdgssvx.c:1029-1076).  TEST INFRASTRUCTURE.

Run here (needs /root/reference; `make -C oracle _ref/symb_dump`):
    python oracle/gen/make_symb_golden.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
DUMP = os.path.join(REPO, "oracle", "_ref", "symb_dump")
sys.path.insert(0, REPO)

NATURAL, MMD_ATA, MMD_AT_PLUS_A, MY_PERMC = 0, 1, 2, 7


def stencil3d(k):
    n = k ** 3
    cols = [[] for _ in range(n)]
    for i in range(k):
        for j in range(k):
            for l in range(k):
                c = (i * k + j) * k + l
                for di, dj, dl in ((0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0),
                                   (0, 0, -1), (0, 0, 1)):
                    a, b, d = i + di, j + dj, l + dl
                    if 0 <= a < k and 0 <= b < k and 0 <= d < k:
                        cols[c].append((a * k + b) * k + d)
    return n, cols


def random_unsym(n, per_col, seed):
    """Structurally unsymmetric pattern with a full diagonal; rows in each
    column in a random order (the search order follows it)."""
    rng = np.random.default_rng(seed)
    cols = []
    for c in range(n):
        rows = set(rng.integers(0, n, per_col).tolist()) | {c}
        # a few long-range couplings, mostly below the diagonal
        r = list(rows)
        rng.shuffle(r)
        cols.append(r)
    return n, cols


def upwind2d(k):
    """2D grid, 5-point diffusion plus one-sided (west, south) upwind
    couplings two cells away: unsymmetric structure."""
    n = k * k
    cols = [[] for _ in range(n)]
    for i in range(k):
        for j in range(k):
            r = i * k + j
            ent = [r]
            if j > 0: ent.append(r - 1)
            if j < k - 1: ent.append(r + 1)
            if i > 0: ent.append(r - k)
            if i < k - 1: ent.append(r + k)
            if j > 1: ent.append(r - 2)
            if i > 1: ent.append(r - 2 * k)
            for c in ent:            # row r has entries in columns ent
                cols[c].append(r)
    return n, cols


def hb(name):
    from superlu_dist_amd.hbio import read_hb
    n, colptr, rowind, _, _ = read_hb(os.path.join(GOLDEN, "matrices", name))
    colptr = np.asarray(colptr, np.int64)
    rowind = np.asarray(rowind, np.int64)
    if colptr[0] == 1:
        colptr = colptr - 1
        rowind = rowind - 1
    return n, [rowind[colptr[c]:colptr[c + 1]].tolist() for c in range(n)]


CASES = {
    # name: (pattern, colperm, relax, maxsup)
    "g20_mmd": (lambda: hb("g20.rua"), MMD_AT_PLUS_A, 60, 256),
    "g20_r4s10": (lambda: hb("g20.rua"), MMD_AT_PLUS_A, 4, 10),
    "big_mmd": (lambda: hb("big.rua"), MMD_AT_PLUS_A, 60, 256),
    "big_r8s20": (lambda: hb("big.rua"), MMD_AT_PLUS_A, 8, 20),
    "lap3d12_mmd": (lambda: stencil3d(12), MMD_AT_PLUS_A, 60, 256),
    "lap3d12_nat": (lambda: stencil3d(12), NATURAL, 4, 20),
    "upwind30_mmd": (lambda: upwind2d(30), MMD_AT_PLUS_A, 16, 64),
    "upwind30_ata": (lambda: upwind2d(30), MMD_ATA, 16, 64),
    "rand2000_mmd": (lambda: random_unsym(2000, 3, 11), MMD_AT_PLUS_A, 10, 32),
    "rand2000_ata": (lambda: random_unsym(2000, 3, 12), MMD_ATA, 1, 512),
}


def write_input(path, n, cols, perm_c=None):
    colptr = np.zeros(n + 1, np.int64)
    colptr[1:] = np.cumsum([len(c) for c in cols])
    rowind = np.asarray([r for c in cols for r in c], np.int64)
    with open(path, "wb") as fh:
        np.asarray([n, n, len(rowind)], np.int64).tofile(fh)
        colptr.tofile(fh)
        rowind.tofile(fh)
        if perm_c is not None:
            np.asarray(perm_c, np.int64).tofile(fh)


def read_dump(path):
    out = {}
    with open(path, "rb") as fh:
        while True:
            nm = fh.read(16)
            if not nm:
                break
            cnt = int(np.frombuffer(fh.read(8), np.int64)[0])
            out[nm.rstrip(b"\0").decode()] = np.frombuffer(fh.read(8 * cnt), np.int64).copy()
    return out


def run(name, n, cols, colperm, relax, maxsup, perm_c=None):
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        write_input(fin, n, cols, perm_c)
        r = subprocess.run([DUMP, fin, fout, str(colperm), str(relax), str(maxsup)],
                           capture_output=True, text=True, check=True)
        d = read_dump(fout)
    t = [float(x) for x in r.stdout.split()[-3:]]
    return d, t


def main(names):
    for name in names or CASES:
        pat, colperm, relax, maxsup = CASES[name]
        n, cols = pat()
        d, t = run(name, n, cols, colperm, relax, maxsup)
        d["meta"] = np.asarray([n, colperm, relax, maxsup], np.int64)
        np.savez_compressed(os.path.join(GOLDEN, f"symb_{name}.npz"), **d)
        print(f"{name}: n {n} nsupers {d['supno'][n] + 1} lsub {len(d['lsub'])} "
              f"usub {len(d['usub'])} ret {d['scalars'][0]} times {t}")


if __name__ == "__main__":
    main(sys.argv[1:])
