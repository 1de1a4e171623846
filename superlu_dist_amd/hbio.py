"""Harwell-Boeing (.rua / .cua) reader -- the input format of the reference's
EXAMPLE/pddrive (SRC/dreadhb.c, SRC/zreadhb.c).  Pure Python, fixed-width
Fortran fields; returns 0-based CSC arrays."""
import re

import numpy as np


def _fmt(s):
    m = re.search(r"\((\d*)[A-Za-z](\d+)", s)
    per = int(m.group(1)) if m.group(1) else 1
    return per, int(m.group(2))


def _read_fields(lines, count, per, width, conv):
    out = []
    for line in lines:
        line = line.rstrip("\n")
        for k in range(per):
            if len(out) == count:
                break
            f = line[k * width:(k + 1) * width]
            if not f.strip():
                continue
            out.append(conv(f))
        if len(out) == count:
            break
    return out


def read_hb(path):
    """Returns (n, colptr, rowind, values, is_complex)."""
    with open(path) as fh:
        lines = fh.readlines()
    totcrd, ptrcrd, indcrd, valcrd, rhscrd = (int(x) for x in lines[1].split()[:5])
    h3 = lines[2]
    mxtype = h3[:3].upper()
    nrow, ncol, nnz = (int(x) for x in h3[3:].split()[:3])
    ptrfmt, indfmt, valfmt = lines[3][:16], lines[3][16:32], lines[3][32:52]
    start = 4 + (1 if rhscrd > 0 else 0)
    p_per, p_w = _fmt(ptrfmt)
    i_per, i_w = _fmt(indfmt)
    v_per, v_w = _fmt(valfmt)
    cur = start
    colptr = _read_fields(lines[cur:cur + ptrcrd], ncol + 1, p_per, p_w, int)
    cur += ptrcrd
    rowind = _read_fields(lines[cur:cur + indcrd], nnz, i_per, i_w, int)
    cur += indcrd
    cplx = mxtype[0] == "C"
    nval = nnz * (2 if cplx else 1)
    conv = lambda f: float(f.replace("D", "E").replace("d", "e"))
    vals = _read_fields(lines[cur:cur + valcrd], nval, v_per, v_w, conv)
    colptr = np.array(colptr, dtype=np.int64) - 1
    rowind = np.array(rowind, dtype=np.int64) - 1
    v = np.array(vals, dtype=np.float64)
    if cplx:
        v = v[0::2] + 1j * v[1::2]
    assert nrow == ncol, "square matrices only"
    return ncol, colptr, rowind, v, cplx
