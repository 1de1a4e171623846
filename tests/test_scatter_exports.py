"""The host scatter helpers libslu_mi355x.so exports because the reference's
pdgstrf.c.o defines them (SRC/pdgstrf.c:171 includes SRC/dscatter.c; the 3D
code still calls them): [dsz]scatter_l_1, [dsz]scatter_l and
[dsz]scatter_u must do exactly what the reference's do.  CPU only: both
libraries are called on the same random blocks (the reference's compiled
into oracle/_ref/libref_factor.so from /root/reference/SRC) and the
destinations must agree bit for bit."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT

REFLIB = os.path.join(ROOT, "oracle", "_ref", "libref_factor.so")
pytestmark = pytest.mark.skipif(not os.path.exists(REFLIB), reason="reference not built here")

i64p = C.POINTER(C.c_int64)
VT = {"d": (np.float64, 1), "s": (np.float32, 1), "z": (np.complex128, 1)}


def _libs():
    from superlu_dist_amd.lib import LIB_PATH
    from superlu_dist_amd import capi
    mine = C.CDLL(LIB_PATH, mode=C.RTLD_LOCAL)
    ref = C.CDLL(REFLIB, mode=C.RTLD_LOCAL)
    return mine, ref, capi


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _case(rng, t):
    """Random supernode partition, one source panel L(:,k) / U(k,jb) and one
    destination block column jb (for _l) / block row ib (for _u)."""
    dt = VT[t][0]
    ns = 12
    w = rng.integers(2, 9, size=ns)
    xsup = np.concatenate([[0], np.cumsum(w)]).astype(np.int64)
    k, jb, ib = 2, 5, 8            # source step k, destination column jb, row block ib > jb
    klst = int(xsup[k + 1])
    nsupc = int(w[jb])
    # U(k, jb): per column fstnz in [xsup[k], klst]; some columns empty
    fst = rng.integers(xsup[k], klst + 1, size=nsupc)
    fst[0] = xsup[k]               # at least one nonempty column
    usub = np.concatenate([[0, 0, 0, jb, 0], fst]).astype(np.int64)
    iukp = 5
    # L(:,k) rows of block ib: a random subset of ib's rows
    rows_ib = np.arange(xsup[ib], xsup[ib + 1])
    src = np.sort(rng.choice(rows_ib, size=max(1, len(rows_ib) - 1), replace=False))
    lsub = np.concatenate([[7, 7], src]).astype(np.int64)   # two leading junk entries
    lptr = 2
    temp_nbrow = len(src)
    ncols_nz = int((klst - fst > 0).sum())
    nbrow = temp_nbrow + 3                                   # LD of tempv > rows used
    tempv = (rng.standard_normal((ncols_nz, nbrow)) +
             (1j * rng.standard_normal((ncols_nz, nbrow)) if t == "z" else 0)).astype(dt)
    return xsup, k, jb, ib, klst, nsupc, usub, iukp, lsub, lptr, temp_nbrow, nbrow, tempv, rng


def _lcol(rng, xsup, jb, ib, t):
    """Destination L block column jb: blocks jb (diag), one before ib, ib, one after."""
    dt = VT[t][0]
    blocks = [jb, ib - 1, ib, ib + 1]
    idx, nsupr = [len(blocks), 0], 0
    for b in blocks:
        r = np.arange(xsup[b], xsup[b + 1])
        r = rng.permutation(r)                                # rows in any order
        idx += [b, len(r)] + list(r)
        nsupr += len(r)
    idx[1] = nsupr
    idx = np.array(idx, dtype=np.int64)
    val = rng.standard_normal(nsupr * int(xsup[jb + 1] - xsup[jb])).astype(dt)
    if t == "z":
        val = val + 1j * rng.standard_normal(val.shape)
    return idx, val.astype(dt)


@pytest.mark.parametrize("t", ["d", "s", "z"])
@pytest.mark.parametrize("seed", range(6))
def test_scatter_l_matches_reference(t, seed):
    mine, ref, capi = _libs()
    rng = np.random.default_rng(seed)
    xsup, k, jb, ib, klst, nsupc, usub, iukp, lsub, lptr, tnb, nbrow, tempv, rng = _case(rng, t)
    idx, val0 = _lcol(rng, xsup, jb, ib, t)
    usub32, lsub32 = usub.astype(np.int32), lsub.astype(np.int32)
    grid = capi.grid_1x1()
    outs = []
    for lib in (mine, ref):
        for fn in ("scatter_l", "scatter_l_1"):
            val = val0.copy()
            ind = np.zeros(1024, dtype=np.int32)
            ind2 = np.zeros(1024, dtype=np.int32)
            iptrs = (C.POINTER(C.c_int64) * 8)()
            vptrs = (C.c_void_p * 8)()
            ljb = 1
            iptrs[ljb] = idx.ctypes.data_as(i64p)
            vptrs[ljb] = _p(val)
            f = getattr(lib, t + fn)
            f.restype = None
            # dscatter_l_1 takes 32-bit usub / lsub (SRC/dscatter.c:29-43)
            us, ls = (usub, lsub) if fn == "scatter_l" else (usub32, lsub32)
            common = [C.c_int(ib), C.c_int(ljb), C.c_int(nsupc), C.c_int64(iukp), _p(xsup),
                      C.c_int(klst), C.c_int(nbrow), C.c_int64(lptr), C.c_int(tnb), _p(us),
                      _p(ls), _p(tempv), _p(ind)]
            if fn == "scatter_l":
                common.append(_p(ind2))
            f(*common, iptrs, vptrs, C.byref(grid))
            outs.append(val)
    np.testing.assert_array_equal(outs[0], outs[2])     # scatter_l: mine == reference
    np.testing.assert_array_equal(outs[1], outs[3])     # scatter_l_1
    assert not np.array_equal(outs[0], val0)             # something was updated


@pytest.mark.parametrize("t", ["d", "s", "z"])
@pytest.mark.parametrize("seed", range(6))
def test_scatter_u_matches_reference(t, seed):
    mine, ref, capi = _libs()
    rng = np.random.default_rng(100 + seed)
    xsup, k, jb, ib, klst, nsupc, usub, iukp, lsub, lptr, tnb, nbrow, tempv, rng = _case(rng, t)
    # destination U block row "ib" := a row block above jb: re-use ib < jb by
    # swapping roles (dscatter_u updates U(ib, jb) with ib < jb)
    ib_u = 3
    rows = np.arange(xsup[ib_u], xsup[ib_u + 1])
    src = np.sort(rng.choice(rows, size=len(rows), replace=False))
    lsub = np.concatenate([[7, 7], src]).astype(np.int64)
    tnb = len(src)
    nbrow = tnb + 2
    ncols_nz = int((klst - usub[iukp:] > 0).sum())
    dt = VT[t][0]
    tempv = rng.standard_normal((ncols_nz, nbrow)).astype(dt)
    if t == "z":
        tempv = (tempv + 1j * rng.standard_normal(tempv.shape)).astype(dt)
    ilst = int(xsup[ib_u + 1])
    # destination block row ib_u holds blocks 4, jb=5, 9 with per-column fstnz
    blocks = [4, jb, 9]
    uidx, uval_len = [len(blocks), 0, 0], 0
    for b in blocks:
        wb = int(xsup[b + 1] - xsup[b])
        f = rng.integers(xsup[ib_u], ilst + 1, size=wb)
        if b == jb:
            f[:] = xsup[ib_u]      # full segments in the destination block
        nnz = int((ilst - f).sum())
        uidx += [b, nnz] + list(f)
        uval_len += nnz
    uidx[1] = uval_len
    uidx[2] = len(uidx)
    uidx = np.array(uidx, dtype=np.int64)
    u0 = rng.standard_normal(uval_len).astype(dt)
    grid = capi.grid_1x1()
    outs = []
    for lib in (mine, ref):
        uv = u0.copy()
        iptrs = (C.POINTER(C.c_int64) * 8)()
        vptrs = (C.c_void_p * 8)()
        iptrs[ib_u] = uidx.ctypes.data_as(i64p)
        vptrs[ib_u] = _p(uv)
        f = getattr(lib, t + "scatter_u")
        f.restype = None
        f(C.c_int(ib_u), C.c_int(jb), C.c_int(nsupc), C.c_int64(iukp), _p(xsup), C.c_int(klst),
          C.c_int(nbrow), C.c_int64(lptr), C.c_int(tnb), _p(lsub), _p(usub), _p(tempv), iptrs,
          vptrs, C.byref(grid))
        outs.append(uv)
    np.testing.assert_array_equal(outs[0], outs[1])
    assert not np.array_equal(outs[0], u0)
