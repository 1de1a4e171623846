"""Per-level model of the 2D-grid factorization time.

Inputs:
  * the 1-GPU per-level log of `bench.py --level-log` (stderr lines
    "[slu rank 0] lvl nsup diag trsm big small atomic GFLOP diag_ms trsm_ms
    big_ms small_ms comm_ms TF/s wall_ms");
  * the per-level panel volumes of the same LU structure (computed here:
    bytes of L(:,k) below the diagonal block and of U(k,:) for the
    supernodes of each level) -- the coarse partition the plans factor
    (the amalgamated reference structure, Symbolic(reference=True,
    coarse=True); --frontend: the library front-end's, for round-2 logs).

For a Pr x Pc grid (P = Pr Pc ranks, one per GPU) each level costs
  chain_L = diag_L + trsm_L / ((Pr + Pc) / 2) + comm_L
  comm_L  = n_coll * lat + recv_bytes_L / bw
            recv_bytes_L = Lp_L / Pr * (Pc - 1) / Pc + Up_L / Pc * (Pr - 1) / Pr
  schur_L = schur1_L * waves(tiles_L / P) / waves(tiles_L),  waves(t) = ceil(t / 512)
            (512 = two 128x128 tiles per CU resident on 256 CUs)
and with the engine's one-level look-ahead (the next level's diag LU, TRSMs
and broadcasts run beside this level's bulk Schur update)
  T = chain_0 + sum_L max(schur_L, chain_{L+1}).
The 1-GPU times are the measured ones (no look-ahead modelled at P = 1).

usage: python tools/scale_model.py LEVEL_LOG [--nx 100] [--bw 50] [--lat 30]
       (bw in GB/s per rank for a row/column broadcast over xGMI, lat in us)
"""
import argparse
import json
import math
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_log(path):
    rows = []
    for line in open(path):
        m = re.match(r"\[slu rank 0\]\s+(\d+)\s+(\d+)\s+(\d+)\s+(\d+)\s+(\d+)\s+(\d+)\s+(\d+)\s+"
                     r"([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+"
                     r"([\d.]+)\s+([\d.]+)", line)
        if m:
            v = m.groups()
            rows.append({"lvl": int(v[0]), "nsup": int(v[1]), "big": int(v[4]), "small": int(v[5]),
                         "gflop": float(v[7]), "diag": float(v[8]), "trsm": float(v[9]),
                         "schur": float(v[10]) + float(v[11]), "wall": float(v[14])})
    # keep the last complete log (bench prints one per timed step)
    out, seen = [], set()
    for r in reversed(rows):
        if r["lvl"] in seen:
            break
        seen.add(r["lvl"])
        out.append(r)
    return sorted(out, key=lambda r: r["lvl"])


def level_volumes(nx, frontend=False):
    """Per supernode: level, bytes of L(:,k) below the diagonal block, bytes
    of U(k,:), and the L block rows / U block columns (for the need masks)."""
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    S = (Symbolic(A, nd_order(nx, nx, nx), 60, 256) if frontend else
         Symbolic(A, nd_order(nx, nx, nx), 60, 256, reference=True, coarse=True))
    lu = S.distribute()
    ns, xs = S.nsupers, S.xsup
    lvl = np.zeros(ns, dtype=np.int64)
    sn = []
    for k in range(ns):
        ix = lu.Lidx[lu.Loff[k]:]
        w = xs[k + 1] - xs[k]
        lrows, p, ib_list = [], 2, []
        for _ in range(int(ix[0])):
            ib, nr = int(ix[p]), int(ix[p + 1])
            if ib != k:
                lvl[ib] = max(lvl[ib], lvl[k] + 1)
                ib_list.append((ib, nr))
            p += 2 + nr
        jb_list, ub = [], 0.0
        if lu.Uoff[k] >= 0:
            iu = lu.Uidx[lu.Uoff[k]:]
            ub = iu[1] * 8.0
            p = 3
            for _ in range(int(iu[0])):
                jb = int(iu[p])
                lvl[jb] = max(lvl[jb], lvl[k] + 1)
                jb_list.append(jb)
                p += 2 + xs[jb + 1] - xs[jb]
        sn.append((k, int(w), ib_list, jb_list, ub))
    return lvl, sn


def recv_volumes(lvl, sn, pr, pc):
    """Average bytes a rank receives per level with the sparse sections of
    engine.hip (a rank gets L(:,k) only if U(k,:) has blocks on its process
    column, U(k,:) only if L(:,k) has rows on its process row)."""
    nl = int(lvl.max()) + 1
    vol = np.zeros(nl)
    for k, w, ib_list, jb_list, ub in sn:
        cols = {jb % pc for jb in jb_list} - {k % pc}
        rows_with = {}
        for ib, nr in ib_list:
            rows_with[ib % pr] = rows_with.get(ib % pr, 0) + nr
        # L panel rows of process row r go to the needing columns of that row
        lbytes = sum(nr * w * 8.0 for nr in rows_with.values())
        vol[lvl[k]] += lbytes * len(cols) / (pr * pc)
        # U(k,:) on column c (1/pc of it) goes to the rows that have L rows
        need_rows = set(rows_with) - {k % pr}
        vol[lvl[k]] += ub * len(need_rows) / (pr * pc)
    return vol


def model(rows, vol, pr, pc, bw, lat, chunks=1, trsm_scale=1.0):
    P = pr * pc
    waves = lambda t: max(1, math.ceil(t / 512))  # noqa: E731
    chain, schur = [], []
    for r in rows:
        L = r["lvl"]
        if P == 1:
            chain.append(r["diag"] + r["trsm"])
            schur.append(r["schur"])
            continue
        recv = vol[L]
        ncoll = (pr > 1) + (pc > 1)  # one grouped diag broadcast + one grouped panel broadcast
        xfer = recv / bw / 1e6
        trsm = trsm_scale * r["trsm"] / ((pr + pc) / 2)
        # chunks > 1 (engine.hip, SLU_PANEL_CHUNKS): the panels go out in
        # `chunks` groups on the comm stream -- TRSM of chunk c + 1 beside
        # the transfer of chunk c -- and the level's Schur tiles of a chunk
        # start when it is in, so the chain to the level's first tiles holds
        # one chunk's TRSM and transfer, and the rest of both run beside the
        # level's own update
        # (the latency of the later chunks' groups runs beside the update too)
        comm = 2 * ncoll * lat * 1e-3 + xfer / chunks
        chain.append(r["diag"] + trsm / chunks + comm)
        tiles = r["big"] + r["small"]
        s1 = r["schur"] * waves(tiles / P) / waves(tiles)
        tail = max(xfer + ncoll * lat * 1e-3 * chunks, trsm) * (chunks - 1) / chunks
        schur.append(max(s1, tail + s1 / chunks) if chunks > 1 else s1)
    if P == 1:
        return sum(r["wall"] for r in rows), chain, schur
    t = chain[0] + sum(max(schur[i], chain[i + 1] if i + 1 < len(rows) else 0.0)
                       for i in range(len(rows)))
    return t, chain, schur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--nx", type=int, default=100)
    ap.add_argument("--bw", type=float, default=50.0, help="GB/s per rank per broadcast")
    ap.add_argument("--lat", type=float, default=30.0, help="us per collective")
    ap.add_argument("--frontend", action="store_true",
                    help="volumes of the library front-end's partition (round-2 logs)")
    ap.add_argument("--t1", type=float, default=None,
                    help="measured 1-GPU factor time (ms); default: sum of the log's level walls")
    ap.add_argument("--diag-scale", type=float, default=1.0,
                    help="what-if: multiply every level's diagonal-LU time (grid chains only)")
    ap.add_argument("--trsm-scale", type=float, default=1.0,
                    help="what-if: multiply every level's TRSM time (grid chains only)")
    ap.add_argument("--chunks", type=int, default=1,
                    help="panel exchange in this many groups, the Schur update starting with the first")
    a = ap.parse_args()
    rows = parse_log(a.log)
    t1, _, _ = model(rows, None, 1, 1, a.bw, a.lat)
    for r in rows:
        r["diag"] *= a.diag_scale
    lvl, sn = level_volumes(a.nx, a.frontend)
    if a.t1:
        t1 = a.t1
    out = {"levels": len(rows), "bw_GBs": a.bw, "lat_us": a.lat, "t1_ms": round(t1, 1),
           "diag_scale": a.diag_scale, "trsm_scale": a.trsm_scale, "chunks": a.chunks}
    for pr, pc in ((1, 2), (2, 2), (2, 4), (4, 2)):
        vol = recv_volumes(lvl, sn, pr, pc)
        t, chain, schur = model(rows, vol, pr, pc, a.bw, a.lat, a.chunks, a.trsm_scale)
        bound = sum(1 for i in range(len(rows) - 1) if chain[i + 1] > schur[i])
        out[f"{pr}x{pc}"] = {"t_ms": round(t, 1), "speedup": round(t1 / t, 2),
                             "levels_chain_bound": bound,
                             "recv_GB_per_rank": round(float(vol.sum()) / 1e9, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
