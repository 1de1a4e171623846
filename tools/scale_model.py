"""Per-level model of the 2D-grid factorization time.

Inputs:
  * the 1-GPU per-level log of `bench.py --level-log` (stderr lines
    "[slu rank 0] lvl nsup diag trsm big small atomic GFLOP diag_ms trsm_ms
    big_ms small_ms comm_ms TF/s wall_ms");
  * the per-level panel volumes of the same LU structure (computed here from
    the front-end: bytes of L(:,k) below the diagonal block and of U(k,:)
    for the supernodes of each level).

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


def level_volumes(nx):
    """Per level: bytes of L panels below the diagonal blocks and of U panels."""
    from superlu_dist_amd.frontend import STENCIL_3D7, Csc, Symbolic, nd_order
    A = Csc.stencil(STENCIL_3D7, nx, nx, nx)
    S = Symbolic(A, nd_order(nx, nx, nx), 60, 256)
    lu = S.distribute()
    ns, xs = S.nsupers, S.xsup
    lvl = np.zeros(ns, dtype=np.int64)
    lp = np.zeros(ns)
    up = np.zeros(ns)
    for k in range(ns):
        ix = lu.Lidx[lu.Loff[k]:]
        w = xs[k + 1] - xs[k]
        lp[k] = (ix[1] - w) * w * 8.0
        p = 2
        for _ in range(int(ix[0])):
            ib = ix[p]
            if ib != k:
                lvl[ib] = max(lvl[ib], lvl[k] + 1)
            p += 2 + ix[p + 1]
        if lu.Uoff[k] >= 0:
            iu = lu.Uidx[lu.Uoff[k]:]
            up[k] = iu[1] * 8.0
            p = 3
            for _ in range(int(iu[0])):
                jb = iu[p]
                lvl[jb] = max(lvl[jb], lvl[k] + 1)
                p += 2 + xs[jb + 1] - xs[jb]
    nl = int(lvl.max()) + 1
    return ([float(lp[lvl == L].sum()) for L in range(nl)],
            [float(up[lvl == L].sum()) for L in range(nl)])


def model(rows, Lp, Up, pr, pc, bw, lat):
    P = pr * pc
    waves = lambda t: max(1, math.ceil(t / 512))  # noqa: E731
    chain, schur = [], []
    for r in rows:
        L = r["lvl"]
        if P == 1:
            chain.append(r["diag"] + r["trsm"])
            schur.append(r["schur"])
            continue
        recv = Lp[L] / pr * (pc - 1) / pc + Up[L] / pc * (pr - 1) / pr
        ncoll = (pr > 1) + (pc > 1)  # one grouped diag broadcast + one grouped panel broadcast
        comm = 2 * ncoll * lat * 1e-3 + recv / bw / 1e6
        chain.append(r["diag"] + r["trsm"] / ((pr + pc) / 2) + comm)
        tiles = r["big"] + r["small"]
        schur.append(r["schur"] * waves(tiles / P) / waves(tiles))
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
    a = ap.parse_args()
    rows = parse_log(a.log)
    Lp, Up = level_volumes(a.nx)
    t1, _, _ = model(rows, Lp, Up, 1, 1, a.bw, a.lat)
    out = {"levels": len(rows), "bw_GBs": a.bw, "lat_us": a.lat, "t1_ms": round(t1, 1),
           "panel_volume_GB": round((sum(Lp) + sum(Up)) / 1e9, 2)}
    for pr, pc in ((1, 2), (2, 2), (2, 4), (4, 2)):
        t, chain, schur = model(rows, Lp, Up, pr, pc, a.bw, a.lat)
        bound = sum(1 for i in range(len(rows) - 1) if chain[i + 1] > schur[i])
        out[f"{pr}x{pc}"] = {"t_ms": round(t, 1), "speedup": round(t1 / t, 2),
                             "levels_chain_bound": bound,
                             "comm_recv_GB_per_rank": round(
                                 sum(Lp[L] / pr * (pc - 1) / pc + Up[L] / pc * (pr - 1) / pr
                                     for L in range(len(rows))) / 1e9, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
