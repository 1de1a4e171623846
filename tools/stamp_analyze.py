"""Summarise the per-tile k_schur_big stamps of a diagnostics build
(tools/ab_build.sh stamp "-DSLU_SB_STAMP"; SLU_STAMP_OUT=file).

Per tile: prologue (table loads + first stage), K loop and epilogue (C
through LDS + scatter) in shader cycles; which CU it ran on; how many other
workgroups shared its CU while it was in each phase.
usage: python tools/stamp_analyze.py stamps.bin
"""
import sys
from collections import defaultdict

import numpy as np


def load(fn):
    a = np.fromfile(fn, dtype=np.uint64).reshape(-1, 4)
    rt0 = (a[:, 0] & ((1 << 40) - 1)).astype(np.int64)
    dur = (a[:, 0] >> 40).astype(np.int64)
    pro = (a[:, 1] & 0xFFFFFFFF).astype(np.int64)
    kl = (a[:, 1] >> 32).astype(np.int64)
    epi = (a[:, 2] & 0xFFFFFFFF).astype(np.int64)
    hw = (a[:, 2] >> 32).astype(np.int64)
    m = a[:, 3]
    xcc = (m & 15).astype(np.int64)
    kw = ((m >> 4) & 1023).astype(np.int64)
    mr = ((m >> 14) & 255).astype(np.int64)
    nc = ((m >> 22) & 255).astype(np.int64)
    at = ((m >> 30) & 1).astype(np.int64)
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    return dict(rt0=rt0, dur=dur, pro=pro, kl=kl, epi=epi, xcc=xcc, kw=kw, mr=mr, nc=nc,
                at=at, cuid=cuid)


def main():
    d = load(sys.argv[1])
    n = len(d["kw"])
    tot = d["pro"] + d["kl"] + d["epi"]
    print(f"{n} tiles, {len(np.unique(d['cuid']))} distinct CUs")
    full = (d["mr"] == 128) & (d["nc"] == 128)
    for name, sel in (("all", np.ones(n, bool)), ("full 128x128, kw>=192", full & (d["kw"] >= 192)),
                      ("full, kw 256", full & (d["kw"] == 256)), ("kw<64", d["kw"] < 64)):
        if not sel.any():
            continue
        p, k, e, t = (x[sel].sum() for x in (d["pro"], d["kl"], d["epi"], tot))
        print(f"{name:24s} {sel.sum():8d} tiles: prologue {p / t:6.1%} K loop {k / t:6.1%} "
              f"epilogue {e / t:6.1%}; mean cycles pro {d['pro'][sel].mean():8.0f} "
              f"K {d['kl'][sel].mean():9.0f} epi {d['epi'][sel].mean():8.0f}; "
              f"K cycles per 16-deep stage {(d['kl'][sel] / ((d['kw'][sel] + 15) // 16)).mean():7.0f}")
    # cycles per realtime tick (100 MHz) -> clock
    sel = d["dur"] > 100
    print(f"shader clock ~ {np.median(tot[sel] / d['dur'][sel]) * 100:.0f} MHz")
    # co-residency: for each tile, mean number of tiles on the same CU overlapping it
    by = defaultdict(list)
    for i in range(n):
        by[int(d["cuid"][i])].append(i)
    ov = []
    for cu, idx in by.items():
        idx = sorted(idx, key=lambda i: d["rt0"][i])
        for j, i in enumerate(idx):
            s, e = d["rt0"][i], d["rt0"][i] + d["dur"][i]
            c = 0
            for q in idx[max(0, j - 8):j + 8]:
                if q != i and d["rt0"][q] < e and d["rt0"][q] + d["dur"][q] > s:
                    c += 1
            ov.append(c)
    ov = np.array(ov)
    print("tiles overlapping on the same CU:", {int(v): int((ov == v).sum()) for v in np.unique(ov)})


if __name__ == "__main__":
    main()
