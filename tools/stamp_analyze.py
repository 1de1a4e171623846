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
    # phase alignment: per CU, the time with >= 1 tile resident, with >= 1 /
    # 2 tiles in their K loop (K-loop intervals placed by the cycle counts)
    cpt = np.median(tot[sel] / d["dur"][sel])  # cycles per 100 MHz tick
    res = k1 = k2 = 0.0
    for cu, idx in by.items():
        ev_r, ev_k = [], []
        for i in idx:
            s0 = float(d["rt0"][i])
            ev_r += [(s0, 1), (s0 + d["dur"][i], -1)]
            ks = s0 + d["pro"][i] / cpt
            ev_k += [(ks, 1), (ks + d["kl"][i] / cpt, -1)]
        for ev, acc in ((ev_r, "r"), (ev_k, "k")):
            ev.sort()
            c, last = 0, None
            for t, dv in ev:
                if last is not None and c > 0:
                    if acc == "r":
                        res += t - last
                    else:
                        k1 += t - last
                        if c > 1:
                            k2 += t - last
                last = t
                c += dv
    print(f"per CU, of the time with a tile resident: >=1 tile in its K loop {k1 / res:.1%}, "
          f">=2 tiles in their K loops {k2 / res:.1%}")
    # what a full kw-256 tile's K loop overlapped on its CU: the other tiles'
    # prologue / K loop / epilogue time over its K interval, and its cycles
    # per stage binned by the dominant one
    bins = defaultdict(list)
    for cu, idx in by.items():
        idx = sorted(idx, key=lambda i: d["rt0"][i])
        ph = []
        for i in idx:
            s0 = float(d["rt0"][i])
            a = s0 + d["pro"][i] / cpt
            b = a + d["kl"][i] / cpt
            ph.append((s0, a, b, b + d["epi"][i] / cpt))
        for j, i in enumerate(idx):
            if not (full[i] and d["kw"][i] == 256):
                continue
            ks, ke = ph[j][1], ph[j][2]
            ov = [0.0, 0.0, 0.0]
            for q in range(max(0, j - 8), min(len(idx), j + 8)):
                if q == j:
                    continue
                p0, p1, p2, p3 = ph[q]
                for t, (lo, hi) in enumerate(((p0, p1), (p1, p2), (p2, p3))):
                    ov[t] += max(0.0, min(hi, ke) - max(lo, ks))
            L = max(ke - ks, 1e-9)
            f = [x / L for x in ov]
            key = "alone" if sum(f) < 0.3 else ("pro", "K", "epi")[int(np.argmax(f))]
            bins[key].append(d["kl"][i] / 16)
    for key in ("alone", "pro", "K", "epi"):
        v = np.array(bins.get(key, [0]))
        print(f"full kw-256 tiles whose K loop mostly overlapped {key:5s}: {len(bins.get(key, [])):7d} tiles, "
              f"cycles per stage mean {v.mean():7.0f} median {np.median(v):7.0f}")


if __name__ == "__main__":
    main()
