"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE run separately: they do not fit one TCC pass on gfx950).

Units and corrections (MI355X_MICROARCH.md, HBM section): both counters are in
KiB; on gfx950 FETCH_SIZE tallies 128-B read requests at 64 B, i.e. it reports
1/2 of the bytes of a wide coalesced read, so it is doubled here.  WRITE_SIZE
is taken as is.
usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR [out.txt [KEY]]
With KEY (e.g. lap3d_100_1x1) the bytes per launch are also merged into
profiles/traffic.json, which bench.py reports as roofline.traffic.
"""
import collections
import csv
import glob
import os
import sys


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    tot, calls = collections.defaultdict(float), collections.defaultdict(set)
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k] += float(r["Counter_Value"])
            calls[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in calls.items()}


def main(fd, wd, out=None):
    fetch, nf = load(fd, "FETCH_SIZE")
    write, nw = load(wd, "WRITE_SIZE")
    lines = ["# HBM traffic per kernel (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), KiB -> bytes",
             f"{'kernel':<44} {'calls':>6} {'read_GB':>10} {'write_GB':>10} {'MB/launch':>11}"]
    res = {}
    for k in sorted(fetch, key=lambda k: -fetch[k]):
        rd = 2 * fetch[k] * 1024
        wr = write.get(k, 0.0) * 1024
        n = nf[k]
        res[k] = (rd + wr) / n
        lines.append(f"{k[:44]:<44} {n:>6} {rd/1e9:>10.3f} {wr/1e9:>10.3f} {(rd+wr)/n/1e6:>11.2f}")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)
    return res


if __name__ == "__main__":
    res = main(*sys.argv[1:4])
    if len(sys.argv) > 4:
        import json
        key = sys.argv[4]
        jf = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                          "traffic.json")
        d = json.load(open(jf)) if os.path.exists(jf) else {}
        d[key] = {k.replace("slu::", ""): round(v) for k, v in res.items() if "slu::" in k}
        d[key]["source"] = os.path.basename(sys.argv[3]) if len(sys.argv) > 3 else ""
        json.dump(d, open(jf, "w"), indent=1, sort_keys=True)
