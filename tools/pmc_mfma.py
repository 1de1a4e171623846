"""MFMA utilisation of a kernel from one rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE.

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over every
SIMD; GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS
note), so the dispatch's wall cycles are GRBM_GUI_ACTIVE / 8 and
    mfma_util = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
and the effective clock = GRBM_GUI_ACTIVE / 8 / kernel duration.
usage: python tools/pmc_mfma.py PMC_DIR [KERNEL_SUBSTRING] [out.txt]
"""
import collections
import csv
import glob
import os
import sys


def main(d, kname="k_schur_big", out=None):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"]
            if kname not in k:
                continue
            did = r["Dispatch_Id"]
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            names[did] = k.split("(")[0].replace("void ", "")
            if "End_Timestamp" in r and r.get("Start_Timestamp"):
                dur[did] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for v in per.values())
    grbm = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in per.values())
    sqb = sum(v.get("SQ_BUSY_CYCLES", 0) for v in per.values())
    wall_cyc = grbm / 8
    t = sum(dur.values())
    lines = [f"# MFMA utilisation of {sorted(set(names.values()))} over {len(per)} dispatches",
             f"SQ_VALU_MFMA_BUSY_CYCLES {busy:.4e}", f"SQ_BUSY_CYCLES {sqb:.4e}",
             f"GRBM_GUI_ACTIVE {grbm:.4e} (sum over 8 XCDs)",
             f"mfma_util = MFMA_BUSY / (GRBM/8 * 1024 SIMDs) = {busy / (wall_cyc * 1024):.4f}"]
    if t > 0:
        lines.append(f"kernel time {t * 1e3:.2f} ms, effective clock {wall_cyc / t / 1e9:.3f} GHz")
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
