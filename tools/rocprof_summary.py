"""Summarise a rocprofv3 --kernel-trace --stats run (SQLite .db or
kernel_stats.csv) into a small text table for profiles/."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4]))
            for r in c.execute("select name,total_calls,total_duration,average,percentage "
                               "from top_kernels")]


def from_csv(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return rows


def main(d, out=None):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    lines = [f"# rocprofv3 --kernel-trace --stats summary of {d}",
             f"{'kernel':<60} {'calls':>6} {'total_ms':>10} {'avg_us':>10} {'pct':>6}"]
    for name, calls, tot_us, avg_us, pct in rows:
        short = name.split("(")[0].replace("void ", "")[:60]
        lines.append(f"{short:<60} {calls:>6} {tot_us/1e3:>10.3f} {avg_us:>10.1f} {pct:>6.2f}")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
