"""Per-kernel statistics from a rocprofv3 rocpd database (--kernel-trace; ROCm 7 writes SQLite):
name, calls, total / average / min / max duration.  Usage: python tools/kstats.py <db> [--csv out]"""
import sqlite3
import sys
from collections import defaultdict


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels").fetchall()
    d = defaultdict(list)
    for name, s, e in rows:
        d[name].append((e - s) / 1e3)      # ns -> us
    out = []
    for k, v in d.items():
        out.append((k, len(v), sum(v), sum(v) / len(v), min(v), max(v)))
    out.sort(key=lambda r: -r[2])
    return out


if __name__ == "__main__":
    st = stats(sys.argv[1])
    lines = ["Name,Calls,TotalDurationUs,AverageUs,MinUs,MaxUs"]
    for r in st:
        lines.append('"%s",%d,%.2f,%.3f,%.3f,%.3f' % r)
    if "--csv" in sys.argv:
        open(sys.argv[sys.argv.index("--csv") + 1], "w").write("\n".join(lines) + "\n")
    tot = sum(r[2] for r in st)
    for r in st[:25]:
        print("%-70s %6d %10.1f us %8.2f avg  %5.1f%%" % (r[0][:70], r[1], r[2], r[3], 100 * r[2] / tot))
