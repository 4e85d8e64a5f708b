"""List the kernels of the LAST stage call in a tools/prof_stage.py trace (in order, with durations): the call's
kernels are the last K of the trace, K = (kernels after the setup's k_f0post) / N.
usage: python tools/stage_kernels.py RUN.db N [-v]"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("rvcx::", "").replace("(anonymous namespace)::", "")
    head = n.split("(")[0]
    return head[:60]


def main():
    db, n = sys.argv[1], int(sys.argv[2])
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    nc = "kernel_name" if "kernel_name" in cols else "name"
    rows = con.execute(f"select {nc}, start, end from kernels order by start").fetchall()
    idx = max(i for i, r in enumerate(rows) if "k_f0post" in r[0])
    rest = rows[idx + 1:]
    k = len(rest) // n
    last = rest[-k:]
    t0 = last[0][1]
    print(f"{k} kernels per call, span {(last[-1][2] - t0) / 1e3:.1f} us, busy {sum(e - s for _, s, e in last) / 1e3:.1f} us")
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in last:
        agg[short(name)][0] += 1
        agg[short(name)][1] += (e - s) / 1e3
    for key, (c, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {c:4d} {us:8.1f} us  {key}")
    if "-v" in sys.argv:
        for name, s, e in last:
            print(f"    {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {short(name)}")


if __name__ == "__main__":
    main()
