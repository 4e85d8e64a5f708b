"""Per-kernel-name, per-grid comparison of two rocprofv3 kernel-trace databases (same workload)."""
import sqlite3
import sys
from collections import defaultdict


def load(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, grid_x, grid_y, grid_z, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    for n, gx, gy, gz, s, e in rows:
        short = n.split("(")[0].replace("void ", "").replace("rvcx::", "")
        key = (short, gx, gy, gz)
        agg[key][0] += 1
        agg[key][1] += (e - s) / 1e3
    return agg


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    keys = set(a) | set(b)
    rows = []
    for k in keys:
        ca, ta = a.get(k, [0, 0.0])
        cb, tb = b.get(k, [0, 0.0])
        rows.append((tb - ta, k, ca, ta, cb, tb))
    rows.sort(key=lambda r: -abs(r[0]))
    print(f"{'kernel':48s} {'grid':>22s} {'nA':>4s} {'usA':>9s} {'nB':>4s} {'usB':>9s} {'dB-A':>8s}")
    for d, k, ca, ta, cb, tb in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
        print(f"{k[0][:48]:48s} {str(k[1:]):>22s} {ca:4d} {ta:9.1f} {cb:4d} {tb:9.1f} {d:8.1f}")
    print(f"total A {sum(v[1] for v in a.values()):.1f} us  B {sum(v[1] for v in b.values()):.1f} us")


if __name__ == "__main__":
    main()
