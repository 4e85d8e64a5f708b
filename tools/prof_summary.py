"""Summarise a rocprofv3 kernel-trace database (.db) into a per-kernel table.

Usage: prof_summary.py RUN.db STEPS [FAMILY_SUBSTRING ...]
STEPS = number of pipeline steps the traced program ran (warm-up + timed); per-step figures
divide by it. Each FAMILY_SUBSTRING adds an aggregate line over all kernels whose name contains
it (e.g. conv_gemm_kernel: the dominant kernel bench.py's roofline is computed for).
"""
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = cur.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
    return agg


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    families = sys.argv[3:]
    agg = from_db(path)
    total = sum(v[1] for v in agg.values())
    print(f"{'kernel':90s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'%':>6s}")
    for n, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        short = n if len(n) < 88 else n[:85] + "..."
        print(f"{short:90s} {c:7d} {ms:10.3f} {1000 * ms / c:9.2f} {100 * ms / total:6.2f}")
    print(f"TOTAL kernel ms {total:.3f}  (per step over {steps:g} steps: {total / steps:.3f})")
    for fam in families:
        c = sum(v[0] for k, v in agg.items() if fam in k)
        ms = sum(v[1] for k, v in agg.items() if fam in k)
        print(f"FAMILY {fam}: calls {c} ({c / steps:g}/step)  total {ms:.3f} ms  per step {ms / steps:.3f} ms  "
              f"avg {1000 * ms / max(c, 1):.2f} us/launch")


if __name__ == "__main__":
    main()
