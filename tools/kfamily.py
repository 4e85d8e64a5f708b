"""Per-step kernel time by family (template instance) from a rocprofv3 kernel-trace database, averaged over the
steps after the first (k_odd_ext marks a step start). usage: python tools/kfamily.py RUN.db"""
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, start, end from kernels order by start").fetchall()
starts = [r[1] for r in rows if "k_odd_ext" in r[0]]
if len(starts) < 3:
    sys.exit("fewer than 3 steps in the trace")
t0, t1 = starts[1], starts[-1]
n = len(starts) - 2
fam = defaultdict(float)
for name, s, e in rows:
    if t0 <= s < t1:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("rvcx::", "")
        fam[short] += (e - s) / 1e3 / n
tot = sum(fam.values())
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {v:9.1f} us/step  {k[:90]}")
for fam_name in ("conv_wsb16", "conv_wst16", "conv_gs", "k_rb_pair"):
    print(f"  {sum(v for k, v in fam.items() if k.startswith(fam_name)):9.1f} us/step  all {fam_name}*")
print(f"  {tot:9.1f} us/step  total over {n} steps")
