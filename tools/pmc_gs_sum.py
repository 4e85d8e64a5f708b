"""Average per-dispatch counters of one kernel over the PMC passes of tools/pmc_gs.sh.
usage: python tools/pmc_gs_sum.py gpurun_out PREFIX KERNEL_SUBSTRING"""
import collections
import csv
import glob
import os
import sys

d, prefix, kern = sys.argv[1], sys.argv[2], sys.argv[3]
tot = collections.defaultdict(float)
cnt = collections.defaultdict(int)
for f in sorted(glob.glob(os.path.join(d, prefix + "_p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
print(prefix, kern)
for k in sorted(tot):
    print(f"  {k:32s} {tot[k] / cnt[k]:16.1f}")
