"""Average the PMC counters of every conv_gemm_kernel dispatch in gpurun_out/pmc_c*_g*_p*/ (tools/pmc_conv.sh)."""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc_c3_g1"
kern = sys.argv[2:] or ["conv_gemm", "conv_emu"]
agg = collections.defaultdict(float)
cnt = collections.Counter()
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if not any(k in r["Kernel_Name"] for k in kern):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / cnt[k]:16.1f}")
