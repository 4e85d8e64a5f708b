"""PMC counters of the conv dispatches in gpurun_out/<tag>_p*/ (tools/pmc_conv.sh), averaged per kernel instance
(full name with template arguments, so the arithmetic modes of one tile are told apart), with the derived ratios:
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM_GUI_ACTIVE / 8 (tools/pmc_shapes.py's normalisation).
usage: python tools/pmc_conv.py TAG [kernel-substring ...]"""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc_c3_g23"
kern = sys.argv[2:] or ["conv_gemm", "conv_emu", "conv_wsb", "conv_wst", "conv_gs", "k_rb_pair"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(collections.Counter)
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not any(k in name for k in kern):
            continue
        short = name.replace("(anonymous namespace)::", "").replace("rvcx::", "").split("(")[0].replace("void ", "")
        agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[short][r["Counter_Name"]] += 1
for short in sorted(agg):
    a = {k: agg[short][k] / cnt[short][k] for k in agg[short]}
    print(short)
    for k in sorted(a):
        print(f"  {k:28s} {a[k]:16.1f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:  # tools/pmc_shapes.py's normalisation
        print(f"  -> MFMA busy {a['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1.0, 1024 * a['GRBM_GUI_ACTIVE'] / 8):.3f}")
    if "SQ_INSTS_MFMA" in a and "SQ_INSTS_VALU" in a:
        print(f"  -> VALU / MFMA instructions {a['SQ_INSTS_VALU'] / max(1.0, a['SQ_INSTS_MFMA']):.2f}, "
              f"SALU / MFMA {a.get('SQ_INSTS_SALU', 0) / max(1.0, a['SQ_INSTS_MFMA']):.2f}, "
              f"LDS / MFMA {a.get('SQ_INSTS_LDS', 0) / max(1.0, a['SQ_INSTS_MFMA']):.2f}")
    if "SQ_WAIT_ANY" in a and "SQ_WAVE_CYCLES" in a:
        print(f"  -> wait_any / wave_cycles {a['SQ_WAIT_ANY'] / max(1.0, a['SQ_WAVE_CYCLES']):.3f}, "
              f"wait_inst_lds / wave_cycles {a.get('SQ_WAIT_INST_LDS', 0) / max(1.0, a['SQ_WAVE_CYCLES']):.3f}")
