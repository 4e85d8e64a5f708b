"""Per-shape table of the C2 step's contraction launches from the three PMC passes of tools/pmc_traffic.sh.

Each pass ran bench.py with the per-launch events inline on one stream and RVCX_PROF_DUMP set, so the conv-family
dispatches of the timed step, in dispatch order, are the dump's lines in order (the split-K combine dispatches
are charged to the contraction before them). Per shape (2d, M, N, C_in, taps, batch, ksplit; taps < 0 marks the
fused ResBlock pair of kernel size -taps): launches, event time, TFLOP/s, algorithmic bytes (operands read once,
result written once), measured HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md), their ratio, and
MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM_GUI_ACTIVE / 8).
usage: python tools/pmc_shapes.py [gpurun_out] [top]
"""
import collections
import csv
import glob
import os
import sys

FAMILY = ("conv_emu_kernel", "conv_wsb_kernel", "conv_wsb16_kernel", "conv_wst16_kernel", "conv_gs16_kernel",
          "conv_gsw16_kernel", "k_rb_pair",
          "conv_gemm_kernel", "conv_tiny", "k_conv2d_")  # conv_tiny(_rows)_kernel, k_conv2d_small / _h16


def dispatches(d, tag):
    """[(kernel, {counter: value})] of every dispatch of one pass, in dispatch order."""
    f = glob.glob(os.path.join(d, f"pmc_{tag}", "**", "*counter_collection.csv"), recursive=True)[0]
    by = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        by.setdefault(k, [r["Kernel_Name"], {}])[1][r["Counter_Name"]] = float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def per_launch(d, tag, n):
    """Counter dicts of the last n conv-family launches (split-K combines folded into their contraction)."""
    out = []
    for name, cnt in dispatches(d, tag):
        if any(f in name for f in FAMILY):
            out.append(dict(cnt))
        elif "splitk_reduce" in name and out:
            for k, v in cnt.items():
                if k != "GRBM_GUI_ACTIVE":
                    out[-1][k] = out[-1].get(k, 0.0) + v
    return out[-n:]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dump = [r for r in csv.reader(open(os.path.join(d, "convdump_FETCH_SIZE.csv")))]
    n = len(dump)
    fe = per_launch(d, "FETCH_SIZE", n)
    wr = per_launch(d, "WRITE_SIZE", n)
    sq = per_launch(d, "SQ_VALU_MFMA_BUSY_CYCLES", n)
    assert len(fe) == len(wr) == len(sq) == n, (len(fe), len(wr), len(sq), n)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0])
    for i, r in enumerate(dump):
        key = tuple(map(int, r[:7]))
        a = agg[key]
        a[0] += 1
        a[1] += float(r[7])
        a[2] += float(r[8])
        a[3] += float(r[9])
        a[4] += 2.0 * fe[i].get("FETCH_SIZE", 0.0) * 1024 + wr[i].get("WRITE_SIZE", 0.0) * 1024
        a[5] += sq[i].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[6] += sq[i].get("GRBM_GUI_ACTIVE", 0.0) / 8.0 * 1024
    tot = [sum(v[j] for v in agg.values()) for j in range(7)]
    print(f"{n} contraction launches: {tot[1]:.2f} ms, {tot[2] / 1e9:.1f} GFLOP ({tot[2] / tot[1] / 1e9:.1f} TF/s), "
          f"algorithmic {tot[3] / 1e9:.2f} GB, measured HBM {tot[4] / 1e9:.2f} GB (x{tot[4] / tot[3]:.2f}), "
          f"MFMA busy {100 * tot[5] / max(1.0, tot[6]):.1f} %")
    print(" 2d       M     N     C taps   b ks   n     ms     TF   alg_MB  hbm_MB  ratio  mfma%")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k[0]:3d} {k[1]:7d} {k[2]:5d} {k[3]:5d} {k[4]:4d} {k[5]:3d} {k[6]:2d} {v[0]:3d} {v[1]:6.3f} "
              f"{v[2] / v[1] / 1e9:6.1f} {v[3] / 1e6:8.1f} {v[4] / 1e6:7.1f} {v[4] / v[3]:6.2f} "
              f"{100 * v[5] / max(1.0, v[6]):6.1f}")


if __name__ == "__main__":
    main()
