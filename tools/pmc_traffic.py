"""HBM bytes per conv-GEMM launch from the two PMC passes of tools/pmc_traffic.sh.

FETCH_SIZE and WRITE_SIZE are in KB per dispatch (rocprofv3 derived counters). On gfx950 FETCH_SIZE reports
half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section), so it is doubled;
WRITE_SIZE is taken as is. The bench runs warm-up + 1 timed step + 1 event pass (inline: the timed step
carries the events), so each kernel of the step appears `steps` times; per-launch numbers are averages.
usage: python tools/pmc_traffic.py gpurun_out [kernel-substring,...] > profiles/pmc_traffic.json
Default family: the conv dispatches bench.py's roofline counts (conv_emu / conv_wsb / k_rb_pair / conv_gemm /
conv_tiny / conv_tiny_rows / k_conv2d_small / k_conv2d_h16);
the split-K reduce kernels' bytes are added to the family's total, launches count the conv kernels only.
The record carries the source-tree hash (rvcx.provenance) so bench.py can tell whether it applies.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "retrieval-based-voice-conversion-mlx_amd"))


def load(d, counter):
    f = glob.glob(os.path.join(d, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    out = collections.defaultdict(list)
    for r in rows:
        if r["Counter_Name"] == counter:
            out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    keys = (sys.argv[2] if len(sys.argv) > 2 else
            "conv_emu_kernel,conv_wsb_kernel,conv_wsb16_kernel,conv_wst16_kernel,conv_gs16_kernel,conv_gsw16_kernel,k_rb_pair,"
            "conv_gemm_kernel,conv_tiny,k_conv2d_").split(",")
    key = ",".join(keys)
    fam = lambda k: any(s in k for s in keys)  # noqa: E731
    bytes_fam = lambda k: fam(k) or "splitk_reduce" in k  # noqa: E731
    fe, wr = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    tot_f = sum(sum(v) for k, v in fe.items() if bytes_fam(k))
    tot_w = sum(sum(v) for k, v in wr.items() if bytes_fam(k))
    n = sum(len(v) for k, v in fe.items() if fam(k))
    fetch = 2.0 * tot_f * 1024 / max(1, n)
    write = tot_w * 1024 / max(1, n)
    rec = {"kernel": key, "launches": n, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write,
           "note": "FETCH_SIZE doubled (gfx950 16-B/lane reads), WRITE_SIZE as is; KB counters x 1024"}
    # per kernel family (the names bench.py's roofline.dominant uses, rvcx_profile_kind_name): HBM bytes per launch of
    # the family's own kernels (its split-K combines are separate kernels, not attributed)
    famnames = {"conv_wsb16_kernel": "conv_wsb16_kernel", "conv_wst16_kernel": "conv_wst16_kernel",
                "conv_wsb_kernel": "conv_wsb_kernel<",
                "conv_gs16_kernel": "conv_gs16_kernel", "conv_gsw16_kernel": "conv_gsw16_kernel", "k_rb_pair": "k_rb_pair",
                "k_conv2d_h16/k_conv2d_small": "k_conv2d_", "conv_emu_kernel": "conv_emu_kernel",
                "conv_gemm_kernel": "conv_gemm_kernel", "conv_tiny_kernel": "conv_tiny"}
    rec["families"] = {}
    for fname, sub in famnames.items():
        fk = [k for k in fe if sub in k]
        nl = sum(len(fe[k]) for k in fk)
        if nl:
            b = sum(2.0 * sum(fe[k]) + sum(wr.get(k, [])) for k in fk) * 1024
            rec["families"][fname] = {"launches": nl, "hbm_bytes_per_launch": b / nl}
    all_f = sum(sum(v) for v in fe.values()) * 2 * 1024
    all_w = sum(sum(v) for v in wr.values()) * 1024
    rec["all_kernels_bytes"] = all_f + all_w
    # per step: the conv family's measured HBM bytes (each kernel ran once per pipeline call: warm-up + the timed
    # step) against the algorithmic bytes of the timed step's launches (operands read once, result written once:
    # the RVCX_PROF_DUMP csv of the same pass, last column)
    dump = glob.glob(os.path.join(d, "convdump_FETCH_SIZE.csv"))
    if dump:
        lines = [r for r in open(dump[0]) if r.strip()]
        calls = max(1, round(n / max(1, len(lines))))
        # columns: 2d, M, N, C_in, taps, batch, ksplit, ms, flops, algorithmic bytes, the launch's MFMA ceiling (TF)
        alg = sum(float(r.split(",")[9]) for r in lines)
        rec["step_hbm_bytes"] = (2.0 * tot_f + tot_w) * 1024 / calls
        rec["step_alg_bytes"] = alg
        rec["step_ratio"] = rec["step_hbm_bytes"] / alg if alg > 0 else None
    from rvcx.provenance import source_tree_hash

    rec["tree"] = source_tree_hash()
    rec["file"] = d
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
