"""Summarise an RVCX_PROF_DUMP csv (one line per conv launch: 2d,M,N,C_in,taps,batch,ksplit,ms,flops)."""
import collections
import csv
import sys


def main():
    rows = list(csv.reader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    tot_ms = tot_fl = 0.0
    for r in rows:
        key = tuple(map(int, r[:7]))
        ms, fl = float(r[7]), float(r[8])
        agg[key][0] += 1
        agg[key][1] += ms
        agg[key][2] += fl
        tot_ms += ms
        tot_fl += fl
    print(f"total {tot_ms:.2f} ms  {tot_fl / 1e9:.1f} GFLOP  {tot_fl / tot_ms / 1e9:.1f} TFLOP/s  ({len(rows)} launches)")
    print("2d       M     N     C taps   b ks   n     ms     TF  cum%")
    cum = 0.0
    for k, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        cum += ms
        print(f"{k[0]:2d} {k[1]:7d} {k[2]:5d} {k[3]:5d} {k[4]:4d} {k[5]:3d} {k[6]:2d} {n:3d} {ms:6.3f} {fl / ms / 1e9:6.1f} "
              f"{100 * cum / tot_ms:5.1f}")


if __name__ == "__main__":
    main()
