"""Critical-path view of one C2 step from a rocprofv3 kernel-trace database: per stream, the busy time and the
span of each phase (high-pass, RMVPE, HuBERT, synthesizer) of step STEP (0-based, k_odd_ext marks a step start).
usage: python tools/timeline.py RUN.db [STEP] [-v] [--mark=KERNEL] (--mark: another kernel marks a step start, e.g.
k_reflect1d for a stand-alone RMVPE trace)"""
import sqlite3
import sys
from collections import defaultdict


def phase(name):
    n = name
    if "sos" in n or "odd_ext" in n or "filt_pad" in n:
        return "highpass"
    if "gru" in n or "conv2d_small" in n or "avgpool" in n or "nhwc" in n or "decode" in n or "stftmag" in n:
        return "rmvpe"
    if "gn_" in n:
        return "hubert"
    if "sine" in n or "conv_post" in n or "k_zp" in n or "k_gate" in n or "flip" in n or "softmax_rel" in n:
        return "synth"
    return "other"


def main():
    db, step = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 1
    mark = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--mark=")), "k_odd_ext")
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    starts = [r[1] for r in rows if mark in r[0]]
    t0 = starts[step]
    t1 = starts[step + 1] if step + 1 < len(starts) else max(r[2] for r in rows)
    sel = [r for r in rows if t0 <= r[1] < t1]
    print(f"step {step}: wall {(max(r[2] for r in sel) - t0) / 1e6:.3f} ms, {len(sel)} kernels")
    by_q = defaultdict(list)
    for r in sel:
        by_q[r[4]].append(r)
    for q, rs in by_q.items():
        busy = sum(r[2] - r[1] for r in rs) / 1e6
        print(f"  queue {q}: {len(rs)} kernels, busy {busy:.3f} ms, span {(rs[0][1] - t0) / 1e6:.3f} .. "
              f"{(rs[-1][2] - t0) / 1e6:.3f} ms")
        # contiguous segments of big-name groups
        segs = []
        for r in rs:
            short = r[0].split("(")[0].replace("void ", "").replace("rvcx::", "").replace("(anonymous namespace)::", "")
            short = short.split("<")[0] + ("<" + r[0].split("<")[1].split(">")[0] + ">" if "<" in r[0] else "")
            segs.append((short[:60], (r[1] - t0) / 1e6, (r[2] - r[1]) / 1e3))
        if "-v" in sys.argv:
            for s in segs:
                print(f"     {s[1]:8.3f} ms  {s[2]:8.1f} us  {s[0]}")


if __name__ == "__main__":
    main()
