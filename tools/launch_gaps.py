"""Host launch time vs kernel start for the main queue's idle gaps of one C2 step, from rocprofv3 CSV output
(--kernel-trace --hip-trace --output-format csv). usage: python tools/launch_gaps.py DIR [STEP]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
step = int(sys.argv[2]) if len(sys.argv) > 2 else 2
kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
hf = glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0]
ks = list(csv.DictReader(open(kf)))
hs = list(csv.DictReader(open(hf)))
print("kernel cols:", list(ks[0].keys())[:20])
print("hip cols:", list(hs[0].keys())[:20])
api = {}
names = defaultdict(int)
for h in hs:
    names[h.get("Function", h.get("Kind", ""))] += 1
    if "Launch" in h.get("Function", "") or "launch" in h.get("Function", "").lower():
        api[h["Correlation_Id"]] = (int(h["Start_Timestamp"]), int(h["End_Timestamp"]), h["Function"])
print("top hip calls:", sorted(names.items(), key=lambda kv: -kv[1])[:12])
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in ks if "k_odd_ext" in r["Kernel_Name"]]
t0, t1 = starts[step], starts[step + 1]
sel = [r for r in ks if t0 <= int(r["Start_Timestamp"]) < t1]
q1 = min(r["Queue_Id"] for r in sel)
qs = [r for r in sel if r["Queue_Id"] == q1]
late = 0
for a, b in zip(qs, qs[1:]):
    gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if gap > 15:
        c = api.get(b["Correlation_Id"])
        rel = (c[1] - int(a["End_Timestamp"])) / 1e3 if c else None
        late += rel is not None and rel > 0
        print(f"{(int(a['End_Timestamp']) - t0) / 1e6:7.3f} ms gap {gap:6.1f} us; launch API of next returned "
              f"{rel if rel is None else round(rel, 1)} us after the previous kernel ended; next {b['Kernel_Name'][:50]}")
# host issue time of the step: first to last launch API call
ls = [api[r["Correlation_Id"]] for r in sel if r["Correlation_Id"] in api]
if ls:
    print(f"host launches of the step span {(max(x[1] for x in ls) - min(x[0] for x in ls)) / 1e6:.3f} ms "
          f"for {len(ls)} kernels; GPU step {(t1 - t0) / 1e6:.3f} ms; gaps where the launch was late: {late}")
    dur = sorted((x[1] - x[0]) / 1e3 for x in ls)
    print(f"launch API duration p50 {dur[len(dur) // 2]:.1f} us p90 {dur[int(len(dur) * 0.9)]:.1f} us max {dur[-1]:.1f}")
