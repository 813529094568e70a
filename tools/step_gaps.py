"""Idle time inside the steady-state steps of a rocprofv3 --kernel-trace directory: the steps are delimited
by a marker kernel launched once per step (default: the AdamW update), and for the last N complete steps the
script reports the wall time per step, the busy union (time with >= 1 kernel running), and the idle gaps.
  python tools/step_gaps.py <trace dir> [--marker adamw_kernel] [--steps 10]"""
import argparse
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("d")
ap.add_argument("--marker", default="adamw_kernel")
ap.add_argument("--steps", type=int, default=10)
a = ap.parse_args()
f = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
marks = [e for s, e, k in rows if a.marker in k]
if len(marks) < 2:
    raise SystemExit(f"fewer than 2 '{a.marker}' dispatches")
marks = marks[-(a.steps + 1):]
t0, t1 = marks[0], marks[-1]
win = [(max(s, t0), min(e, t1)) for s, e, _ in rows if e > t0 and s < t1]
win.sort()
union, gaps, cur_s, cur_e = 0, [], None, None
for s, e in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
            gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
n = len(marks) - 1
span = t1 - t0
gaps.sort()
print(f"steps {n}: {span / n / 1e6:.3f} ms per step, busy union {union / n / 1e6:.3f} ms ({union / span:.3f}), "
      f"idle {(span - union) / n / 1e6:.3f} ms in {len(gaps) / n:.1f} gaps per step; "
      f"gap median {gaps[len(gaps) // 2] / 1e3 if gaps else 0:.1f} us, p90 {gaps[int(len(gaps) * 0.9)] / 1e3 if gaps else 0:.1f} us, "
      f"max {gaps[-1] / 1e3 if gaps else 0:.1f} us")
