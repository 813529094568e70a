"""Per-kernel summary and stream overlap of one rocprofv3 --kernel-trace directory (CSV output):

  python tools/trace_timeline.py gpurun_out/<TAG>/trace > timeline.json

Per kernel (the name with its template arguments, tools/collect_profiles.short_name): launches, mean
and median dispatch duration in us (under two concurrent streams a duration includes time shared with
the other stream's kernels), and its share of the summed durations.  Whole trace: the wall span from
the first to the last dispatch, the union of busy intervals (time with at least one kernel running),
the summed durations, and their ratio (the mean number of kernels in flight while any runs)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from collect_profiles import short_name  # noqa: E402


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no *kernel_trace.csv under {d}")
    rows = []
    for r in csv.DictReader(open(f[0])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short_name(r["Kernel_Name"]),
                     r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    per = defaultdict(list)
    for s, e, k, _ in rows:
        per[k].append((e - s) / 1e3)
    total = sum(sum(v) for v in per.values())
    union = 0.0
    cur_s, cur_e = None, None
    for s, e, _, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0.0
    kern = {}
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        v2 = sorted(v)
        kern[k] = {"launches": len(v), "mean_us": round(sum(v) / len(v), 2), "median_us": round(v2[len(v2) // 2], 2),
                   "share_of_summed": round(sum(v) / total, 4) if total else None}
    queues = sorted({q for _, _, _, q in rows})
    print(json.dumps({"dispatches": len(rows), "queues": queues, "span_us": round(span, 1),
                      "busy_union_us": round(union / 1e3, 1), "summed_us": round(total, 1),
                      "mean_in_flight": round(total / (union / 1e3), 3) if union else None, "kernels": kern}, indent=1))


if __name__ == "__main__":
    main()
