"""Where the fp16 builds' headline time goes against bf16: per build, from one
rocprofv3 --pmc GRBM_GUI_ACTIVE pass over tools/headline.py --dtype X (kernels serialised by the
profiler), the kernel time (sum of dispatch durations), the shader cycles (GRBM_GUI_ACTIVE / 8 XCDs)
and their quotient, the effective clock; split into GEMM, attention and the rest.
  python tools/fp16_clock.py gpurun_out/r05_fp/bf16 gpurun_out/r05_fp/fp16 gpurun_out/r05_fp/fp16_precise"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def klass(name):
    n = name.split("(")[0]
    if "gemm" in n:
        return "gemm"
    if "attn" in n:
        return "attention"
    return "other"


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    cyc, dur = defaultdict(float), defaultdict(float)
    seen = {}
    for row in csv.DictReader(open(f)):
        k = klass(row["Kernel_Name"])
        did = row["Dispatch_Id"]
        cyc[k] += float(row["Counter_Value"]) / 8.0
        if did not in seen:
            seen[did] = 1
            dur[k] += (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-9
    out = {}
    for k in sorted(cyc):
        out[k] = {"kernel_s": round(dur[k], 5), "cycles_G": round(cyc[k] / 1e9, 4),
                  "clock_GHz": round(cyc[k] / dur[k] / 1e9, 3) if dur[k] else None}
    tc, td = sum(cyc.values()), sum(dur.values())
    out["all"] = {"kernel_s": round(td, 5), "cycles_G": round(tc / 1e9, 4), "clock_GHz": round(tc / td / 1e9, 3)}
    return out


res = {os.path.basename(d.rstrip("/")): load(d) for d in sys.argv[1:]}
base = res.get("bf16")
if base:
    for name, r in res.items():
        a, b = r["all"], base["all"]
        r["vs_bf16"] = {"time": round(a["kernel_s"] / b["kernel_s"], 4), "cycles": round(a["cycles_G"] / b["cycles_G"], 4),
                        "clock": round(a["clock_GHz"] / b["clock_GHz"], 4)}
print(json.dumps(res, indent=1))
