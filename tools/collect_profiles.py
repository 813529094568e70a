"""Copy one profiling session (tools/profile_round.sh -> gpurun_out/<TAG>/) into profiles/ as the
files bench.py cites, each stamped with the build (vclip_amd.build.source_hash) the bench line of
that session reports:

  profiles/<TAG>_bench.json          the bench JSON line
  profiles/<TAG>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary of the same command
  profiles/<TAG>_traffic.json        HBM bytes per launch: FETCH_SIZE x2 (gfx950 half-count,
                                     MI355X_MICROARCH.md "HBM") + WRITE_SIZE, counters in KiB
  profiles/<TAG>_pmc.json            per-launch averages of the SQ / GRBM counter groups

  python tools/collect_profiles.py r02_v8
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short_name(k: str) -> str:
    """Kernel name with its template arguments (they tell the bf16 / fp16 builds and the GEMM
    epilogues apart), without the namespace and the parameter list."""
    k = re.sub(r"^void ", "", k)
    k = k.split("(")[0]
    return re.sub(r"^vc::", "", k).strip()


def per_kernel(d):
    """{kernel: {counter: mean per dispatch}} from one rocprofv3 --pmc output directory."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    per = defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f[0])):
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] += float(row["Counter_Value"])
        names[row["Dispatch_Id"]] = short_name(row["Kernel_Name"])
    acc = defaultdict(lambda: defaultdict(list))
    for (disp, c), v in per.items():
        acc[names[disp]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"launches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


def bench_mode(command: str) -> str:
    """bench.py's --mode in a command line ("fwd" when absent): the workload a summary measured."""
    m = re.search(r"--mode[= ](\w+)", command)
    return m.group(1) if m else "fwd"


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    if "--dst" in sys.argv:  # on the GPU box: the session's own summaries, for its bench line (VCLIP_PROFILES)
        dst = sys.argv[sys.argv.index("--dst") + 1]
        os.makedirs(dst, exist_ok=True)
    bf = os.path.join(src, "bench.json")
    bench = json.loads(open(bf).read()) if os.path.exists(bf) else None
    if bench is not None:
        build = bench.get("build")
    else:  # a session without its bench line (NO_BENCH=1): the tree's own build
        sys.path.insert(0, ROOT)
        from vclip_amd.build import source_hash
        build = source_hash()
    cf = os.path.join(src, "pmc_command.txt")
    if not os.path.exists(cf):
        raise SystemExit(f"{cf} missing: profile with tools/profile_round.sh, which records the command")
    command = open(cf).read().strip()
    mode = bench_mode(command)
    if bench is not None:
        with open(os.path.join(dst, f"{tag}_bench.json"), "w") as f:
            json.dump(bench, f, indent=1)
    tl = os.path.join(src, "timeline.json")
    if os.path.exists(tl):
        d = json.load(open(tl))
        with open(os.path.join(dst, f"{tag}_timeline.json"), "w") as f:
            json.dump({"build": build, "mode": mode, "note": "the concurrent headline (tools/headline.py: "
                       "its streams, graph replay), rocprofv3 --kernel-trace", **d}, f, indent=1)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    hstats = glob.glob(os.path.join(src, "htrace", "**", "*kernel_stats.csv"), recursive=True)
    if hstats:
        shutil.copy(hstats[0], os.path.join(dst, f"{tag}_headline_kernel_stats.csv"))
    fe, wr = per_kernel(os.path.join(src, "pmc_FETCH_SIZE")), per_kernel(os.path.join(src, "pmc_WRITE_SIZE"))
    if fe and wr:
        out = {"build": build, "mode": mode, "command": command,
               "correction": "FETCH_SIZE x2 (gfx950 half-count), counters in KiB", "kernels": {}}
        for k in sorted(set(fe) | set(wr)):
            fb = 2.0 * 1024.0 * fe.get(k, {}).get("FETCH_SIZE", 0.0)
            wb = 1024.0 * wr.get(k, {}).get("WRITE_SIZE", 0.0)
            out["kernels"][k] = {"launches": fe.get(k, {}).get("launches", 0), "fetch_bytes": fb, "write_bytes": wb,
                                 "hbm_bytes_per_launch": fb + wb}
        with open(os.path.join(dst, f"{tag}_traffic.json"), "w") as f:
            json.dump(out, f, indent=1)
    groups = sorted(glob.glob(os.path.join(src, "pmc_g*")))
    groups = [g for g in groups if os.path.isdir(g)]
    if groups:
        merged = defaultdict(dict)
        for g in groups:
            for k, cs in per_kernel(g).items():
                merged[k].update(cs)
        with open(os.path.join(dst, f"{tag}_pmc.json"), "w") as f:
            json.dump({"build": build, "mode": mode, "command": command,
                       "note": "per-dispatch means; SQ_* cycle counters in quad-cycles except "
                               "SQ_VALU_MFMA_BUSY_CYCLES; GRBM_GUI_ACTIVE summed over 8 XCDs",
                       "kernels": merged}, f, indent=1)
    print(f"collected {tag} (build {build}, mode {mode}) into profiles/")


if __name__ == "__main__":
    main()
