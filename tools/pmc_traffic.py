"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/rNN_traffic.json]

Each directory holds one `--pmc` pass (`run_counter_collection.csv`) of the same command
(tools/traffic.sh runs `bench.py` twice, once per counter: the TCC slots cannot hold both).
Corrections follow MI355X_MICROARCH.md "HBM [CDNA4]": the counters are in KiB, and on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads, so it is doubled.
WRITE_SIZE is exact for 16-B-per-lane stores, which is how every kernel here stores.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short_name(k: str) -> str:
    k = re.sub(r"\(.*", "", k)
    k = re.sub(r"^void ", "", k)
    return k.split("<")[0].split("::")[-1] if "<" in k else k.split("::")[-1]


def per_kernel(d: str, counter: str):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    with open(f[0]) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                acc[short_name(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--cmd", default="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline")
    a = ap.parse_args()
    fe = per_kernel(a.fetch_dir, "FETCH_SIZE")
    wr = per_kernel(a.write_dir, "WRITE_SIZE")
    res = {"command": a.cmd, "correction": "FETCH_SIZE x2 (gfx950 half-count), counters in KiB",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe.get(k, [0])) / max(1, len(fe.get(k, [])))
        w = sum(wr.get(k, [0])) / max(1, len(wr.get(k, [])))
        res["kernels"][k] = {"launches": len(fe.get(k, [])), "fetch_bytes": 2.0 * f, "write_bytes": w,
                             "hbm_bytes_per_launch": 2.0 * f + w}
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")
    for k, v in res["kernels"].items():
        if "vc" in k or "attn" in k or "gemm" in k or "layernorm" in k or "gather" in k or "im2col" in k or "cls" in k:
            print(f"{k:40s} n={v['launches']:4d} fetch {v['fetch_bytes'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:8.1f} MB")


if __name__ == "__main__":
    main()
