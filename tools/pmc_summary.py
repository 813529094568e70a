"""Average per-dispatch PMC counter values of one kernel from rocprofv3 --pmc CSV output
directories (tools/pmc_attn.sh):  python tools/pmc_summary.py <kernel-substring> <dir>..."""
import csv
import glob
import sys
from collections import defaultdict

kern = sys.argv[1]
vals = defaultdict(list)
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
for c, v in sorted(vals.items()):
    print(f"{c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
