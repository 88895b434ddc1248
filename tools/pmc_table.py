"""Print per-kernel averages of every counter in gpurun_out/pmc_<tag>/ (tools/pmc_sq.sh)."""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}", "**", "*counter_collection.csv"),
                   recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("kmhg::", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}")
