"""Summarise rocprofv3 --pmc CSVs for the fused kernel (k_fused), per dispatch."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
match = sys.argv[2] if len(sys.argv) > 2 else "k_fused<float, false, false"
vals = defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(f)):
        if match not in row["Kernel_Name"]:
            continue
        per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    for c, d in per.items():
        vals[c] = [d[k] for k in sorted(d, key=int)]
out = {c: sum(v) / len(v) for c, v in vals.items() if v}
print(json.dumps(out, indent=1))
