"""Summarise a rocprofv3 --kernel-trace run: per-kernel calls and mean
duration, and every dispatch of the bench's k_fused launch shape, so the
profile's average can be set beside bench.py's HIP-event launch times.

  python3 scripts/trace_summary.py <trace dir> <bench log> <out json>
"""
import csv
import glob
import json
import sys
from collections import defaultdict

d, bench_log, out = sys.argv[1:4]
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = defaultdict(list)


def short(name):
    """kernel name without its parameter list: 'k_fused<float, false, false, false, 1>'"""
    name = name.replace("void ", "", 1).replace("(anonymous namespace)::", "").replace("tfg_kern::", "")
    return name.split("(")[0][:120]


for r in rows:
    per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
bench = None
for line in open(bench_log):
    if line.startswith("{"):
        bench = json.loads(line)
fused = [(k, v) for k, v in per.items() if "k_fused<float, false, false" in k]
res = {
    "kernels": {short(k): {"calls": len(v), "mean_ms": sum(v) / len(v)} for k, v in
                sorted(per.items(), key=lambda kv: -sum(kv[1]))},
    "k_fused_bench_shape_ms": {short(k): v for k, v in fused},
}
if bench:
    res["bench"] = {"value": bench["value"], "launches": bench.get("launches"),
                    "kernel_ms_per_launch": bench["roofline"]["kernel_ms_per_launch"]}
    if fused:
        v = fused[0][1]
        res["rocprof_mean_ms_over_bench_launches"] = sum(v) / len(v)
        res["agreement"] = (sum(v) / len(v)) / bench["roofline"]["kernel_ms_per_launch"]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in res if k != "kernels"}, indent=1))
