"""Summarise scripts/gpu_pmc_issue.sh: per wave and cell-step instruction
counts of the fused kernel for each engine, and the share of SIMD time the
vector pipe was issuing (SQ_ACTIVE_INST_VALU, quad-cycles summed over waves,
against GRBM_GUI_ACTIVE x 1024 SIMDs; MI355X_MICROARCH.md: SQ cycle counters
count quad-cycles).
  python3 scripts/issue_summary.py <dir> [f32_fuse f64_fuse]"""
import csv
import glob
import json
import sys
from collections import defaultdict

SIMDS = 256 * 4
d = sys.argv[1]
res = {}
# the timed instances only (the NaN-safe and other forms have other template arguments); the runs carry no
# parity or drop-in legs, so every dispatch of these is a whole `fuse`-step launch
F32_FUSE, F64_FUSE = (int(a) for a in (sys.argv[2:4] if len(sys.argv) > 3 else (128, 192)))
for name, kern, cells, fuse in (("f32", "k_fused<float, false, false, false, false, 1, false, false>", 8192 * 8192, F32_FUSE),
                                ("f32_flux_f64", "k_fused<float, false, false, false, false, 1, false, true>", 8192 * 8192,
                                 F32_FUSE),
                                ("f64", "k_fused<double, true, false, false, false, 1, false, false>", 4096 * 4096, F64_FUSE)):
    raw = defaultdict(list)
    for f in sorted(glob.glob(f"{d}/{name}/p*/run_counter_collection.csv")):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if kern in row["Kernel_Name"]:
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for c, dd in per.items():
            raw[c] += list(dd.values())
    m = {c: sum(v) / len(v) for c, v in raw.items() if v}
    if "SQ_WAVES" not in m:
        continue
    wave_steps = m["SQ_WAVES"] * fuse * (cells / (m["SQ_WAVES"] * 64))  # waves x steps x cells per lane
    per = {c: v / wave_steps for c, v in m.items() if c.startswith("SQ_") and c != "SQ_WAVES"}
    out = {"kernel": kern, "grid_cells": cells, "fuse": fuse, "per_wave_cell_step": per, "raw_mean_per_dispatch": m}
    if "GRBM_GUI_ACTIVE" in m and "SQ_ACTIVE_INST_VALU" in m:
        out["valu_issue_share"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * m["GRBM_GUI_ACTIVE"])
    res[name] = out
print(json.dumps(res, indent=1))
