"""Turn the rocprofv3 --pmc passes of scripts/gpu_pmc.sh into the traffic
profile bench.py quotes (profiles/pmc_<nx>x<ny>_fuse<K>.json).

  python3 scripts/pmc_profile.py <pmc dir> <out json> [nx ny fuse [cal cells, cal steps [engine]]]

engine float32 (default): k_fused<float, false, false, false, false, 1, false>,
4-byte lanes.  engine float64: k_fused<double, true, false, false, false, 1,
false>, whose forcing, geometry, state and output planes are 8-byte lanes and
whose window slots are 4-byte lanes; each counter is corrected per lane width,
weighted by the algorithmic bytes of each width (bench.bytes_model).

* k_fused passes: <dir>/p*/run_counter_collection.csv (one counter set each).
* Calibration passes: <dir>/cal_fetch, <dir>/cal_write (tools/hbm_mix ... cal):
  streaming kernels with known bytes per dispatch give the FETCH_SIZE and
  WRITE_SIZE scale for 4-byte lanes, the width k_fused uses.  The guide's
  gfx950 FETCH_SIZE x2 is calibrated for 16-byte lanes only
  (MI355X_MICROARCH.md, HBM/rocprofv3 section); this file records both.
* kernel_code_sha256: the sha256 of the measured kernel's own gfx950 machine
  code (k_fused<float, false, false, false, false, 1>, its kernel descriptor
  and the functions it calls; _native.kernel_code_sha256).  bench.py quotes
  `traffic` only when the running library's kernel has the same hash, so edits
  to other kernels leave the measurement valid.  code_object_sha256 (the whole
  .hip_fatbin) is recorded beside it.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "topoflow-glacier_amd"))
from topoflow_glacier import _native as nat  # noqa: E402

sys.path.insert(0, str(ROOT))
from bench import launch_bytes_per_cell  # noqa: E402  


def per_dispatch(paths, match):
    """{counter: mean value per dispatch} over kernels whose name contains `match`."""
    vals = defaultdict(list)
    for f in paths:
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if match not in row["Kernel_Name"]:
                continue
            per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for c, d in per.items():
            vals[c] += [d[k] for k in sorted(d, key=int)]
    return {c: sum(v) / len(v) for c, v in vals.items() if v}


def calibration(d: Path, cells: int, steps: int):
    """Counter KiB x 1024 / known bytes for each calibration kernel (first
    dispatch is the warm-up; all dispatches move the same bytes)."""
    kernels = {  # tools/hbm_mix.hip k_mix<R, W, V, NT>
        "read only 4 B/lane": ("k_mix<7, 0, 1, false,", "FETCH_SIZE", 7),
        "read only 16 B/lane": ("k_mix<7, 0, 4, false,", "FETCH_SIZE", 7),
        "read only 8 B/lane": ("k_mix<7, 0, 2, false,", "FETCH_SIZE", 7),
        "write only 8 B/lane nt": ("k_mix<0, 7, 2, true,", "WRITE_SIZE", 7),
        "write only 4 B/lane": ("k_mix<0, 7, 1, false,", "WRITE_SIZE", 7),
        "write only 4 B/lane nt": ("k_mix<0, 7, 1, true,", "WRITE_SIZE", 7),
        "k_fused mix reads 4 B/lane nt": ("k_mix<6, 7, 1, true,", "FETCH_SIZE", 6),
        "k_fused mix writes 4 B/lane nt": ("k_mix<6, 7, 1, true,", "WRITE_SIZE", 7),
    }
    out = {}
    for name, (kern, counter, planes) in kernels.items():
        sub = "cal_fetch" if counter == "FETCH_SIZE" else "cal_write"
        v = per_dispatch(glob.glob(str(d / sub / "run_counter_collection.csv")), kern).get(counter)
        if v is None:
            continue
        known = cells * steps * 4 * planes
        out[name] = {"counter": counter, "counter_bytes": v * 1024, "known_bytes": known,
                     "counter_over_known": v * 1024 / known}
    return out


KERNELS = {  # engine -> (rocprofv3 kernel-name match, _native symbol prefix, description)
    "float32": ("k_fused<float, false, false", "BENCH_KERNEL", "k_fused<float,false,false,false,false,1,false,false> (fp32 engine, clean form"),
    "float64": ("k_fused<double, true, false, false, false", "BENCH_KERNEL_F64",
                "k_fused<double,true,false,false,false,1,false,false> (fp64 engine"),
    "float32_flux64": ("k_fused<float, false, false", "BENCH_KERNEL_PREC",
                       "k_fused<float,false,false,false,false,1,false,true> (fp32 engine, fp64-flux form"),
}


def scale_of(cal, name, default):
    return 1.0 / cal[name]["counter_over_known"] if name in cal else default


def main():
    d, out = Path(sys.argv[1]), Path(sys.argv[2])
    nx, ny, fuse = (int(x) for x in sys.argv[3:6]) if len(sys.argv) > 5 else (8192, 8192, 96)
    engine = sys.argv[8] if len(sys.argv) > 8 else "float32"
    match, sym, desc = KERNELS[engine]
    raw = per_dispatch(sorted(glob.glob(str(d / "p*" / "run_counter_collection.csv"))), match)
    cal = calibration(d, cells=int(sys.argv[6]) if len(sys.argv) > 6 else 67108864,
                      steps=int(sys.argv[7]) if len(sys.argv) > 7 else 8)
    rd4 = scale_of(cal, "read only 4 B/lane", 2.0)
    wr4 = scale_of(cal, "write only 4 B/lane nt", 1.0)
    if engine.startswith("float32"):  # the fp64-flux form moves the fp32 form's bytes
        rd_scale, wr_scale = rd4, wr4
        elem = 4
    else:
        # bytes by lane width per cell and launch (bench.bytes_model, elem 8):
        # reads: forcing 5x8 per step + geometry 7x8 + state 7x8 (8 B lanes),
        # window slot 4 per step (4 B); writes: outputs 6x8 per step + state
        # 7x8 (8 B), window slot 4 per step (4 B)
        elem = 8
        rd8, wr8 = scale_of(cal, "read only 8 B/lane", rd4), scale_of(cal, "write only 8 B/lane nt", wr4)
        r8, r4 = 40 * fuse + 56 + 56, 4 * fuse
        w8, w4 = 48 * fuse + 56, 4 * fuse
        rd_scale = (r8 + r4) / (r8 / rd8 + r4 / rd4)
        wr_scale = (w8 + w4) / (w8 / wr8 + w4 / wr4)
    rd = raw["FETCH_SIZE"] * 1024 * rd_scale
    wr = raw["WRITE_SIZE"] * 1024 * wr_scale
    alg = nx * ny * launch_bytes_per_cell(fuse, elem)
    symbol = getattr(nat, sym)
    res = {
        "kernel": f"{desc}, {fuse} steps fused) at {nx}x{ny}",
        "engine": engine,
        "command": "bash scripts/gpu_pmc.sh (rocprofv3 --pmc <pass> -- python3 bench.py ...; one counter set per pass; "
                   "calibration: rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- tools/hbm_mix 67108864 8 2048 0 cal); "
                   "python3 scripts/pmc_profile.py",
        "kernel_symbol": symbol,
        "kernel_code_sha256": nat.kernel_code_sha256(symbol),
        "code_object_sha256": nat.code_object_sha256(),
        "correction": {
            "read_scale": rd_scale, "write_scale": wr_scale,
            "source": ("measured on the same box: tools/hbm_mix cal kernels with known bytes per dispatch at 4, 8 "
                       "and 16 B lanes (counter_over_known below); the read and write scales are the inverse of the "
                       "measured ratios at the kernel's lane widths"
                       + ("" if engine == "float32" else "; fp64 engine: the 8 B and 4 B lane scales weighted by "
                          "the algorithmic bytes of each width"))
                      if cal else "not measured in this run: the defaults, FETCH_SIZE x 2 (MI355X_MICROARCH.md, gfx950) "
                                  "and WRITE_SIZE x 1",
            "calibration": cal,
        },
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (rd + wr) / alg,
        "raw_counters_mean_per_dispatch": raw,
    }
    waves = raw.get("SQ_WAVES")
    if waves:
        cells_per_lane = nx * ny / (waves * 64)
        res["per_wave_step"] = {k: v / (waves * fuse * cells_per_lane) for k, v in raw.items()
                                if k.startswith("SQ_") and k != "SQ_WAVES"}
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch",
                                          "traffic_over_algorithmic", "kernel_code_sha256")}))
    print(json.dumps(cal, indent=1))


if __name__ == "__main__":
    main()
