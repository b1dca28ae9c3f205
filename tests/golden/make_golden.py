"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

This script is test infrastructure.  It runs only in the build container, where
the read-only reference checkout lives at /root/reference; it is never run on a
GPU box, and nothing in the product imports it.  The reference needs four
offline import shims; they are written into a private
temporary directory at run time and never enter the repository.

Fixtures written (all small .npz, float64):

* ``cat3062920_265.npz`` -- the reference's own known-answer workflow
  (tests/integration_test.py:67-153): cat-3062920 parameters, forcing
  tests/data/sample-cat-3062920.csv filtered to 2013032000..2013033100 (265 rows).
  Holds the 7 BMI inputs fed per step, the 8 BMI outputs after each update,
  and internal diagnostics (Q_sum, fluxes, cold contents, albedo, clock scalars,
  mass-balance integrals).
* ``grid64.npz`` -- 64 independent single-catchment reference runs of 288 steps
  with per-cell elev/slope/aspect/initial depths and per-cell perturbed forcing.
  A grid cell of the MI355X engine is one of these runs, so this pins the
  elementwise generalisation of the reference's scalar branches.
* ``clock_windows.npz`` -- short runs across the 2013-11-03 DST end, the
  2014-03-09 DST start and the 2013/2014 year boundary (America/Los_Angeles).
* ``dt2.npz`` -- a dt = 2 h run (int dt, accepted by the reference loader).
* ``dt_quarter.npz`` -- a dt = 0.25 h run; the reference loader rejects float
  dt (config.py:15), so ONLY here the config class is widened to float.

* ``satterlund.npz`` -- SATTERLUND = True (the alternative vapour-pressure and
  emissivity formulas).
* ``params.npz`` -- non-default dust_atten / canopy_factor / cloud_factor.
* ``clock_<zone>.npz`` (phoenix, anchorage, denver, boise, chicago, new_york,
  honolulu) -- runs outside America/Los_Angeles across a US DST change, one
  interior point of every other zone the build's lat/lon table returns,
  carrying the zone name the timezonefinder stub returned.

Usage:  python3 tests/golden/make_golden.py   (takes ~1 minute)
        python3 tests/golden/make_golden.py --only satterlund,params,zones
"""

from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import textwrap
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference")

SHIMS = {
    "sitecustomize.py": """
        import datetime, sys, types
        if not hasattr(datetime, "UTC"):
            datetime.UTC = datetime.timezone.utc
        v = types.ModuleType("topoflow_glacier._version"); v.__version__ = "0.1.0+ref"
        sys.modules["topoflow_glacier._version"] = v
    """,
    "bmipy.py": """
        class Bmi:
            pass
    """,
    # timezonefinder's polygon data is not available offline.  The stub answers
    # what its polygons give for the points the fixtures use: the Pacific
    # Northwest box (every reference config), and one interior point per other
    # zone the build's table (physics/clock.py) can return: central Arizona
    # (34.0 N, 111.5 W: America/Phoenix, no DST), Wolverine Glacier, Alaska
    # (60.4 N, 148.9 W), Arapaho Glacier, Colorado (40.02 N, 105.65 W), the
    # Sawtooth Range, Idaho (44.1 N, 114.9 W), central Iowa (41.9 N, 93.1 W),
    # Mount Washington, New Hampshire (44.27 N, 71.3 W) and Mauna Kea, Hawaii
    # (19.82 N, 155.47 W).
    "timezonefinder.py": """
        POINTS = {(34.0, -111.5): "America/Phoenix", (60.4, -148.9): "America/Anchorage",
                  (40.02, -105.65): "America/Denver", (44.1, -114.9): "America/Boise",
                  (41.9, -93.1): "America/Chicago", (44.27, -71.3): "America/New_York",
                  (19.82, -155.47): "Pacific/Honolulu"}
        class TimezoneFinder:
            def timezone_at(self, lat=None, lng=None):
                if -125 <= lng <= -114 and 32 <= lat <= 49.5 and not (abs(lat - 44.1) < 0.01 and abs(lng + 114.9) < 0.01):
                    return "America/Los_Angeles"
                for (la, lo), zone in POINTS.items():
                    if abs(lat - la) < 0.01 and abs(lng - lo) < 0.01:
                        return zone
                return None
            def certain_timezone_at(self, lat=None, lng=None):
                return self.timezone_at(lat=lat, lng=lng)
    """,
}

BASE_CFG = {
    "site_prefix": "cat-3062920",
    "forcing_file": "data/sample-cat-3062920.csv",
    "dt": 1,
    "start_time": "2013032000",
    "end_time": "2013033100",
    "da": 11.418749923500716,
    "slope": 88.582729,
    "aspect": 242.8644693769529,
    "lon": -121.81418,
    "lat": 46.81953220,
    "elev": 2446.3922737596167,
    "h_active_layer": 0.125,
    "h0_snow": 5.0,
    "h0_ice": 2.0,
    "h0_swe": 0.25,
    "h0_iwe": 1.834,
    "T_rain_snow": 0.0,
}

IN_NAMES = [
    "land_surface_radiation~incoming~longwave__energy_flux",
    "land_surface_air__pressure",
    "atmosphere_air_water~vapor__relative_saturation",
    "atmosphere_water__liquid_equivalent_precipitation_rate",
    "land_surface_radiation~incoming~shortwave__energy_flux",
    "land_surface_air__temperature",
    "wind_speed_UV",
]
IN_SHORT = ["LW_in", "P_air", "Hum_sp", "P", "SW_in", "T_air", "uz"]
OUT_NAMES = [
    "snowpack__depth",
    "snowpack__liquid-equivalent_depth",
    "snowpack__melt_volume_flux",
    "glacier_ice__thickness",
    "glacier__liquid_equivalent_depth",
    "glacier_ice__melt_volume_flux",
    "land_surface_water__runoff_volume_flux",
    "atmosphere_bottom_air_water-vapor__relative_saturation",
]
OUT_SHORT = ["h_snow", "h_swe", "SM", "h_ice", "h_iwe", "IM", "M_total", "RH"]
INTERNAL = [
    "p0", "T_surf", "Q_sum", "Qn_SW", "Qn_LW", "Qh", "Qe", "W_p", "Eccs", "Ecci",
    "albedo", "n", "TSN_offset", "GMT_offset", "julian_day",
    "vol_P", "vol_PR", "vol_PS", "vol_SM", "vol_IM", "P_max",
]


# --------------------------------------------------------------------------
# Child-process side: runs with the shims and the reference on sys.path.
# --------------------------------------------------------------------------
def _child_main(job_path: str, out_path: str) -> None:
    import json

    import numpy as np
    import yaml

    job = json.loads(Path(job_path).read_text())
    if job.get("float_dt"):
        # Oracle-only widening of config.py:15 (dt: int) so a 15-minute step
        # can be generated.  Nothing else in the reference is touched.
        from topoflow_glacier.bmi import bmi_topoflow_glacier as btg
        from topoflow_glacier.bmi.config import TopoflowGlacierConfig

        class _FloatDtConfig(TopoflowGlacierConfig):
            dt: float

        btg.TopoflowGlacierConfig = _FloatDtConfig

    from topoflow_glacier import BmiTopoflowGlacier

    res = {}
    cells = job["cells"]
    nsteps = job["nsteps"]
    tmpd = Path(tempfile.mkdtemp())
    outs = np.zeros((len(OUT_SHORT), nsteps, len(cells)))
    ints = np.zeros((len(INTERNAL), nsteps, len(cells)))
    for c, cell in enumerate(cells):
        cfg = dict(BASE_CFG)
        cfg.update(cell["cfg"])
        cfile = tmpd / f"cfg{c}.yaml"
        cfile.write_text(yaml.dump(cfg))
        m = BmiTopoflowGlacier()
        m.initialize(str(cfile))
        forc = np.asarray(cell["forcing"], dtype=np.float64)  # [7][nsteps]
        for k in range(nsteps):
            for i, name in enumerate(IN_NAMES):
                m.set_value(name, np.array([forc[i, k]]))
            m.update()
            d = np.zeros(1)
            for j, name in enumerate(OUT_NAMES):
                outs[j, k, c] = m.get_value(name, d).item()
            for j, attr in enumerate(INTERNAL):
                ints[j, k, c] = float(np.asarray(getattr(m, attr)).reshape(-1)[0])
        m.finalize()
    np.savez(out_path, outs=outs, ints=ints)


# --------------------------------------------------------------------------
# Parent side: builds jobs (forcing, per-cell configs), runs children, saves.
# --------------------------------------------------------------------------
def _run_job(job: dict) -> dict:
    import json

    import numpy as np

    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        for name, src in SHIMS.items():
            (td / name).write_text(textwrap.dedent(src))
        jp, op = td / "job.json", td / "out.npz"
        jp.write_text(json.dumps(job))
        env = dict(os.environ)
        env["PYTHONPATH"] = f"{td}:{REF / 'src'}"
        env["PYTHONDONTWRITEBYTECODE"] = "1"
        env["TOPOFLOW_GLACIER_LOGFILEPATH"] = str(td / "ref.log")
        env["TOPOFLOW_GLACIER_LOGLEVEL"] = "ERROR"
        subprocess.run(
            [sys.executable, __file__, "--child", str(jp), str(op)], env=env, check=True, cwd=td
        )
        z = np.load(op)
        return {"outs": z["outs"].copy(), "ints": z["ints"].copy()}


def _csv_forcing():
    import numpy as np
    import pandas as pd

    df = pd.read_csv(HERE / "sample-cat-3062920.csv")
    df["Time"] = pd.to_datetime(df["Time"])
    return df, np


def _caller_units(df, np):
    """Unit conversions exactly as the reference caller applies them
    (tests/integration_test.py:93-115)."""
    K_to_C = -273.15
    P = df["RAINRATE"].values * 10 ** (-3)
    T = K_to_C + df["T2D"].values
    LW = df["LWDOWN"].values
    SW = df["SWDOWN"].values
    Pa = df["PSFC"].values
    q = df["Q2D"].values
    uz = (((df["U2D"]) ** 2 + (df["V2D"]) ** 2) ** 0.5).values
    # order = IN_SHORT = LW_in, P_air, Hum_sp, P, SW_in, T_air, uz
    return np.stack([LW, Pa, q, P, SW, T, uz]).astype(np.float64)


def build_cat3062920():
    import pandas as pd

    df, np = _csv_forcing()
    s = pd.to_datetime(BASE_CFG["start_time"], format="%Y%m%d%H")
    e = pd.to_datetime(BASE_CFG["end_time"], format="%Y%m%d%H")
    df = df[(df["Time"] >= s) & (df["Time"] <= e)].copy()
    forc = _caller_units(df, np)
    job = {"nsteps": forc.shape[1], "cells": [{"cfg": {}, "forcing": forc.tolist()}]}
    r = _run_job(job)
    return forc[:, :, None], r, [{}]


def _perturbed_cells(ncell: int, nsteps: int, seed: int, start_time: str, extra_cfg: dict | None = None):
    """Per-cell configs and per-cell perturbed forcing built from the CSV."""
    df, np = _csv_forcing()
    base = _caller_units(df, np)  # [7][288]
    reps = int(np.ceil(nsteps / base.shape[1]))
    base = np.tile(base, (1, reps))[:, :nsteps]
    rng = np.random.default_rng(seed)
    cells, forcs = [], []
    for c in range(ncell):
        cfg = {
            "elev": float(rng.uniform(1500.0, 3000.0)),
            "slope": float(rng.uniform(0.5, 100.0)),
            "aspect": float(rng.uniform(0.0, 360.0)),
            "h0_swe": float(0.25 * rng.uniform(0.8, 1.2)),
            "h0_iwe": float(1.834 * rng.uniform(0.8, 1.2)),
            "start_time": start_time,
        }
        cfg["h0_snow"] = cfg["h0_swe"] * 20.0 * float(rng.uniform(0.9, 1.1))
        cfg["h0_ice"] = cfg["h0_iwe"] * (1000.0 / 917.0) * float(rng.uniform(0.9, 1.1))
        if extra_cfg:
            cfg.update(extra_cfg)
        f = base.copy()
        f[5] = f[5] + rng.uniform(-6.0, 8.0)  # T_air offset (degC)
        f[5] = f[5] + rng.normal(0.0, 0.7, nsteps)
        pmul = [1.0, 30.0, 300.0, 3000.0][c % 4]  # exercise the 3-day >= 0.03 threshold
        f[3] = f[3] * pmul * rng.uniform(0.5, 1.5, nsteps)
        f[2] = f[2] * rng.uniform(0.8, 1.2)  # specific humidity
        f[1] = f[1] * rng.uniform(0.98, 1.02)  # surface pressure
        f[6] = f[6] * rng.uniform(0.0, 2.0, nsteps)  # wind
        # edge-case cells (fixed positions)
        if c == 0:  # no snow, no ice (integration_test.py:192-243 generalised)
            cfg.update(h0_snow=0.0, h0_ice=0.0, h0_swe=0.0, h0_iwe=0.0)
        if c == 1:  # bare ice from the start
            cfg.update(h0_snow=0.0, h0_swe=0.0)
        if c == 2:  # thin snow that melts out early -> IM switch-on
            cfg.update(h0_swe=0.003, h0_snow=0.06)
            f[5] = f[5] + 6.0
            f[3] = 0.0 * f[3]
        if c == 3:  # calm air (bot == 0 branch, bmi_topoflow_glacier.py:642-643)
            f[6][::5] = 0.0
        if c == 4:  # T_air exactly at the rain/snow threshold on some steps
            f[5][::7] = 0.0
        if c == 5:  # no ice, snow only
            cfg.update(h0_ice=0.0, h0_iwe=0.0)
        if c == 6:  # deep snow, heavy snowfall, cold
            f[5] = f[5] - 8.0
            f[3] = f[3] * 10.0
        if c == 7:  # near-flat cell
            cfg.update(slope=0.0, aspect=0.0)
        cells.append({"cfg": cfg, "forcing": f.tolist()})
        forcs.append(f)
    return cells, np.stack(forcs, axis=-1)  # [7][nsteps][ncell]


def build_grid64():
    nsteps = 288
    cells, forc = _perturbed_cells(64, nsteps, 20251001, "2013032000")
    r = _run_job({"nsteps": nsteps, "cells": cells})
    return forc, r, [c["cfg"] for c in cells]


def build_clock_windows():
    parts = []
    for tag, start, n in (("dst_end", "2013110112", 96), ("dst_start", "2014030712", 96), ("new_year", "2013123006", 60)):
        cells, forc = _perturbed_cells(4, n, 7, start)
        r = _run_job({"nsteps": n, "cells": cells})
        parts.append((tag, forc, r, [c["cfg"] for c in cells]))
    return parts


ZONE_WINDOWS = (  # (tag, lat, lon, zone the stub returns, start, steps): each crosses a US DST change
    ("phoenix", 34.0, -111.5, "America/Phoenix", "2014030712", 96),
    ("anchorage", 60.4, -148.9, "America/Anchorage", "2013110112", 96),
    ("denver", 40.02, -105.65, "America/Denver", "2014030712", 96),
    ("boise", 44.1, -114.9, "America/Boise", "2013110112", 96),
    ("chicago", 41.9, -93.1, "America/Chicago", "2014030712", 96),
    ("new_york", 44.27, -71.3, "America/New_York", "2013110112", 96),
    ("honolulu", 19.82, -155.47, "Pacific/Honolulu", "2013110112", 96),  # no DST: the offset stays -10
)


def build_zone_windows():
    """Runs outside America/Los_Angeles, so the reference's own
    gmt_offset_hours (solar_funcs.py:1616-1637) and zoneinfo pin the UTC
    offset of another zone: Arizona keeps -7 across the DST start, Alaska
    goes from -8 to -9 at the DST end."""
    parts = []
    for tag, lat, lon, zone, start, n in ZONE_WINDOWS:
        cells, forc = _perturbed_cells(4, n, 13, start, extra_cfg={"lat": lat, "lon": lon})
        r = _run_job({"nsteps": n, "cells": cells})
        parts.append((tag, zone, forc, r, [c["cfg"] for c in cells]))
    return parts


def build_dt(dt, float_dt, nsteps, ncell=8):
    cells, forc = _perturbed_cells(ncell, nsteps, 99, "2013032000", extra_cfg={"dt": dt})
    r = _run_job({"nsteps": nsteps, "cells": cells, "float_dt": float_dt})
    return forc, r, [c["cfg"] for c in cells]


def build_variant(extra_cfg, nsteps=288, ncell=8, seed=31):
    """Perturbed cells under a non-default configuration (SATTERLUND branches
    :784-796, :1190-1192; dust / canopy / cloud factors config.py:29-31)."""
    cells, forc = _perturbed_cells(ncell, nsteps, seed, "2013032000", extra_cfg=extra_cfg)
    r = _run_job({"nsteps": nsteps, "cells": cells})
    return forc, r, [c["cfg"] for c in cells]


def _save(name, forc, r, cfgs, **extra):
    import json

    import numpy as np

    keys = ["elev", "slope", "aspect", "h0_snow", "h0_ice", "h0_swe", "h0_iwe"]
    static = np.array([[dict(BASE_CFG, **c)[k] for k in keys] for c in cfgs], dtype=np.float64)
    np.savez_compressed(
        HERE / name,
        forcing=forc,  # [7 inputs][nsteps][ncell], IN_SHORT order
        outputs=r["outs"],  # [8 outputs][nsteps][ncell], OUT_SHORT order
        internal=r["ints"],  # [len(INTERNAL)][nsteps][ncell]
        static=static,  # [ncell][7]: elev, slope, aspect, h0_snow, h0_ice, h0_swe, h0_iwe
        in_names=np.array(IN_SHORT),
        out_names=np.array(OUT_SHORT),
        internal_names=np.array(INTERNAL),
        static_names=np.array(keys),
        base_cfg=json.dumps(BASE_CFG),
        cell_cfgs=json.dumps([dict(BASE_CFG, **c) for c in cfgs]),
        **extra,
    )
    print("wrote", name, r["outs"].shape)


def main(only=None):
    if only:
        if "satterlund" in only:
            f, r, c = build_variant({"SATTERLUND": True})
            _save("satterlund.npz", f, r, c)
        if "params" in only:
            f, r, c = build_variant({"dust_atten": 0.14, "canopy_factor": 0.2, "cloud_factor": 0.45}, seed=32)
            _save("params.npz", f, r, c)
        if "zones" in only:
            for tag, zone, f, r, c in build_zone_windows():
                _save(f"clock_{tag}.npz", f, r, c, tz_name=zone)
        return
    f, r, c = build_cat3062920()
    _save("cat3062920_265.npz", f, r, c)
    f, r, c = build_grid64()
    _save("grid64.npz", f, r, c)
    for tag, f, r, c in build_clock_windows():
        _save(f"clock_{tag}.npz", f, r, c)
    f, r, c = build_dt(2, False, 120)
    _save("dt2.npz", f, r, c)
    f, r, c = build_dt(0.25, True, 400)
    _save("dt_quarter.npz", f, r, c)
    main(["satterlund", "params", "zones"])


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        _child_main(sys.argv[2], sys.argv[3])
    elif len(sys.argv) > 2 and sys.argv[1] == "--only":
        main(sys.argv[2].split(","))
    else:
        main()
