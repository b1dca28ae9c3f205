"""Single-catchment driver: the reference's examples/run_topoflow_glacier.py on
this engine.

  python -m topoflow_glacier.run CONFIG.yaml [--forcing CSV] [--mode bmi|bulk] [--out run.npz]

Modes
  bmi   the reference driver's loop (:50-110): per step, set_value() the seven
        inputs, update(), get_value() the eight outputs -- through the drop-in
        BmiTopoflowGlacier (fp64 engine, bit-near the reference).
  bulk  the same run with every forcing row uploaded once as an HBM-resident
        frame and all steps advanced by fused launches (tfg_step over the
        whole window); outputs read back once.  Same arithmetic as `bmi`
        (fusion is invisible, tests/test_gpu_parity.py), without the per-step
        host round trips.

Both return the eight outputs per step (bulk: h_swe/h_iwe at the last step
only, they are engine state), runoff [m3 s-1] = M_total * da_m2 (:112) and the
20-tap routed runoff (:129-131).
"""

from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

from .forcing import read_forcing_csv
from .routing import boxcar_route

__all__ = ["run_catchment", "main"]

OUT_BMI = {
    "h_snow": "snowpack__depth",
    "h_swe": "snowpack__liquid-equivalent_depth",
    "SM": "snowpack__melt_volume_flux",
    "h_ice": "glacier_ice__thickness",
    "h_iwe": "glacier__liquid_equivalent_depth",
    "IM": "glacier_ice__melt_volume_flux",
    "M_total": "land_surface_water__runoff_volume_flux",
    "RH": "atmosphere_bottom_air_water-vapor__relative_saturation",
}


def _resolve_forcing(cfg_path: Path, forcing_file: str) -> Path:
    p = Path(forcing_file)
    for cand in (p, cfg_path.parent / p, cfg_path.parent.parent / p):
        if cand.exists():
            return cand
    raise FileNotFoundError(f"forcing file {forcing_file} not found (relative to . or {cfg_path.parent})")


def run_catchment(config: str | Path, forcing: str | Path | None = None, mode: str = "bmi") -> dict:
    """Run one catchment over its configured window.  Returns a dict of arrays."""
    from .bmi.bmi_topoflow_glacier import BmiTopoflowGlacier

    cfg_path = Path(config)
    model = BmiTopoflowGlacier()
    model.initialize(cfg_path)
    table = read_forcing_csv(forcing or _resolve_forcing(cfg_path, model.cfg.forcing_file),
                             model.cfg.start_time, model.cfg.end_time)
    nsteps = len(table)
    out = {k: np.zeros(nsteps) for k in OUT_BMI}
    if mode == "bmi":
        dest = np.zeros(1)
        for i in range(nsteps):
            table.apply(model, i)
            model.update()
            for k, name in OUT_BMI.items():
                out[k][i] = model.get_value(name, dest).item()
    elif mode == "bulk":
        from .bmi.bmi_topoflow_glacier import configure_engine, make_engine

        eng = make_engine(model.cfg, n_frames=nsteps, hist_depth=nsteps)
        if configure_engine(eng, model.cfg):
            eng.close()
            raise AttributeError("'BmiTopoflowGlacier' object has no attribute 'beta'")  # as update() would
        for internal in ("P", "T_air", "Hum_sp", "P_air", "uz"):  # LW_in / SW_in are never read (:1122, :1235)
            for i in range(nsteps):
                eng.set_field(internal, np.float64(table.inputs[internal][i]), index=i)
        eng.run(nsteps, frames=np.arange(nsteps, dtype=np.int32))
        eng.sync()
        for k in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH"):
            out[k] = np.array([eng.get_field(k, index=i)[0] for i in range(nsteps)])
        out["h_swe"][:] = np.nan
        out["h_iwe"][:] = np.nan
        out["h_swe"][-1] = eng.get_field("h_swe")[0]
        out["h_iwe"][-1] = eng.get_field("h_iwe")[0]
        eng.close()
    else:
        raise ValueError(f"mode must be 'bmi' or 'bulk', not {mode!r}")
    da_m2 = model.da_m2
    model.finalize()
    runoff = out["M_total"] * da_m2  # m/s -> m3/s (:112)
    return dict(out, times=table.times, runoff=runoff, routed=boxcar_route(runoff), da_m2=da_m2)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m topoflow_glacier.run", description=__doc__.split("\n\n")[0])
    ap.add_argument("config")
    ap.add_argument("--forcing", default=None, help="forcing CSV (default: the config's forcing_file)")
    ap.add_argument("--mode", default="bmi", choices=["bmi", "bulk"])
    ap.add_argument("--out", default=None, help="write all series to this .npz")
    a = ap.parse_args(argv)
    import time

    t0 = time.perf_counter()
    r = run_catchment(a.config, a.forcing, a.mode)
    print(f"steps: {len(r['runoff'])}  mode: {a.mode}  wall: {time.perf_counter() - t0:.3f} s (incl. initialize)")
    for k, label in (("RH", "Relative Humidity"), ("SM", "Snow Melt"), ("IM", "Ice Melt"), ("h_swe", "Height SWE"),
                     ("h_iwe", "Height IWE"), ("h_snow", "Snow Height"), ("h_ice", "Ice Height")):
        print(f"|- Final Timestep {label}: {r[k][-1]}")
    print(f"|- Final Timestep Runoff from melt: {r['runoff'][-1]}")
    print(f"|- Final Timestep Routed runoff: {r['routed'][-1]}")
    if a.out:
        np.savez(a.out, **{k: v for k, v in r.items() if isinstance(v, np.ndarray)})
    return 0


if __name__ == "__main__":
    sys.exit(main())
