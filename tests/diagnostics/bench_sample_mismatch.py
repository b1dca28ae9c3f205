"""Which cells of bench.py's parity spot check are neither within 1e-5 nor a
melt-out flip, and why?  Runs the spot check's workload (first N cells of the
synthetic grid, S hourly steps, every step kept) on the GPU and in the C
oracle, classifies with tests.harness.melt_out_flips, and for each remaining
cell prints the step-by-step outputs of the GPU, the C oracle and the numpy
oracle around the first bad step.  Diagnostic only (test infrastructure)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
import tfg_oracle as O  # noqa: E402
import tfg_oracle_c as OC  # noqa: E402

import bench  # noqa: E402
from tests.harness import melt_out_flips  # noqa: E402
from topoflow_glacier.bmi.config import TopoflowGlacierConfig  # noqa: E402
from topoflow_glacier.engine import GlacierEngine  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table, synthetic_cells  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 96
seed = 20251001
names = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")

cfg = dict(bench.BASE_CFG)
scfg = TopoflowGlacierConfig.model_validate(dict(cfg, ny=1, nx=n))
eng = GlacierEngine(scfg, 1, n, engine="float32", device=0, n_frames=24, hist_depth=steps, fuse_steps=96)
eng.fill_synthetic(seed, diurnal_table(24), nx_global=n)
eng.run(steps)
eng.sync()
gpu = {k: np.stack([eng.get_field(k, index=j) for j in range(steps)]) for k in names}
eng.close()

syn = synthetic_cells(seed, np.arange(n), diurnal_table(24))
static = {k: np.asarray(v, np.float64) for k, v in dict(
    elev=syn["elev"], slope=syn["slope"], aspect=syn["aspect"], h0_snow=syn["h_snow"], h0_ice=syn["h_ice"],
    h0_swe=syn["h_swe"], h0_iwe=syn["h_iwe"]).items()}
frames = np.arange(steps) % 24
forcing = {k: syn[k].astype(np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
clock = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
ref, _ = OC.run_oracle_c(cfg, static, forcing, steps, clock=(clock[0], clock[3]), frames=frames, nthreads=16)
flip, genuine = melt_out_flips(gpu, ref)
print(f"cells {n} steps {steps}: flips {(flip >= 0).sum()}, genuine {len(genuine)}")
cells = [c for c, _, _ in genuine[:8]]
if cells:
    sub = {k: v[cells] for k, v in static.items()}
    fnp = {k: syn[k][frames][:, cells].astype(np.float64) for k in forcing}
    npo, _ = O.run_oracle(cfg, sub, fnp, steps, clock=(clock[0], clock[3]))
    for i, (c, k, vs) in enumerate(genuine[:8]):
        print(f"\ncell {c}: first bad step {k}, vars {vs}; static "
              + " ".join(f"{kk}={static[kk][c]:.6g}" for kk in static))
        for j in range(max(0, k - 3), min(steps, k + 2)):
            f = frames[j]
            print(f"  step {j} P={syn['P'][f, c]:.3e} T={syn['T_air'][f, c]:.3f}")
            for v in names:
                print(f"    {v:8s} gpu {gpu[v][j, c]: .9e}  C {ref[v][j, c]: .9e}  numpy {npo[v][j, i]: .9e}")
        for v in ("albedo", "n", "Eccs", "Ecci", "Q_sum", "Qn_SW"):
            print(f"    numpy {v:6s} " + " ".join(f"{npo[v][j, i]: .6e}" for j in range(max(0, k - 3), min(steps, k + 2))))

# Where does the largest in-tolerance error sit?  Per variable: the max
# floored error over unflipped (cell, step) pairs and the worst cell's trace.
from tests.harness import valid_mask  # noqa: E402

ok = valid_mask(flip, steps)
worst = []
for v in names:
    r, g = ref[v], gpu[v]
    nz = np.abs(r[r != 0])
    s_v = np.percentile(nz, 99) if nz.size else 0.0
    e = np.where(ok, np.abs(g - r) / np.maximum(np.maximum(np.abs(r), s_v), 1e-300), 0.0)
    k, c = np.unravel_index(np.argmax(e), e.shape)
    print(f"{v:8s} max floored err {e.max():.3e} at cell {c} step {k}; s_v {s_v:.3e}; "
          f"frac > 1e-6: {np.mean(e > 1e-6):.2e}")
    worst.append((e.max(), v, int(c), int(k)))
worst.sort(reverse=True)
cells = sorted({c for _, _, c, _ in worst[:3]})
sub = {kk: v[cells] for kk, v in static.items()}
fnp = {kk: syn[kk][frames][:, cells].astype(np.float64) for kk in forcing}
npo, _ = O.run_oracle(cfg, sub, fnp, steps, clock=(clock[0], clock[3]))
for err, v, c, k in worst[:3]:
    i = cells.index(c)
    print(f"\nworst {v} cell {c} step {k} err {err:.3e}")
    for j in range(max(0, k - 4), min(steps, k + 2)):
        print(f"  step {j}: {v} gpu {gpu[v][j, c]: .9e} ref {ref[v][j, c]: .9e}; numpy Eccs {npo['Eccs'][j, i]: .6e} "
              f"Ecci {npo['Ecci'][j, i]: .6e} Q_sum {npo['Q_sum'][j, i]: .6e} h_swe {npo['h_swe'][j, i]: .6e}")
