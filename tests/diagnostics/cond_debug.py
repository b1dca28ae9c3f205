import sys, numpy as np
sys.path[:0] = ["/root/repo", "/root/repo/topoflow-glacier_amd"]
from tests.harness import run_gpu_vs_oracle
from tests.test_conduction import _cold, KS, KI
ny, nx, nsteps = 24, 32, 48
cond = dict(k_snow=KS, k_ice=KI, dx=1.0, dy=1.0, every=16)
for c in (cond, None):
    r = run_gpu_vs_oracle(ny, nx, nsteps, engine="float32", seed=17, cold=_cold(ny, nx, 6), conduction=c)
    print(r["summary"])
    g, f = r["gpu"], r["ref"]
    cell = 764
    for k in range(28, 40):
        print(k, " ".join(f"{v}={g[v][k, cell]:.9e}/{f[v][k, cell]:.9e}" for v in ("SM", "M_total", "IM", "h_snow")),
              " ".join(f"{t}={f[t][k, cell]:.4e}" for t in ("Q_sum", "Qn_SW", "Qn_LW", "Qh", "Qe", "Eccs")))
