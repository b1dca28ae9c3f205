"""Extract the 43 catchment divides of the reference's hydrofabric
(/root/reference/data/12082500.gpkg, layer `divides`) into a small fixture,
tests/golden/hydrofabric_12082500.npz: divide ids, areasqkm, and the polygon
rings (EPSG:5070 metres) as concatenated vertex arrays with offsets.

Test infrastructure; runs only in the build container, read-only on the
reference file (sqlite immutable mode).  Usage: python3 tests/golden/make_hydrofabric.py
"""

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1] / "topoflow-glacier_amd"))
from topoflow_glacier.hydrofabric import read_divides  # noqa: E402

srs, dv = read_divides("/root/reference/data/12082500.gpkg")
pts, ring_off, ring_poly, poly_div = [], [0], [], []
for k, d in enumerate(dv):
    for p in d.polygons:
        poly_div.append(k)
        for r in p:
            pts.append(r)
            ring_off.append(ring_off[-1] + len(r))
            ring_poly.append(len(poly_div) - 1)
np.savez_compressed(HERE / "hydrofabric_12082500.npz", srs=srs, divide_id=np.array([d.divide_id for d in dv]),
                    areasqkm=np.array([d.areasqkm for d in dv]), xy=np.concatenate(pts), ring_off=np.array(ring_off),
                    ring_poly=np.array(ring_poly), poly_div=np.array(poly_div))
print(f"{len(dv)} divides, {sum(len(r) for r in pts)} vertices, srs {srs}")
