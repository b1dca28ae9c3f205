"""One rank of the nccl backend (RCCL) on one GPU, launched by torchrun with
world size 1 from tests/test_sharding.py::test_rccl_paths_world1.  Test
infrastructure.

The GPU box of this build has one MI355X, and RCCL refuses two ranks on one
device ("Duplicate GPU detected"), so world size 1 is how the RCCL code paths
run here: the diagnostics all-reduce, a batched point-to-point exchange of
device tensors with the rank itself, and the nccl branches of
sharding.lateral_conduction and sharding.ice_flow (edge rows written into CUDA
tensors, the MAX all-reduce of the CFL bound, interior / edge sub-step parts),
each against the same work without a process group.  Writes <out>/rank0.npz.
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]


def main():
    out = Path(sys.argv[1])
    import torch
    import torch.distributed as dist

    from tests.harness import BASE_CFG, conduction_state, glacier_valley, make_engine
    from topoflow_glacier.sharding import allreduce_diagnostics, ice_flow, lateral_conduction

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    res = {"backend": np.array(dist.get_backend())}
    # the diagnostics all-reduce (sum of columns 0-4, max of column 5) on device tensors
    d = np.arange(18, dtype=np.float64).reshape(3, 6) * 0.25 - 1.0
    res["diag_in"], res["diag_out"] = d, allreduce_diagnostics(d)
    # config 5's per-catchment mass balance through the same all-reduce: an
    # engine shard with bench.py's 43-catchment block raster (rows 6144.. of a
    # 16384-row grid, as rank 3 of 8 holds them), dt = 0.25 h, 96 fused steps
    import bench
    from topoflow_glacier.synthetic import diurnal_table

    cny, cnx, crow0 = 64, 512, 6144
    e = make_engine(dict(BASE_CFG, dt=0.25), cny, cnx, "float32", n_frames=24, hist_depth=96, n_catch=44,
                    fuse_steps=96, row0=crow0)
    e.fill_synthetic(20251001, diurnal_table(24), nx_global=cnx)
    e.set_field("catch_id", bench.catchment_blocks(crow0, cny, 16384, cnx, 43))
    e.run(192)
    e.sync()
    dc = e.diagnostics()
    e.close()
    res["catch_diag_in"], res["catch_diag_out"] = dc, allreduce_diagnostics(dc)
    # a batched isend / irecv of a device tensor with this rank itself
    x = torch.arange(64, dtype=torch.float64, device="cuda") * 1.5
    y = torch.full_like(x, -1.0)
    try:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, y, 0)]):
            w.wait()
        torch.cuda.synchronize()
        res["p2p_sent"], res["p2p_received"] = x.cpu().numpy(), y.cpu().numpy()
    except (ValueError, RuntimeError) as e:  # torch may refuse a self exchange; recorded, not hidden
        res["p2p_refused"] = np.array(str(e)[:300])
    # sharding.lateral_conduction, nccl branch against no process group
    ny, nx = 48, 40
    swe, iwe, eccs, ecci = conduction_state(ny, nx)
    qc = []
    for distributed in (True, False):
        e = make_engine(dict(BASE_CFG), ny, nx, "float64", n_frames=1, hist_depth=1)
        e.init_state()
        for name, v in (("h_swe", swe), ("h_iwe", iwe), ("Eccs", eccs), ("Ecci", ecci)):
            e.set_field(name, v.reshape(-1))
        lateral_conduction(e, 0.3, 2.1, 2.0, 3.0, distributed=distributed)
        qc.append(e.get_field("Qc"))
        e.close()
    res["qc_rccl"], res["qc_local"] = qc
    # sharding.ice_flow, nccl branch (device edge rows, RCCL MAX of the CFL
    # bound, interior then edge parts) against one unsharded run
    bed, iwe0 = glacier_valley(ny, nx)
    flow = []
    for distributed in (True, False):
        e = make_engine(dict(BASE_CFG), ny, nx, "float32", n_frames=1, hist_depth=1)
        e.set_field("elev", bed.reshape(-1).astype(np.float32))
        e.set_field("h_iwe", iwe0.reshape(-1))
        e.init_state()
        n_sub = ice_flow(e, 0.5, 100.0, 100.0, distributed=distributed)
        flow.append((e.get_field("h_iwe"), n_sub))
        e.close()
    (res["iwe_rccl"], res["nsub_rccl"]), (res["iwe_local"], res["nsub_local"]) = flow
    np.savez(out / "rank0.npz", **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
