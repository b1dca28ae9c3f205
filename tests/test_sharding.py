"""Row-block sharding over torch.distributed: world size 2,
launched with torchrun on 127.0.0.1, gloo for the diagnostics all-reduce.

CPU: every rank runs the oracle on its block; the all-reduced diagnostics and
the stitched fields must equal one oracle run over the whole grid.
GPU: every rank runs the HIP engine on its block (both on cuda:0); stitched
fields equal an unsharded GPU run bit for bit, reduced diagnostics match the
oracle of the whole grid."""

from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.harness import ROOT, oracle_diag, oracle_synthetic, run_gpu_vs_oracle
from topoflow_glacier.sharding import row_block

NY, NX, STEPS = 7, 12, 30  # 7 rows over 2 ranks: uneven blocks (4 + 3)


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(mode: str, out, world: int = 2, ny: int = NY, nx: int = NX, steps: int = STEPS):
    env = dict(os.environ, OMP_NUM_THREADS="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "shard_worker.py"),
           "--mode", mode, "--ny", str(ny), "--nx", str(nx), "--steps", str(steps), "--out", str(out)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return [dict(np.load(out / f"rank{i}.npz")) for i in range(world)]


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(b != 0, np.abs(a - b) / np.abs(b), np.abs(a - b))
    return float(np.max(r))


def test_row_block_partition():
    for ny in (1, 2, 7, 8192, 16385):
        for world in (1, 2, 3, 8):
            blocks = [row_block(ny, r, world) for r in range(world)]
            assert sum(b[1] for b in blocks) == ny
            assert all(blocks[i][0] + blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            assert max(b[1] for b in blocks) - min(b[1] for b in blocks) <= 1
    with pytest.raises(ValueError):
        row_block(8, 2, 2)


def test_sharded_oracle_gloo_world2(tmp_path):
    ranks = _torchrun("oracle", tmp_path)
    ref, m = oracle_synthetic(11, NY, NX, STEPS)
    whole = oracle_diag(m)
    for r in ranks:
        # sums: the two shards' partial sums add to the whole-grid sum up to reassociation
        assert _rel(r["reduced"][0, :5], whole[0, :5]) <= 1e-13
        assert r["reduced"][0, 5] == whole[0, 5]
        np.testing.assert_array_equal(r["reduced"], ranks[0]["reduced"])
    assert [int(r["rows"]) for r in ranks] == [4, 3]
    for k in ("h_snow", "SM", "IM", "M_total", "RH"):
        stitched = np.concatenate([r[k] for r in ranks])
        np.testing.assert_array_equal(stitched, ref[k][-1])


def test_config5_catchment_diagnostics_gloo_world2(tmp_path):
    """BASELINE config 5's per-catchment mass balance in its sharded form:
    bench.py's 43-catchment block raster over a row-blocked grid, dt = 0.25 h;
    each rank's [44][6] per-catchment integrals (oracle, binned) combined by
    allreduce_diagnostics over gloo equal the whole grid's."""
    import bench
    from tests.harness import catchment_diag, synthetic_inputs

    ny, nx, steps = 16, 32, 24
    ranks = _torchrun("catch", tmp_path, ny=ny, nx=nx, steps=steps)
    _, m = oracle_synthetic(11, ny, nx, steps, 24, cfg_over={"dt": 0.25})
    syn, _ = synthetic_inputs(11, ny, nx, 24)
    cid = bench.catchment_blocks(0, ny, ny, nx, 43)
    whole = catchment_diag(syn, m, cid, steps, 24, 44, {"dt": 0.25})
    assert set(np.unique(cid)) == set(range(43))  # every catchment id occurs in the grid
    np.testing.assert_array_equal(np.concatenate([r["cid"] for r in ranks]), cid)
    for r in ranks:
        assert r["reduced"].shape == (44, 6)
        np.testing.assert_array_equal(r["reduced"], ranks[0]["reduced"])
        assert _rel(r["reduced"][:, :5], whole[:, :5]) <= 1e-13
        np.testing.assert_array_equal(r["reduced"][:, 5], whole[:, 5])
    assert np.all(whole[:43, 0] > 0) and np.all(whole[43] == 0)


@pytest.mark.gpu
def test_sharded_engine_gloo_world2(tmp_path):
    ny, nx, steps = 64, 96, 48
    ranks = _torchrun("gpu", tmp_path, ny=ny, nx=nx, steps=steps)
    whole = run_gpu_vs_oracle(ny, nx, steps, seed=11)
    assert whole["ok"], whole["summary"]
    for k in ("h_snow", "SM", "IM", "M_total", "RH"):
        stitched = np.concatenate([r[k] for r in ranks])
        np.testing.assert_array_equal(stitched, whole["gpu"][k][-1])
    red = ranks[0]["reduced"][0]
    np.testing.assert_array_equal(red, ranks[1]["reduced"][0])
    assert _rel(red[:3], whole["diag_ref"][:3]) <= 1e-5
    assert red[5] == whole["diag_ref"][5] or _rel(red[5], whole["diag_ref"][5]) <= 1e-7


@pytest.mark.gpu
def test_rccl_paths_world1(tmp_path):
    """RCCL (the nccl backend) on the one GPU of the test box, world size 1
    (RCCL refuses two ranks on one device): the diagnostics all-reduce, a
    batched point-to-point exchange of device tensors with the rank itself,
    and the nccl branches of sharding.lateral_conduction and sharding.ice_flow
    equal the same work without a process group, bit for bit."""
    env = dict(os.environ, OMP_NUM_THREADS="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "rccl_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    z = dict(np.load(tmp_path / "rank0.npz"))
    assert str(z["backend"]) == "nccl"
    np.testing.assert_array_equal(z["diag_out"], z["diag_in"])
    # 43 catchments (+1 spare row) of a config-5 shard through the RCCL all-reduce
    assert z["catch_diag_in"].shape == (44, 6)
    np.testing.assert_array_equal(z["catch_diag_out"], z["catch_diag_in"])
    present = z["catch_diag_in"][:43, 0] > 0  # the shard's rows hold some of the 43 block catchments
    assert present.sum() >= 4 and np.all(z["catch_diag_in"][43] == 0)
    if "p2p_refused" in z:
        print("self point-to-point refused:", z["p2p_refused"])
    else:
        np.testing.assert_array_equal(z["p2p_received"], z["p2p_sent"])
    np.testing.assert_array_equal(z["qc_rccl"], z["qc_local"])
    assert np.any(z["qc_local"] != 0)
    assert int(z["nsub_rccl"]) == int(z["nsub_local"]) >= 1
    np.testing.assert_array_equal(z["iwe_rccl"], z["iwe_local"])
