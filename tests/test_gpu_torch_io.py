"""Device-tensor I/O between torch and the engine (GlacierEngine.set_field with a
CUDA tensor, GlacierEngine.get_field_device).  The engine copies on its own
HIP stream; these tests fail if a copy is not ordered against torch's stream
(the tensor is produced / consumed by torch kernels right before / after)."""

import numpy as np
import pytest

from tests.harness import BASE_CFG, make_engine

pytestmark = pytest.mark.gpu
HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
NY, NX = 512, 8192  # 4 M cells: copies long enough for an unordered read to be caught


def test_get_field_device_equals_host_copy_for_every_plane():
    import torch

    from topoflow_glacier.synthetic import diurnal_table

    e = make_engine(BASE_CFG, NY, NX, "float32", n_frames=24, hist_depth=4, fuse_steps=4)
    try:
        e.fill_synthetic(3, diurnal_table(24), nx_global=NX)
        e.run(4)
        e.sync()
        for k in range(4):
            for v in HIST:
                # a fresh tensor each time: the caching allocator hands back the
                # block just freed, so an unordered copy shows the previous plane
                t = e.get_field_device(v, torch.empty(NY * NX, dtype=torch.float32, device="cuda:0"), index=k)
                got = (t * 1.0).cpu().numpy()  # a torch kernel reads it first
                assert np.array_equal(got, e.get_field(v, index=k, dtype=np.float32)), (v, k)
        s = e.get_field_device("h_swe", torch.empty(NY * NX, dtype=torch.float64, device="cuda:0"))
        assert np.array_equal(s.cpu().numpy(), e.get_field("h_swe"))
    finally:
        e.close()


def test_set_field_from_a_fresh_torch_tensor():
    import torch

    e = make_engine(BASE_CFG, NY, NX, "float32", n_frames=2, hist_depth=1)
    try:
        for f in range(2):
            base = torch.arange(NY * NX, dtype=torch.float32, device="cuda:0")
            x = base * 0.5 + float(f)  # produced on torch's stream just before the call
            e.set_field("T_air", x, index=f)
            del x, base  # freed (and reusable) as soon as set_field returns
            torch.cuda.synchronize()
            want = np.arange(NY * NX, dtype=np.float32) * np.float32(0.5) + np.float32(f)
            assert np.array_equal(e.get_field("T_air", index=f, dtype=np.float32), want), f
    finally:
        e.close()


def test_set_inputs_from_a_dropped_tensor_on_the_engines_own_stream():
    """tfg_set_inputs from a device tensor reads it asynchronously on the
    engine's own stream: the tensor is recorded on that stream, so dropping it
    at once and letting torch refill the freed block cannot change what the
    engine reads (GlacierEngine.set_inputs)."""
    import torch

    e = make_engine(BASE_CFG, NY, NX, "float32", n_frames=2, hist_depth=1)
    try:
        torch.cuda.synchronize()
        for f in range(2):
            x = torch.arange(5 * NY * NX, dtype=torch.float32, device="cuda:0").reshape(5, NY * NX) * 1e-3 + f
            e.set_inputs(x, index=f)  # BMI order P_air, Hum_sp, P, T_air, uz
            del x
            junk = torch.full((5, NY * NX), -7.0, dtype=torch.float32, device="cuda:0")  # the freed block, if reused
            del junk
            want = np.arange(5 * NY * NX, dtype=np.float32).reshape(5, NY * NX) * np.float32(1e-3) + np.float32(f)
            for row, name in enumerate(("P_air", "Hum_sp", "P", "T_air", "uz")):
                assert np.array_equal(e.get_field(name, index=f, dtype=np.float32), want[row]), (name, f)
        with pytest.raises(ValueError):
            e.set_inputs(torch.zeros((5, NY * NX - 1), dtype=torch.float32, device="cuda:0"))
    finally:
        e.close()
