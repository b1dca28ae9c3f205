"""Split launches (include/tfg.h tfg_set_split, ABI 8): a small fp32 grid
stepped as two parts of about half its cells, the second on a second stream
with its own copy of the step uniforms, so that one part's next launch fills
the other's end-of-launch drain.

The update is pointwise (no term couples cells, bmi_topoflow_glacier.py
:413-465), so a split run must equal the one-launch run bit for bit: every
history output of every step, the fp64 state, and -- since each part's
workgroups fold into the slab rows of their own 256-cell chunks, one
workgroup per chunk as unsplit -- the mass-balance diagnostics.  The API calls
between launches (field reads, sets, diagnostics) order the handle's stream
after the second part; the grids below are not multiples of the 256-cell chunk,
so the second part ends in padding."""

import numpy as np
import pytest

from tests.harness import BASE_CFG, make_engine

pytestmark = pytest.mark.gpu

HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
STATE = ("h_swe", "h_iwe", "Eccs", "Ecci", "n", "albedo")


def _run(split, ny, nx, nsteps, fuse, flux="fp32", n_catch=1, nan_safe=False, reads=True, conduction=False):
    from topoflow_glacier.synthetic import diurnal_table

    e = make_engine(BASE_CFG, ny, nx, "float32", n_frames=24, hist_depth=nsteps, n_catch=n_catch,
                    fuse_steps=fuse, flux=flux, split=split)
    try:
        e.fill_synthetic(11, diurnal_table(24))
        if n_catch > 1:
            e.set_field("catch_id", (np.arange(ny * nx) * 7 // (ny * nx) % n_catch).astype(np.int32))
        if nan_safe:
            e.set_step_form(True)
        if conduction:  # the QC instance of k_fused, its Qc plane offset like the others
            e.run(3)
            e.conduction_update(0.3, 2.1, 30.0, 30.0, q_ground=0.5)
        was_split = e.is_split()
        mid = None
        k = 0
        while k < nsteps:  # uneven calls: several launches per call, a partial last launch
            step = min(nsteps - k, fuse + 5)
            e.run(step)
            k += step
            if reads and mid is None:
                mid = e.get_field("Eccs")  # an API read between calls: joins the second part
        hist = {v: np.stack([e.get_field(v, index=j, dtype=np.float32) for j in range(nsteps)]) for v in HIST}
        state = {v: e.get_field(v) for v in STATE if v != "albedo"}
        state["albedo"] = e.get_field("albedo", dtype=np.float32)
        return was_split, hist, state, e.diagnostics(), mid
    finally:
        e.close()


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("ny,nx,nsteps,fuse,flux,n_catch,nan_safe,conduction", [
    (37, 100, 60, 24, "fp32", 1, False, False),     # 3700 cells: 15 chunks, a part of 7
    (64, 513, 50, 16, "fp32", 5, False, False),     # catchment bins in both parts
    (37, 100, 30, 24, "fp64", 1, False, False),     # the fp64-flux form
    (37, 100, 30, 24, "fp32", 1, True, False),      # the NaN-safe form
    (37, 100, 30, 24, "fp32", 1, False, True),      # the lateral conduction term on
])
def test_split_equals_one_launch_bit_for_bit(ny, nx, nsteps, fuse, flux, n_catch, nan_safe, conduction):
    s1, h1, st1, d1, m1 = _run("on", ny, nx, nsteps, fuse, flux, n_catch, nan_safe, conduction=conduction)
    s0, h0, st0, d0, m0 = _run("off", ny, nx, nsteps, fuse, flux, n_catch, nan_safe, conduction=conduction)
    assert s1 and not s0
    for v in HIST:
        assert _same(h1[v], h0[v]), v
    for v in STATE:
        assert _same(st1[v], st0[v]), v
    assert _same(m1, m0)
    assert _same(d1, d0)


def test_auto_splits_a_config2_sized_grid_and_matches():
    """TFG_SPLIT_AUTO splits 2^18 .. 2^24 cells: 512 x 512 (2^18) splits and
    equals the unsplit run; 8192 cells do not split."""
    s1, h1, st1, d1, _ = _run("auto", 512, 512, 30, 24, reads=False)
    s0, h0, st0, d0, _ = _run("off", 512, 512, 30, 24, reads=False)
    assert s1 and not s0
    for v in HIST:
        assert _same(h1[v], h0[v]), v
    for v in STATE:
        assert _same(st1[v], st0[v]), v
    assert _same(d1, d0)
    e = make_engine(BASE_CFG, 64, 128, "float32", n_frames=1, hist_depth=1, split="auto")
    try:
        assert not e.is_split()
    finally:
        e.close()


def test_split_steps_are_joined_before_the_callers_stream_work():
    """On a caller's stream (tfg_set_stream, as bench.py runs): after tfg_join,
    a device-side read of a history slot queued on that stream sees both parts'
    outputs of the last step, and equals the API's own (joining) host read."""
    import torch

    from topoflow_glacier.synthetic import diurnal_table

    ny, nx, fuse = 512, 512, 48
    e = make_engine(BASE_CFG, ny, nx, "float32", n_frames=24, hist_depth=fuse, fuse_steps=fuse, split="on")
    try:
        e.fill_synthetic(3, diurnal_table(24))
        stream = torch.cuda.Stream(0)
        e.set_stream(stream.cuda_stream)
        out = torch.empty(ny * nx, dtype=torch.float32, device="cuda:0")
        for _ in range(3):
            e.run(fuse)
        want = e.get_field("M_total", index=fuse - 1, dtype=np.float32)  # the API joins
        e.run(fuse)
        e.join()
        with torch.cuda.stream(stream):
            e.get_field_device("M_total", out, index=fuse - 1)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert np.isfinite(got).all() and not np.array_equal(got, want)  # a later step's slot, both parts
        assert np.array_equal(got, e.get_field("M_total", index=fuse - 1, dtype=np.float32))
    finally:
        e.close()
