"""bench.py keeps the driver's contract: one JSON line on stdout with the
metric, value, roofline and cpu_baseline objects (small workload, GPU), and
its shard plan partitions BASELINE config 4's one grid over N ranks (CPU)."""

import json
import subprocess
import sys

import numpy as np
import pytest

from tests.harness import ROOT


def _args(*argv):
    sys.path.insert(0, str(ROOT))
    import bench

    old = sys.argv
    try:
        sys.argv = ["bench.py", *argv]
        return bench, bench.parse()
    finally:
        sys.argv = old


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_default_shard_plan_is_config4_strong_scaling(world):
    """--gpus N (the driver's SCALE runs) splits ONE 8192 x 8192 grid by rows:
    every row exactly once, 8192 / N rows per rank; N = 1 is the whole grid."""
    bench, args = _args("--gpus", str(world))
    plans = [bench.shard_plan(args, world, r) for r in range(world)]
    assert all(p["ny_global"] == 8192 for p in plans)
    rows = np.concatenate([np.arange(p["row0"], p["row0"] + p["rows"]) for p in plans])
    assert np.array_equal(rows, np.arange(8192))
    assert plans[0]["workload"] == f"8192x8192 grid ({8192 // world}x8192 per GPU)"
    assert plans[0]["scaling"] == "strong"  # one label for the driver's whole N = 1, 2, 4, 8 series


@pytest.mark.parametrize("world,fuse", [(1, 128), (2, 256), (4, 384), (8, 384)])
def test_driver_command_times_the_same_work_at_every_n(world, fuse):
    """`--steps 20`: whole launches, >= 6, and the same 2304 steps at every N
    (128-step launches for the whole 8192^2 grid, 256 for 4096 x 8192, 384 for
    the smaller slabs)."""
    bench, args = _args("--gpus", str(world), "--steps", "20", "--warmup", "5")
    plan = bench.shard_plan(args, world, 0)
    k = bench.auto_fuse(plan["rows_max"] * args.nx)
    steps = bench.timed_steps(args.steps, k, explicit=False)
    assert k == fuse and steps == 2304 and steps % k == 0 and steps // k >= bench.MIN_LAUNCHES
    assert bench.timed_steps(48, 24, explicit=True) == 144  # an explicit --fuse: >= 6 launches of it
    # the driver's --warmup 5 still warms one whole launch of the timed depth
    assert bench.warmup_steps(args.warmup, k) == k and bench.warmup_steps(400, k) == 400
    # the fp64 engine's history slots are twice as large: half the depth, the same timed steps
    k64 = bench.auto_fuse(plan["rows_max"] * args.nx, 8)
    assert k64 * 2 == k and bench.timed_steps(args.steps, k64, explicit=False) == 2304


def test_byte_model_prices_each_engine_by_its_element_size():
    """roofline.achieved's algorithmic bytes: the fp32 engine 52 B per step +
    120 B per launch (52.9375 B per cell-update at the bench's 128-step
    launches; 172 B at one step per launch, the per-step drop-in path: the
    albedo plane is written in fp32 and not read, round 6), the fp64 engine
    96 + 168 (its forcing frames, output slots and geometry are f64: 96.875 B
    at its automatic 192 steps on 4096^2)."""
    bench, _ = _args()
    assert bench.bytes_model(4) == (52, 120) and bench.bytes_model(8) == (96, 168)
    assert bench.launch_bytes_per_cell(128) / 128 == 52.9375 and bench.launch_bytes_per_cell(1) == 172
    k64 = bench.auto_fuse(4096 * 4096, 8)
    assert k64 == 192 and bench.launch_bytes_per_cell(k64, 8) / k64 == 96.875
    # the catchment variant reads the id raster, the conduction variant Qc, once per launch
    assert bench.bytes_model(4, catchments=True, qc=True) == (52, 120 + 4 + 4)


def test_pmc_traffic_is_keyed_by_engine_and_kernel_code(tmp_path, monkeypatch):
    """roofline.traffic comes from the engine's own PMC profile (_f64 suffix for
    the fp64 engine), and only when the profile's kernel hash equals the
    running library's hash of that engine's timed kernel."""
    bench, args = _args("--ny", "4096", "--nx", "4096", "--engine", "float64", "--fuse", "192")
    from topoflow_glacier import _native as nat

    monkeypatch.setattr(bench, "ROOT", tmp_path)
    (tmp_path / "profiles").mkdir()
    prof = tmp_path / "profiles" / "pmc_4096x4096_fuse192_f64.json"
    t, src = bench.pmc_traffic(4096, args)
    assert t is None and "not measured" in src["reason"]
    monkeypatch.setattr(nat, "kernel_code_sha256", lambda sym=nat.BENCH_KERNEL, path=None: "h-" + sym)
    prof.write_text(json.dumps({"kernel_code_sha256": "h-" + nat.BENCH_KERNEL_F64, "hbm_bytes_per_launch": 1.5e12}))
    t, src = bench.pmc_traffic(4096, args)
    assert t == 1.5e12 and src["match"] and src["kernel"] == nat.BENCH_KERNEL_F64
    prof.write_text(json.dumps({"kernel_code_sha256": "h-" + nat.BENCH_KERNEL, "hbm_bytes_per_launch": 1.5e12}))
    t, src = bench.pmc_traffic(4096, args)  # an fp32 kernel's profile is not quoted for the fp64 engine
    assert t is None and not src["match"]


def test_config5_eight_gpu_command_fits_its_shards():
    """BASELINE config 5 as the driver would run it on 8 GPUs
    (`--gpus 8 --ny 16384 --nx 16384 --dt 0.25 --catchments 43`): 2048 x 16384
    cells per rank, the automatic 256-step depth, a 288-slot snowfall window,
    and a per-rank device footprint (tfg_create's allocations at that depth)
    within the 280 GB budget, so no rank falls back; the 43 catchments of the
    block raster all occur, spread over the ranks' rows."""
    bench, args = _args("--gpus", "8", "--ny", "16384", "--nx", "16384", "--dt", "0.25", "--catchments", "43")
    plans = [bench.shard_plan(args, 8, r) for r in range(8)]
    assert all(p["rows"] == 2048 for p in plans) and plans[0]["workload"] == "16384x16384 grid (2048x16384 per GPU)"
    rows = np.concatenate([np.arange(p["row0"], p["row0"] + p["rows"]) for p in plans])
    assert np.array_equal(rows, np.arange(16384))
    cells = 2048 * 16384
    k = bench.auto_fuse(cells)
    ring = int(3 * 24 / 0.25)
    assert k == 256 and ring == 288
    fp = bench.device_footprint(cells, 24, k, ring, 44, 4, True)
    assert 250e9 < fp <= bench.DEVICE_BYTES_BUDGET, fp
    assert bench.fit_depth(k, cells, 24, ring, 44, 4, True) == k
    steps = bench.timed_steps(20, k, explicit=False)
    assert steps == 2304 and steps % k == 0
    # the 8192^2 headline shard at 128 steps: ~266 GB, also within budget
    assert bench.device_footprint(8192 * 8192, 24, 128, 72, 1) <= bench.DEVICE_BYTES_BUDGET
    # a depth that would not fit falls back down the ladder (each step count divides 768)
    assert bench.fit_depth(384, cells, 24, ring, 44, 4, True) == 256
    assert all(bench.STEP_QUANTUM % d == 0 for d in bench.DEPTH_LADDER)
    ids = np.unique(np.concatenate([bench.catchment_blocks(p["row0"], p["rows"], 16384, 16384, 43) for p in plans]))
    assert np.array_equal(ids, np.arange(43))
    # every rank's parity check covers its own first rows (65536 cells = 4 rows of 16384)
    pp = [bench.parity_plan(args, p, 8) for p in plans]
    assert [q["row0"] for q in pp] == [p["row0"] for p in plans] and all(q["cells"] == 65536 for q in pp)


def test_parity_check_runs_the_timed_launch_shape():
    """N = 1: the parity check's GPU run is a one-step lead-in launch (the
    instance that reads the initial depths) then ONE whole launch of the
    timed depth (128 steps at 8192^2), on the first 32 rows of the grid."""
    bench, args = _args("--gpus", "1")
    args.fuse = bench.auto_fuse(8192 * 8192)
    plan = bench.shard_plan(args, 1, 0)
    pp = bench.parity_plan(args, plan, 1)
    assert pp["launch_steps"] == [1, 128] and pp["steps"] == 129 and pp["cells"] == 262144 and pp["rows"] == 32


def test_weak_scaling_stays_behind_its_flag():
    bench, args = _args("--gpus", "4", "--scaling", "weak")
    p = [bench.shard_plan(args, 4, r) for r in range(4)]
    assert p[3]["row0"] == 3 * 8192 and p[3]["rows"] == 8192 and p[0]["workload"] == "32768x8192 grid (8192x8192 per GPU)"


@pytest.mark.gpu
def test_bench_prints_one_json_line_with_the_contract_keys():
    cmd = [sys.executable, str(ROOT / "bench.py"), "--ny", "256", "--nx", "1024", "--steps", "48", "--warmup", "24",
           "--fuse", "24", "--cpu-cells", "4096", "--cpu-steps", "48", "--parity-cells", "2048",
           "--dropin-instances", "64", "--dropin-queued", "--dropin-clean"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    # --steps 48 with 24-step launches: at least 6 whole launches are timed
    assert d["n_gpus"] == 1 and d["steps"] == 144 and d["steps_requested"] == 48 and d["steps_note"]
    assert d["launches"]["count"] == 6 and d["launches"]["ms_min"] <= d["launches"]["ms_mean"] <= d["launches"]["ms_max"]
    assert d["value"] > 0 and d["higher_is_better"] is True
    assert d["config"]["workload"] and d["dtype"] == "f32" and d["scaling"] == "strong"
    assert d["nan_safe_timed_launches"] == 0  # synthetic data is finite: the clean step form was timed
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["sample"]
    sp = d["sample_parity"]
    assert sp["genuine_mismatches"] == 0 and sp["max_floored_rel"] <= sp["tolerance"]
    assert sp["ok"] and sp["melt_out_flips"] <= sp["flip_budget"] and "flips_fp64_baseline" in sp
    # the check reads the bench handle's own first launches: a one-step lead-in, then a whole launch of the
    # timed depth over the whole shard, on the clean step form; the untimed steps include them
    assert sp["steps"] == 24 and sp["launch_steps"] == [1, 24] and sp["steps_compared"] == 25
    assert sp["cells"] == 2048 and sp["nan_safe_launches"] == 0 and sp["mass_balance"]["P_max_exact"]
    assert "256x1024 shard" in sp["timed_kernel_instance"] and sp["mass_balance"]["cells"] == 256 * 1024
    assert sp["mass_balance"]["vol_P_PR_PS_max_rel"] <= 1e-6 and d["warmup_steps_run"] == 49  # lead-in + parity launch + one more whole launch
    assert d["ranks"]["ranks"][0]["sample_parity"]["ok"]
    # the drop-in legs: per-step K = 1 launches from device inputs, and queued steps; defer_update instances
    g = d["dropin_per_step_grid"]
    assert g["per_step"]["value"] > 0 and g["queued"]["value"] > 0 and g["per_step"]["bytes_per_cell_update"] == 172
    # the same-run A/B of the step forms at K = 1: device-set inputs run NaN-safe, host-checked frames clean
    assert g["per_step"]["nan_safe_launches"] == 24 and g["clean_form_step_launch"]["nan_safe_launches"] == 0
    assert g["clean_form_step_launch"]["nan_safe_over_clean"] > 0
    mi = d["dropin_defer_update_instances"]
    assert mi["instances"] == 64 and mi["us_per_instance_step"] > 0 and mi["all_instances_equal"]
    ts = rf["traffic_source"]  # no PMC profile of this shape: traffic is null and says why
    assert rf["traffic"] is None and ts["reason"]
    # 2^18 cells: split launches (tfg_set_split AUTO), timed as the span of the timed region
    assert d["config"]["launch_parts"] == 2 and "span of the timed region" in rf["launch_time_source"]


@pytest.mark.gpu
def test_bench_parity_holds_at_the_deep_launches_of_the_multi_gpu_lines():
    """The N = 4 / N = 8 lines fuse 384 steps; the synthetic snowpacks start
    to run dry after ~300 steps, so their parity checks meet depletion steps and
    melt onsets, which the GPU suite's rules explain (tests/harness.py
    depletion_steps, melt_onsets).  One 384-step launch over 64 x 1024 cells,
    checked the way each rank of those lines checks its own rows."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--ny", "64", "--nx", "1024", "--fuse", "384", "--steps", "768",
           "--warmup", "0", "--no-cpu-baseline", "--no-dropin"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    sp = d["sample_parity"]
    assert sp["steps"] == 384 and sp["cells"] == 65536 and sp["genuine_mismatches"] == 0, sp.get("genuine_examples")
    assert sp["depletion_steps"] > 0 and sp["melt_onsets_explained"] <= sp["melt_onset_budget"]
    assert sp["max_floored_rel"] <= sp["tolerance"] and sp["ok"], sp["max_floored_rel_at"]


def test_gpus_flag_starts_its_ranks_as_a_child(monkeypatch, capsys):
    """`python bench.py --gpus N` run bare (no WORLD_SIZE) starts N ranks as a
    child torch.distributed.run on 127.0.0.1 with the same arguments, relays
    rank 0's JSON line on stdout (anything else on stderr) and returns the
    child's exit code; --gpus 1 and a launcher's own rank run inline."""
    import io
    import subprocess as sp

    bench, args = _args("--gpus", "4", "--steps", "20", "--warmup", "5")
    seen = {}

    class FakeChild:
        def __init__(self, cmd, **kw):
            seen["cmd"], seen["kw"] = cmd, kw
            self.stdout = io.StringIO('warning from a rank\n{"n_gpus": 4}\n')

        def wait(self):
            return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sp, "Popen", FakeChild)
    rc = bench.launch_ranks(args, ["--gpus", "4", "--steps", "20", "--warmup", "5"])
    cmd = seen["cmd"]
    assert rc == 7 and cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert any(a.startswith("--master-port=") for a in cmd)
    assert cmd[-7:] == [str(ROOT / "bench.py"), "--gpus", "4", "--steps", "20", "--warmup", "5"]
    out = capsys.readouterr()
    assert out.out.strip() == '{"n_gpus": 4}' and "warning from a rank" in out.err
    # inline: one GPU, or already a rank of a launcher whose size matches
    _, one = _args("--gpus", "1")
    assert bench.launch_ranks(one, []) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.launch_ranks(args, []) is None


def test_gpus_flag_refuses_a_launcher_of_another_size():
    """Under a launcher whose WORLD_SIZE differs from --gpus the bench exits 2
    before importing torch, instead of printing a line for another N."""
    import os

    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr and r.stdout == ""


@pytest.mark.gpu
def test_bare_gpus_two_runs_two_ranks():
    """`python3 bench.py --gpus 2 ...` with no launcher around it: the bench
    starts its two ranks itself (here both on the one GPU of the box, over
    gloo) and prints one line with n_gpus 2 and a world-2 process group."""
    import os

    env = dict(os.environ, TFG_BENCH_ONE_DEVICE="1", TFG_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--ny", "512", "--nx", "1024", "--steps", "48",
           "--warmup", "24", "--fuse", "24"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["process_group"] == {"backend": "gloo", "world_size": 2}
    assert [x["rows"] for x in d["ranks"]["ranks"]] == [256, 256] and d["sample_parity"]["ok"]


def test_rank_report_names_the_devices_and_the_slowest_rank():
    """The per-rank record a multi-GPU line carries (bench.rank_report): ranks
    in order, the slowest one, max/min span, distinct GPUs; two RCCL ranks on
    one GPU are refused (the one-device gloo rehearsal may share one)."""
    bench, _ = _args()
    rec = lambda r, bus, t: {"rank": r, "local_rank": r, "device": r, "pci_bus_id": bus, "elapsed_s": t}  # noqa: E731
    rep = bench.rank_report([rec(1, "0000:15:00", 2.0), rec(0, "0000:05:00", 1.6)], "nccl")
    assert [r["rank"] for r in rep["ranks"]] == [0, 1] and rep["slowest_rank"] == 1
    assert rep["distinct_gpus"] and rep["n_distinct_gpus"] == 2 and rep["rank_time_max_over_min"] == 2.0 / 1.6
    shared = [rec(0, "0000:05:00", 1.0), rec(1, "0000:05:00", 1.0)]
    assert not bench.rank_report(shared, "gloo")["distinct_gpus"]
    with pytest.raises(RuntimeError):
        bench.rank_report(shared, "nccl")


@pytest.mark.gpu
def test_multi_rank_line_is_self_verifying():
    """The N > 1 path, rehearsed on one GPU (two ranks over gloo, both on
    cuda:0): the JSON names the process group's backend and size as
    torch.distributed sees them and every rank's device, PCI bus id and launch
    times, so a driver N = 2 / 4 / 8 line shows which GPUs ran and which rank
    set the pace."""
    import os

    env = dict(os.environ, TFG_BENCH_ONE_DEVICE="1", TFG_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29531", str(ROOT / "bench.py"), "--gpus", "2", "--ny", "512", "--nx", "1024",
           "--steps", "48", "--warmup", "24", "--fuse", "24"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["process_group"] == {"backend": "gloo", "world_size": 2}
    rep = d["ranks"]
    assert [x["rank"] for x in rep["ranks"]] == [0, 1] and rep["slowest_rank"] in (0, 1)
    assert [x["rows"] for x in rep["ranks"]] == [256, 256] and rep["rank_time_max_over_min"] >= 1.0
    for x in rep["ranks"]:
        assert x["pci_bus_id"] and x["device"] == 0 and x["launch_ms_min"] <= x["launch_ms_mean"] <= x["launch_ms_max"]
    assert rep["n_distinct_gpus"] == 1 and not rep["distinct_gpus"]  # both ranks on the one GPU of the box
    # every rank checked its OWN rows against the oracle (global row offsets), folded into the line's parity
    for x in rep["ranks"]:
        sp = x["sample_parity"]
        assert sp["ok"] and sp["global_rows"][0] == x["row0"] and sp["genuine_mismatches"] == 0
        assert sp["steps"] == 24 and sp["launch_steps"] == [1, 24]
    assert d["sample_parity"]["ok"] and d["sample_parity"]["ranks_checked"] == [0, 1]


def _agree_worker(rank, world, port, depths, out):
    import os

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench, _ = _args()
    try:
        out[rank] = bench.agree_on_depth(depths[rank], True, torch, dist, 0, "gloo")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("depths,want", [((384, 256), 256), ((384, 0), 0), ((0, 128), 0)])
def test_depth_agreement_completes_when_a_rank_cannot_allocate(depths, want):
    """agree_on_depth: every rank reaches the one all-reduce, a rank
    that could create no engine joining with 0; all ranks then see the minimum
    (0: every rank stops with an error instead of waiting for the failed one
    until the process-group timeout).  gloo, world size 2, on CPU."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.Manager().dict()
    mp.spawn(_agree_worker, args=(2, port, depths, out), nprocs=2, join=True)
    assert dict(out) == {0: want, 1: want}
