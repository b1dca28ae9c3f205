"""bench.py keeps the driver's contract: one JSON line on stdout with the
metric, value, roofline and cpu_baseline objects (small workload)."""

import json
import subprocess
import sys

import pytest

from tests.harness import ROOT

pytestmark = pytest.mark.gpu


def test_bench_prints_one_json_line_with_the_contract_keys():
    cmd = [sys.executable, str(ROOT / "bench.py"), "--ny", "256", "--nx", "1024", "--steps", "48", "--warmup", "24",
           "--fuse", "24", "--cpu-cells", "4096", "--cpu-steps", "48", "--parity-cells", "2048", "--parity-steps", "24",
           "--numpy-cells", "1024", "--no-pcie"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 48 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["config"]["workload"] and d["dtype"] == "f32" and d["scaling"] == "weak"
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["sample"]
    sp = d["sample_parity"]
    assert sp["genuine_mismatches"] == 0 and sp["max_floored_rel"] <= sp["tolerance"]
