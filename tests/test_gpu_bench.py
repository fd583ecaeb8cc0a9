"""bench.py's JSON contract on the GPU: one line on stdout with the driver's keys, `roofline`
and `cpu_baseline`, for the headline preset (reduced N), config 2 and config 5 (the Gibbs preset,
reduced N) -- the runs the round-end driver and DESIGN.md quote."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline")


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *extra], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]  # the JSON line is the only stdout output
    return json.loads(lines[0])


def _check(d, steps, warmup):
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert 0 < rf["frac"] < 1 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["sample"]


def test_bench_headline_contract(dev):
    d = _run("--steps", "20", "--warmup", "5", "--n", "200000", "--cpu-seconds", "0.3")
    _check(d, 20, 5)
    assert d["unit"] == "locations/s" and d["config"]["m"] == 15 and d["config"]["kind"] == "exponential"
    assert d["bad_rows"] == [-1, -1] and d["cpu_baseline"]["parity_max_rel_dF"] < 1e-10
    # the live kernel time at the driver's --steps 20: at least 5 event-bracketed samples, and the
    # per-launch loop time beside it
    rf = d["roofline"]
    assert rf["kernel_ms_samples"] >= 5 and rf["kernel_ms"] > 0 and rf["kernel_ms_loop_samples"] == 20
    assert rf["kernel_ms_loop"] > 0


def test_bench_config2_contract(dev):
    d = _run("--config", "2", "--steps", "20", "--warmup", "5", "--cpu-seconds", "0.3")
    _check(d, 20, 5)
    assert d["config"]["n_per_gpu"] == 100_000 and d["config"]["kind"] == "matern32"


def test_bench_config5_contract(dev):
    d = _run("--config", "5", "--steps", "5", "--warmup", "2", "--n", "20000", "--cpu-seconds", "0.3")
    _check(d, 5, 2)
    assert d["unit"] == "chain-iterations/s" and d["config"]["chains"] == 1
    b = d["breakdown"]
    assert b["n_colors"] > 0 and b["bf_sweep_ms"] > 0 and b["w_sweep_ms"] > 0  # (no timing bounds: a tiny N)


def test_bench_config5_two_chains_per_gpu(dev):
    d = _run("--config", "5", "--steps", "5", "--warmup", "2", "--n", "20000", "--cpu-seconds", "0",
             "--chains-per-gpu", "2")
    assert d["steps"] == 5 and d["value"] > 0 and d["config"]["chains"] == 2 and d["config"]["chains_per_gpu"] == 2


@pytest.mark.parametrize("mode", ["batched-streams", "batched", "batched-percopy", "streams"])
def test_bench_config5_chain_modes(dev, mode):
    d = _run("--config", "5", "--steps", "4", "--warmup", "2", "--n", "20000", "--cpu-seconds", "0",
             "--chains-per-gpu", "4", "--chain-mode", mode)
    assert d["steps"] == 4 and d["value"] > 0 and d["config"]["chains_per_gpu"] == 4
    assert d["config"]["chain_mode"] == mode
