"""bench.py's output contract (the driver parses ONE JSON line per run): a short default-config
run at N=1 -- the metric / config of BASELINE.json, the roofline object with a live measurement
(achieved / peak = frac, HBM traffic from the committed PMC summary), whole-job throughput
consistent with ms_per_step, and the DDIM legs -- so a change to the bench cannot silently drop a
field the round-end run needs."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    log = tmp_path / "bench.log"
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--skip-cpu", "--ddim-steps", "20"]
    with open(log, "w") as fh:
        r = subprocess.run(cmd, cwd=REPO, stdout=fh, stderr=subprocess.STDOUT, timeout=600)
    out = open(log).read()
    assert r.returncode == 0, out[-3000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"].startswith("training imgs/sec") and base["metric"].startswith(d["metric"][:20])
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["unit"] == "imgs/s"
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert "workload" in d["config"] and d["config"]["global_batch"] == 128
    # value = whole-job images / timed seconds
    assert abs(d["value"] - 128 * 1000.0 / d["ms_per_step"]) / d["value"] < 1e-6
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] in ("GB/s", "TFLOP/s")
    assert 0 < rf["achieved"] < rf["peak"] and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert rf["traffic"] is None or rf["traffic"] > 0
    for k in ("ddim_steps_per_sec", "ddim_steps_per_sec_b128"):
        assert d[k]["value"] > 0, k
