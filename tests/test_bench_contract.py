"""bench.py's contract: the CPU-baseline leg on the host (small sample) and, on the GPU, one short
run of the whole command whose JSON line must carry BASELINE.json's metric, the roofline and the
fields the driver reads."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_cpu_baseline_leg_small_sample():
    import bench
    r = bench.cpu_baseline(10, 0.4, procs=2)
    assert r["kind"] == "port" and r["unit"] == "env-steps/s" and r["cores"] == min(2, bench.host_cores())
    assert set(r["by_window"]) == {"W=5", "W=10"}
    for v in r["by_window"].values():
        assert v["env_steps"] > 0 and v["aggregate"] > 0 and v["per_core_min"] <= v["per_core_max"]
    assert r["value"] == r["by_window"]["W=10"]["aggregate"]
    assert r["config1"]["env_steps_per_s"] > 0


@pytest.mark.gpu
def test_bench_json_line(gpu):
    cmd = [sys.executable, "bench.py", "--steps", "20", "--warmup", "5", "--settle", "60", "--no-cpu-baseline",
           "--policy-steps", "20", "--torch-policy-steps", "5", "--board-steps", "20", "--rollout-steps", "100"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"] and d["unit"] == "env-steps/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 5 and d["scaling"] == "weak"
    assert d["value"] > 1e8 and d["ms_per_step"] > 0 and d["dtype"] == "int16x2+f64" and d["data"] == "synthetic"
    assert d["vs_baseline"] is None and d["config"]["envs_per_gpu"] == 65536 and d["config"]["window"] == 10
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9 and rf["kernel"] == "step2_kernel<10, 13, 5>"
    assert rf["traffic"] is None or rf["traffic"] > 0
    for leg in ("policy_rollout", "fused_rollout", "board_profile"):
        assert d[leg]["value"] > 0, leg
    assert "cpu_baseline" not in d or d["cpu_baseline"] is None
