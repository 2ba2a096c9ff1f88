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


def test_board_cpu_baseline_leg_small_sample():
    """The createBoard CPU baseline (oracle/py_board.py on the host cores) beside the board leg."""
    import bench
    r = bench.board_cpu_baseline(0.4, procs=2)
    assert r["kind"] == "port" and r["unit"] == "env-steps/s" and r["cores"] == min(2, bench.host_cores())
    assert r["env_steps"] > 0 and r["value"] > 0 and r["per_core_min"] <= r["per_core"] <= r["per_core_max"]


@pytest.mark.gpu
def test_bench_json_line(gpu):
    cmd = [sys.executable, "bench.py", "--steps", "20", "--warmup", "5", "--settle", "60", "--no-cpu-baseline",
           "--policy-steps", "20", "--torch-policy-steps", "5", "--board-steps", "20", "--rollout-steps", "100",
           "--config2-steps", "50", "--config4-steps", "20", "--large-steps", "20", "--from-reset-steps", "20",
           "--blocks-launches", "8", "--eager-steps", "50", "--shard-steps", "20"]
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
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9 and rf["kernel"] == "step2_kernel<10, 13, 5, true>"
    assert rf["traffic"] is None or rf["traffic"] > 0
    for leg in ("policy_rollout", "fused_rollout", "board_profile", "config2", "config4", "large_batch", "from_reset"):
        assert d[leg]["value"] > 0, leg
    assert d["config2"]["envs_per_gpu"] == 4096 and d["config2"]["window"] == 5
    c4 = d["config4"]
    assert c4["global_envs"] == 262144 and c4["envs_per_rank"] == 262144 and c4["window"] == 10
    assert c4["scaling"] == "strong" and c4["roofline"]["bytes_per_env_step"] == 390 and c4["episodes"]["episodes"] > 0
    assert d["config2"]["roofline"]["bytes_per_env_step"] == 315
    assert d["large_batch"]["envs_per_gpu"] == 1 << 20 and d["large_batch"]["steps"] == 20
    assert d["from_reset"]["untimed_steps_since_reset"] == 0
    for n in (65536, 1 << 20):
        for kind, rowb in (("u8", 29), ("f32", 116)):
            leg = d["blocks_obs"][f"envs_{n}"][kind]
            assert leg["value"] > 0 and leg["bytes_per_env"] == 8 + 4 * 18 + rowb and leg["roofline"]["frac"] > 0
    assert "cpu_baseline" not in d or d["cpu_baseline"] is None
    # config 4's per-rank shards (the 1 -> 8 GPU prediction) and the eager drop-in leg
    sh = c4["shards"]["by_gpus"]
    assert [r["gpus"] for r in sh] == [2, 4, 8] and [r["envs_per_rank"] for r in sh] == [131072, 65536, 32768]
    assert [r["env_offset"] for r in sh] == [131072, 196608, 229376]
    for r in sh:
        assert r["kernel_us_mean"] > 0 and r["projected_node_env_steps_per_s"] > 0 and 0 < r["moved_frac"] <= 1
    # the headline's autoreset pool, and the fused mode at config 2 and at config 4's 8-GPU shard
    ap = rf["autoreset_pool"]
    assert ap["bytes"] > 0 and ap["period"] > 0 and ap["fill_kernel"] == "pool_fill_kernel<10, 13, 5>"
    assert d["config2"]["autoreset_pool"]["fill_kernel"] == "pool_fill_kernel<5, 13, 5>"
    fr = d["fused_rollout"]
    assert fr["config2"]["kernel"] == "rolloutw_kernel<5, 13, 5, 8>" and fr["config2"]["envs"] == 4096
    assert fr["shard_32768"]["kernel"] == "rollout_kernel<10, 13, 5, 0, 1, 10>" and fr["shard_32768"]["envs"] == 32768
    assert fr["shard_32768"]["env_offset"] == 229376 and fr["config2"]["window"] == 5
    for sub in (fr["config2"], fr["shard_32768"]):
        assert sub["kernel_us_per_step"] > 0 and sub["value"] > 0 and sub["bytes_per_env_step"] > 0
        assert 0 < sub["moved_frac"] <= 1 and sub["moved_source"]
    eg = d["eager_step"]
    assert eg["value"] > 0 and eg["host_us_per_step_call"] > 0 and eg["gpu_us_per_iteration"] > 0 and eg["steps"] == 50
    check_bench_sources(d)


def _walk(x, path=""):
    if isinstance(x, dict):
        yield path, x
        for k, v in x.items():
            yield from _walk(v, f"{path}.{k}")
    elif isinstance(x, list):
        for i, v in enumerate(x):
            yield from _walk(v, f"{path}[{i}]")


def check_bench_sources(d, fused_sizes=True):
    """Every roofline-bearing leg reports moved_frac <= 1 (the bytes actually moved: PMC, else the
    engine's be_step_bytes); a frac above 1 (SURVEY's 390-B figure) carries frac_note; and every
    committed profile a leg cites is the NEWEST round's file of that name for that kernel and size.
    fused_sizes: the fused rollout's config-2 / 32 768-env sub-lines are required (round 6 on)."""
    import glob
    import re
    want = ["roofline", "config2.roofline", "config4.roofline", "large_batch.roofline", "from_reset.roofline",
            "cold_action_rows", "fused_rollout", "board_profile.roofline", "board_profile.fused.roofline",
            "policy_rollout.roofline", "blocks_obs.envs_65536.u8.roofline"]
    if fused_sizes:
        want += ["fused_rollout.config2", "fused_rollout.shard_32768"]
    seen = {p.lstrip("."): x for p, x in _walk(d)}
    for w in want:
        assert w in seen and "moved_frac" in seen[w], w
    for p, x in seen.items():
        if "moved_frac" in x:
            assert 0 < x["moved_frac"] <= 1.0, (p, x["moved_frac"])
        if (x.get("frac") or 0) > 1.0 and "bound" in x:
            assert "frac_note" in x, p
        for k, v in x.items():
            if not (k.endswith("_source") and isinstance(v, str) and v.startswith("committed profile ")):
                continue
            rel = v[len("committed profile "):]
            m = re.match(r"profiles/r(\d\d)_(.+)$", rel)
            assert m, (p, k, v)
            named = json.load(open(os.path.join(ROOT, rel)))
            kern, units = named.get("kernel"), named.get("units_per_dispatch", named.get("envs"))
            for other in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_" + m.group(2))):
                rnd = int(os.path.basename(other)[1:3])
                if rnd > int(m.group(1)):
                    o = json.load(open(other))
                    assert not (o.get("kernel") == kern and o.get("units_per_dispatch", o.get("envs")) == units), \
                        (p, k, v, "newer:", other)


def test_bench_source_check_on_the_committed_line():
    """check_bench_sources on the round's committed bench line, where one exists (CPU only)."""
    lines = sorted(glob_bench_lines())
    if not lines:
        pytest.skip("no committed bench line with the moved_frac fields yet")
    d = json.load(open(lines[-1]))
    check_bench_sources(d, fused_sizes=int(os.path.basename(lines[-1])[1:3]) >= 6)


def glob_bench_lines():
    import glob
    out = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench.json")):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        if isinstance(d, dict) and "moved_frac" in (d.get("roofline") or {}):
            out.append(f)
    return out


_ONLY_HEADLINE = ["--no-cpu-baseline", "--policy-steps", "0", "--board-steps", "0", "--rollout-steps", "0",
                  "--cold-steps", "0", "--config2-steps", "0", "--config4-steps", "0", "--large-steps", "0",
                  "--from-reset-steps", "0", "--blocks-launches", "0"]


def _bench_line(args, timeout=110):
    r = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]      # rank 0 only
    return json.loads(lines[0])


def test_bench_gpus_mismatch_refused():
    """--gpus N inside a launch of another world size fails loudly (no silent one-rank run)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *_ONLY_HEADLINE], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in r.stderr


@pytest.mark.gpu
def test_bench_multi_rank_gloo(gpu):
    """`bench.py --gpus 2` starts two ranks itself (a child torch.distributed.run; gloo here, so
    both share the one GPU) and runs bench.py's own multi-rank path end to end: barrier + max
    over ranks of the timed region, the all_gather of the stats records, the device count.  The
    two ranks' combined episodes equal a one-rank run over the same global env ids."""
    common = ["--steps", "20", "--warmup", "5", "--settle", "60", *_ONLY_HEADLINE]
    d2 = _bench_line(["--gpus", "2", "--dist-backend", "gloo", "--envs", "4096", *common])
    assert d2["ranks"] == 2 and d2["n_gpus"] == 1
    assert d2["config"]["envs_per_gpu"] == 4096 and d2["config"]["global_envs"] == 8192
    assert d2["value"] > 0 and d2["roofline"]["kernel"] == "step2_kernel<10, 13, 5, true>"
    # N > 1 explains itself: every rank's own timing, GPU and stats exchange; the line's ms_per_step is
    # the slowest rank's
    rows = d2["per_rank"]
    assert sorted(r["rank"] for r in rows) == [0, 1] and d2["dist_backend"] == "gloo" and d2["rccl_world_size"] is None
    for r in rows:
        assert r["kernel_us_mean"] > 0 and r["ms_per_step"] > 0 and r["stats_all_gather_us"] > 0
        assert r["device_uuid"] and r["envs"] == 4096 and r["env_offset"] == 4096 * r["rank"]
    assert max(r["ms_per_step"] for r in rows) == d2["ms_per_step"]
    d1 = _bench_line(["--gpus", "1", "--envs", "8192", *common])
    assert d1["ranks"] == 1 and d1["config"]["global_envs"] == 8192
    e1, e2 = d1["episodes"], d2["episodes"]
    assert e1["episodes"] > 0 and e2["episodes"] == e1["episodes"]
    assert e2["min_return"] == e1["min_return"] and e2["max_return"] == e1["max_return"]
    assert e2["mean_return"] == pytest.approx(e1["mean_return"], rel=1e-12)
    assert e2["mean_length"] == pytest.approx(e1["mean_length"], rel=1e-12)


@pytest.mark.gpu
def test_bench_config4_split_gloo(gpu):
    """BASELINE config 4 as stated: a fixed 262 144-env batch split over the ranks.  Under
    `--gpus 2` each rank steps its contiguous half (131 072 global ids); the leg reports the
    global batch, and the ranks' all_gathered episodes equal those of one rank stepping the
    whole batch (the same global ids, so the same trajectories)."""
    only_c4 = [a for a in _ONLY_HEADLINE]
    only_c4[only_c4.index("--config4-steps") + 1] = "20"
    common = ["--steps", "5", "--warmup", "2", "--settle", "60", "--envs", "4096", *only_c4]
    d2 = _bench_line(["--gpus", "2", "--dist-backend", "gloo", *common], timeout=200)
    d1 = _bench_line(["--gpus", "1", *common], timeout=200)
    c2, c1 = d2["config4"], d1["config4"]
    assert c2["global_envs"] == c1["global_envs"] == 262144
    assert c2["envs_per_rank"] == 131072 and c1["envs_per_rank"] == 262144 and c2["ranks"] == 2
    assert c2["steps"] == c1["steps"] == 20 and c2["value"] > 0 and c1["value"] > 0
    rows = c2["per_rank"]                      # per-rank shard timing (the leg's ms_per_step is the max)
    assert sorted(r["rank"] for r in rows) == [0, 1] and "per_rank" not in c1
    assert [r["env_offset"] for r in sorted(rows, key=lambda r: r["rank"])] == [0, 131072]
    assert all(r["kernel_us_mean"] > 0 and r["stats_all_gather_us"] > 0 and r["device_uuid"] for r in rows)
    assert max(r["ms_per_step"] for r in rows) == c2["ms_per_step"]
    e1, e2 = c1["episodes"], c2["episodes"]
    assert e1["episodes"] > 0 and e2["episodes"] == e1["episodes"]
    assert e2["min_return"] == e1["min_return"] and e2["max_return"] == e1["max_return"]
    assert e2["mean_return"] == pytest.approx(e1["mean_return"], rel=1e-12)
    assert e2["mean_length"] == pytest.approx(e1["mean_length"], rel=1e-12)


@pytest.mark.gpu
def test_bench_rccl_one_rank(gpu):
    """The RCCL path of bench.py (the driver's torchrun form, backend nccl = RCCL): under
    torch.distributed.run with one rank the process group comes up and every collective of the
    timed regions runs (barriers, the max-over-ranks all_reduce, the stats all_gather, the device
    all_gather_object) -- the multi-GPU code path minus the other ranks, which one GPU cannot host."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           f"--master-port={port}", "bench.py", "--gpus", "1", "--dist-backend", "nccl", "--steps", "20", "--warmup", "5",
           "--settle", "60", "--rollout-steps", "100", "--policy-steps", "20", "--torch-policy-steps", "0",
           "--board-steps", "20", "--cold-steps", "0", "--config2-steps", "20", "--config4-steps", "20",
           "--large-steps", "0",
           "--from-reset-steps", "0", "--blocks-launches", "0", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["ranks"] == 1 and d["n_gpus"] == 1 and d["value"] > 0 and d["episodes"]["episodes"] >= 0
    for leg in ("policy_rollout", "fused_rollout", "board_profile", "config2", "config4"):
        assert d[leg]["value"] > 0, leg
    assert d["config4"]["global_envs"] == 262144 and d["config4"]["episodes"]["episodes"] > 0
