"""bench.py keeps the driver's JSON contract: a short run on one GPU prints one
line with the required keys, and the multi-stream rollout steps count exactly
the env-steps the games played (the histogram's ply total)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline"}


def _run(extra, env_extra=None, secondary=False):
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--games", "65536",
                        "--prewarm-ms", "0"] + ([] if secondary else ["--no-secondary"]) + extra,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("streams", [1, 2])
def test_bench_rollout_line(streams):
    out = _run(["--streams", str(streams)])
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["config"]["streams"] == streams
    assert out["unit"] == "env-steps/s" and out["value"] > 0
    # 65536 random games average ~60.4 plies
    assert 59.5 < out["config"]["env_steps_per_game"] < 61.5
    rf = out["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["launch_ms"] > 0


@pytest.mark.gpu
def test_bench_rollout_rccl_path_one_rank():
    """The N>1 code path (RCCL barrier, per-step async histogram all-reduce on
    each step's stream, max over ranks) at world size 1."""
    out = _run(["--allreduce", "async"], {"BENCH_FORCE_DIST": "1", "RANK": "0", "LOCAL_RANK": "0",
                                           "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
                                           "MASTER_PORT": "29531"})
    assert 59.5 < out["config"]["env_steps_per_game"] < 61.5


@pytest.mark.gpu
def test_bench_dist_secondary_step_lines_one_rank():
    """The N>1 secondary lines (config 2's step over each rank's own mid-game
    positions, barrier + max-over-ranks timing) at world size 1."""
    out = _run([], {"BENCH_FORCE_DIST": "1", "RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29532"}, secondary=True)
    sec = out["secondary"]
    assert set(sec) == {"step_steady_16M", "step_65536"}
    for name, n in (("step_steady_16M", 1 << 24), ("step_65536", 65536)):
        s = sec[name]
        assert s["n_gpus"] == 1 and s["batch"] == n and s["value"] > 0
        assert 0 < s["roofline"]["frac"] < 1


@pytest.mark.gpu
def test_bench_two_ranks_line_the_driver_parses():
    """bench.py's N>1 line end to end at world size 2 (torch.distributed.run,
    both ranks on this box's GPU, the collectives over gloo on host copies):
    one JSON line from rank 0 with n_gpus 2, disjoint per-rank game ids,
    every game of both ranks counted once, and the reduced env-steps and
    win/loss/draw counts equal to one process playing the same global ids."""
    import socket

    import torch

    from subproc_amd import ops
    from subproc_amd.dist import bench_game_id0
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    steps, warmup, games = 3, 1, 65536
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", str(steps), "--warmup", str(warmup), "--games", str(games), "--prewarm-ms", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert REQUIRED <= set(out)
    cfg = out["config"]
    assert out["n_gpus"] == 2 and cfg["world_size"] == 2 and cfg["parallelism"] == "dp2"
    assert cfg["workload"].startswith("config4") and out["scaling"] == "weak"
    assert cfg["games_counted"] == steps * 2 * games and cfg["global_batch"] == 2 * games
    per = cfg["game_ids"]["per_rank"]
    spans = sorted(tuple(x) for rr in per.values() for x in rr)
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))  # disjoint id ranges
    assert per["0"][0] == [bench_game_id0(warmup, 0, 2, games), bench_game_id0(warmup, 0, 2, games) + games]
    assert per["1"][0] == [bench_game_id0(warmup, 1, 2, games), bench_game_id0(warmup, 1, 2, games) + games]
    # the same global ids in one process
    hist = torch.zeros(133, dtype=torch.int64, device="cuda")
    for s_ in range(warmup, warmup + steps):
        for rank in range(2):
            ops.rollout(games, 0x5EED, bench_game_id0(s_, rank, 2, games), hist=hist, device="cuda",
                        want_boards=False, want_diff=False, want_plies=False)
    h = hist.cpu().tolist()
    assert cfg["env_steps"] == h[132] and cfg["black_white_draw"] == h[129:132]
    sec = out["secondary"]
    assert set(sec) == {"step_steady_16M", "step_65536"}
    for name in sec:
        assert sec[name]["n_gpus"] == 2 and sec[name]["value"] > 0


@pytest.mark.gpu
def test_bench_gpus2_plain_command():
    """Exactly `python bench.py --gpus 2 --steps 3 --warmup 1` (no torchrun: the
    bench starts its two ranks itself), both ranks on this box's one GPU with
    the collectives over gloo: one line, n_gpus 2, every game counted once."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == 2 and out["config"]["world_size"] == 2
    assert out["config"]["games_counted"] == 2 * 3 * (1 << 20)
