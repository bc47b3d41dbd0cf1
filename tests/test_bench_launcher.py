"""bench.py's own rank launcher (`python bench.py --gpus N` without torchrun):
the rank environment each child gets, and the exit-code handling when a rank
fails (CPU only: the children here are small Python programs, or bench.py
ranks that fail on a host without a GPU)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ENV_DUMP = ("import json, os, sys; keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', "
            "'MASTER_PORT', 'KEEP'); json.dump({k: os.environ.get(k) for k in keys}, "
            "open(os.path.join(sys.argv[1], 'rank%s.json' % os.environ['RANK']), 'w'))")


def test_spawn_ranks_env(tmp_path):
    env = dict(os.environ, KEEP="yes")
    env.pop("WORLD_SIZE", None)
    rc = bench.spawn_ranks(3, [sys.executable, "-c", ENV_DUMP, str(tmp_path)], env=env, port=29777)
    assert rc == 0
    for r in range(3):
        d = json.load(open(tmp_path / f"rank{r}.json"))
        assert d == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "3", "LOCAL_WORLD_SIZE": "3",
                     "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29777", "KEEP": "yes"}


def test_spawn_ranks_failure_ends_the_others():
    # rank 1 fails at once; rank 0 would wait 120 s for a peer that is gone
    child = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(120)"
    t0 = time.time()
    rc = bench.spawn_ranks(2, [sys.executable, "-c", child])
    assert rc == 3
    assert time.time() - t0 < 30


def test_spawn_ranks_signal_death_is_nonzero():
    child = "import os, signal; os.kill(os.getpid(), signal.SIGKILL) if os.environ['RANK'] == '0' else None"
    assert bench.spawn_ranks(2, [sys.executable, "-c", child]) == 128 + 9


def test_bench_gpus2_without_torchrun_fails_loudly_without_a_gpu():
    """On this GPU-less host both ranks fail to find a device: the launcher
    must return non-zero (not hang, not print a line)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-secondary"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_sigterm_to_the_launcher_ends_its_ranks(tmp_path):
    """A SIGTERM to the launcher (a driver's timeout) reaches the ranks: the
    launcher exits 128 + 15 and no rank outlives it."""
    import signal

    child = ("import os, sys, time; open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write(str(os.getpid())); "
             "time.sleep(120)")
    prog = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(2, [sys.executable, '-c', %r, %r]))" % (ROOT, child, str(tmp_path)))
    p = subprocess.Popen([sys.executable, "-c", prog])
    t0 = time.time()
    while len(os.listdir(tmp_path)) < 2 and time.time() - t0 < 60:
        time.sleep(0.1)
    pids = [int(open(tmp_path / f).read()) for f in os.listdir(tmp_path)]
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    time.sleep(0.5)
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, pid
