"""`--gpus N` launches N ranks itself (rdeic_amd/launch.py): one process per rank,
rank 0 prints the one line, a failing rank fails the job, and a WORLD_SIZE that disagrees with
--gpus is refused. CPU only (gloo stub worker)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "stubs", "launch_stub.py")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in
           ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    return env


def _run(args, env=None, timeout=180):
    return subprocess.run([sys.executable, STUB] + args, capture_output=True, text=True, timeout=timeout,
                          env=env or _env())


def test_launcher_starts_three_ranks_one_line():
    r = _run(["--gpus", "3"])
    assert r.returncode == 0, r.stderr[-2000:]
    # stdout carries rank 0's one line and nothing else (gloo's own "[Gloo] Rank i is connected" lines
    # are routed to stderr by parallel.init_from_env)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3
    assert d["ranks"] == [0, 1, 2] and d["local_ranks"] == [0, 1, 2] and d["lws"] == [3, 3, 3]


def test_launcher_fails_when_a_rank_fails():
    r = _run(["--gpus", "2", "--fail-rank", "1"])
    assert r.returncode != 0
    assert "rank 1 exited with status 3" in r.stderr


def test_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = _run(["--gpus", "3"], env=env)
    assert r.returncode == 2
    assert "disagrees with --gpus 3" in r.stderr


def test_bench_refuses_more_gpus_than_visible():
    """No GPU here: bench.py --gpus 2 refuses before any GPU work instead of measuring one rank."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=180, env=_env())
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""
