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


BENCH_STUB = os.path.join(ROOT, "tests", "stubs", "bench_stub.py")


def test_config4_command_eight_ranks():
    """Config 4's exact command (`bench.py --gpus 8 --global-batch 128 --bpp-sweep 0.04,0.08,0.12`) through
    bench.py's own parser, launcher, sharding and sweep handling (gloo stub step): 8 ranks, one line,
    16 images per rank in global order, and the headline point (0.08, index 1: not the first point; the
    r04 sweep crashed there) is the only one that keeps its output images."""
    r = subprocess.run([sys.executable, BENCH_STUB, "--gpus", "8", "--global-batch", "128",
                        "--bpp-sweep", "0.04,0.08,0.12"], capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["global_batch"] == 128
    assert d["targets"] == [0.04, 0.08, 0.12] and d["main_i"] == 1
    assert d["images_per_point"] == [128, 128, 128]
    assert d["image_order"] == list(range(128))
    assert d["rank_of_image"] == [g // 16 for g in range(128)]  # 16 images per rank, contiguous shards
    assert d["out_kept"] == [False, True, False]
    assert d["rate_gains"][0] < d["rate_gains"][1] < d["rate_gains"][2]


def test_torchrun_form_without_gpus_flag():
    """`torch.distributed.run --nproc-per-node N bench.py` without --gpus: the rank takes WORLD_SIZE from the
    environment (the --gpus default of 1 used to refuse it)."""
    from rdeic_amd import launch
    env = _env()
    env.update(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    old = {k: os.environ.get(k) for k in env}
    try:
        os.environ.update({k: env[k] for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
        assert launch.role(None) == "rank"
        assert launch.role(4) == "rank"
    finally:
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            if old[k] is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = old[k]
