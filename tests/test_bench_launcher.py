"""bench.py --gpus N starts its own N workers (CPU: the launcher and the distributed timing
harness over gloo, no GPU work), and refuses to report N GPUs it does not have."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "GPMDM_BENCH_BACKEND",
              "GPMDM_BENCH_LAUNCHER", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    return env


def test_self_launch_two_ranks_prints_one_line():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--plumbing-check", "--launch-timeout", "120", "--collective-timeout", "60"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["world_size_backend"] == 2
    assert rec["backend"] == "gloo"
    assert rec["launcher"] == "bench.py"
    assert rec["steps"] == 3 and rec["warmup"] == 1


def test_chatty_ranks_do_not_stall_the_launch(tmp_path):
    # every rank writes > 1 MiB to stdout and stderr before rank 0's JSON line: the launcher
    # drains the pipes while the workers run, keeps per-rank logs, and prints exactly one line
    env = _env()
    env["GPMDM_PLUMBING_SPAM_BYTES"] = str(1_200_000)
    env["GPMDM_BENCH_LOGDIR"] = str(tmp_path)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--plumbing-check", "--launch-timeout", "120", "--collective-timeout", "60"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[:2000]
    assert json.loads(lines[0])["n_gpus"] == 2
    for rank in (0, 1):
        assert (tmp_path / f"rank{rank}.stdout").stat().st_size > 1_000_000
        assert (tmp_path / f"rank{rank}.stderr").stat().st_size > 1_000_000
    assert "[rank 1] NCCL INFO rank 1" in r.stderr


def test_refuses_more_gpus_than_visible():
    # no GPU in this container: --gpus 2 without the rehearsal opt-in must fail, not run one rank
    env = _env()
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr
    assert r.stdout.strip() == ""


def test_flag_and_world_size_must_agree():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing-check"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 2
    assert "disagree" in r.stderr


def test_failing_worker_fails_the_launch():
    # rank 1 exits with status 3 after joining the group; rank 0 would wait at the barrier
    # forever: the launcher stops it and reports the failure
    env = _env()
    env["GPMDM_PLUMBING_FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing-check",
                        "--launch-timeout", "120", "--collective-timeout", "100"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with status 3" in r.stderr
    assert "rank 1 stderr tail" in r.stderr
    assert r.stdout.strip() == ""
