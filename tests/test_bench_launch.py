"""bench.py --gpus N started as a plain process launches its own N rank processes (the driver's
scaling run calls ``python3 bench.py --gpus N`` without torch.distributed.run).  On CPU the
ranks run the launcher plumbing only (PPO_BENCH_LAUNCH_CHECK=1: gloo rendezvous, barrier, max
over ranks, rank 0's JSON line); the GPU rehearsal of the full workload is in
tests/test_gpu_distributed.py."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(PPO_BENCH_LAUNCH_CHECK="1", **env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                           "--steps", "2", "--warmup", "1"], env=e, capture_output=True,
                          text=True, timeout=120)


def test_self_launch_two_ranks_prints_one_line():
    p = _run(2)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1


def test_self_launch_four_ranks():
    p = _run(4)
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 4


def test_self_launch_failing_rank_fails_the_run():
    p = _run(2, PPO_BENCH_LAUNCH_CHECK_FAIL_RANK="1")
    assert p.returncode != 0
    assert "failed" in p.stderr
