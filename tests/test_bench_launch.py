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


def test_self_launch_hung_rank_hits_the_wall_clock_bound():
    """A rank that never reaches the next collective (PPO_BENCH_LAUNCH_CHECK_HANG_RANK) leaves the
    other blocked in it: the launcher's bound (PPO_BENCH_RANK_TIMEOUT) terminates both, prints ONE
    JSON line naming the ranks still alive, and exits 124."""
    p = _run(2, PPO_BENCH_LAUNCH_CHECK_HANG_RANK="1", PPO_BENCH_RANK_TIMEOUT="8")
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert "error" in rec and rec["value"] is None
    assert rec["alive_ranks"] == [0, 1], rec
    assert "still running" in p.stderr


def test_self_launch_capture_failure_on_one_rank_falls_back_on_every_rank():
    """The update-loop capture fails on rank 1 only: both ranks agree (DataParallel.capture_agreed),
    both retire the native communicator and run the same eager exchanges, and the replicas end
    bitwise equal; the line's ``comm`` reports the exchange as it then runs."""
    for fail in ("1", "0"):
        p = _run(2, PPO_BENCH_LAUNCH_CHECK_CAPTURE_FAIL_RANK=fail)
        assert p.returncode == 0, p.stderr[-2000:]
        rec = json.loads(p.stdout.strip().splitlines()[-1])
        cap = rec["capture"]
        assert cap["fallback"] and cap["native_retired"] and cap["replicas_bitwise_equal"], rec
        assert rec["comm"] == {"backend": "gloo", "native": False, "nranks": 2, "rank": 0}, rec


def test_self_launch_capture_success_keeps_the_native_path():
    """No rank fails (fail rank outside the world): no fallback, the stand-in stays attached."""
    p = _run(2, PPO_BENCH_LAUNCH_CHECK_CAPTURE_FAIL_RANK="7")
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert not rec["capture"]["fallback"] and not rec["capture"]["native_retired"]
    assert rec["capture"]["replicas_bitwise_equal"]
