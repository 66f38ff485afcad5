"""bench.py's multi-GPU launcher on CPU (no GPU): `bench.py --gpus N` starts N rank processes
of itself and every rank checks the process group it joined; the gloo selftest workload runs
the same barrier-bracketed timing and max-over-ranks path as the GPU workloads."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_gloo_ranks(n):
    r = _run(["--gpus", str(n), "--workload", "selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["rank_sum"] == n * (n - 1) / 2  # every rank took part in the all-reduce
    assert out["config"]["parallelism"] == f"dp{n}"


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--workload", "selftest"], env_extra={"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "process group has 1 rank" in r.stderr


def test_more_gpus_than_visible_fails_loudly():
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("machine has that many devices")
    r = _run(["--gpus", "64"])
    assert r.returncode == 2
    assert "HIP device(s) visible" in r.stderr


def test_failed_rank_ends_the_run_within_seconds():
    """A rank that dies after joining the process group: the launcher terminates its siblings
    (blocked in the barrier) and returns the failed rank's status, well before any timeout."""
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "3", "--workload", "selftest", "--selftest-fail-rank", "1"],
             env_extra={"TTS_BENCH_PG_TIMEOUT": "120"}, timeout=90)
    took = time.monotonic() - t0
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with status 7" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert took < 60, took


def test_driver_torchrun_form_8_ranks():
    """The driver's N=8 launch, verbatim (torch.distributed.run, one node, 8 processes, master on
    127.0.0.1), on the gloo selftest: one JSON line from rank 0 with every rank in the all-reduce."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "8",
                        "--workload", "selftest"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["rank_sum"] == 28.0 and out["config"]["parallelism"] == "dp8"
