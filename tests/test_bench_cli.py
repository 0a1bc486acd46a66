"""bench.py's process contract on the CPU (no GPU here): `--gpus N` with no launcher starts N
ranks itself and fails as a whole when a rank fails; a launcher's WORLD_SIZE must agree with
--gpus.  The GPU form (two spawned ranks sharing one GPU) is
tests/test_gpu_dist.py::test_bench_spawns_ranks_without_launcher."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--steps", "1", "--warmup", "0", "--ntrain", "256", "--configs", "0", "--lml", "0", "--build-iters", "0",
         "--cpu-n", "0", "--predict-q", "0", "--variance-q", "0", "--cpu-lml-ns", "", "--cpu-predict-q", "0"]


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + QUICK, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 1" in r.stderr


def test_spawned_ranks_fail_together_without_gpu():
    """Two ranks spawned by bench.py itself (no WORLD_SIZE in the environment); with no GPU here
    every rank's context creation fails, and the parent must return non-zero promptly, having
    printed no JSON line, instead of hanging on the rank that is left."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GPRX_BENCH_TIMEOUT_S"] = "240"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + QUICK, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert time.monotonic() - t0 < 240
