"""The C++ host API (include/gpr/*.h, gpr_amd/host/) — GaussianProcess<T>, Kernel<T>,
KernelFactory<T>, Likelihood<T>, MatrixIO — driven through its two test executables
(tests/cpp/*.cpp, built by `make cpptests`).

* host_cpu_test: kernels / factory / file format on the host, and that a GaussianProcess
  throws when no GPU is visible (no CPU fallback).
* gp_host_test (-m gpu): the reference's GaussianProcessTest 1-7 and IOTest 1-3 with the
  reference's thresholds, plus a likelihood gradient consistency check, the sparse GP and
  PosteriorProcessTest 1-2 (Predict / operator() from 8 threads at once, on a fresh and on a
  loaded GP), and a user Kernel<T> subclass with no device form (host-evaluated through its
  virtual operator(), factored on the device), all running their fits on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gpr_amd", "lib")


def _run(exe, *args, timeout=600):
    path = os.path.join(LIB, exe)
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", ROOT, "cpptests"], check=True, timeout=900)
    r = subprocess.run([path, *args], capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith(("PASS", "FAIL"))]
    return r.returncode, lines, r.stdout + r.stderr


def _gpu_visible():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_host_cpu():
    args = [] if _gpu_visible() else ["--no-device"]
    rc, lines, out = _run("host_cpu_test", *args)
    assert rc == 0, out
    assert len(lines) == 5 + len(args), out


@pytest.mark.gpu
def test_host_gpu_reference_scenarios():
    rc, lines, out = _run("gp_host_test")
    assert rc == 0, out
    assert len(lines) == 21 and all(l.startswith("PASS") for l in lines), out
