"""The drop-in boundary: libgprx loads on a GPU-less host and exports every symbol the
public headers declare (include/gprx.h, include/gprx_dev.h).  No compute calls here."""
import ctypes
import os
import re

import pytest

import gpr_amd
from gpr_amd import gprx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gprx_[a-z_0-9]+)\s*\(", text)))


@pytest.mark.parametrize("header", ["gprx.h", "gprx_dev.h"])
def test_header_symbols_exported(header):
    lib = ctypes.CDLL(gprx.LIB_PATH)
    syms = declared_symbols(header)
    assert syms, header
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_lists_all_abi_symbols():
    assert sorted(gprx.EXPORTED) == declared_symbols("gprx.h")


def test_abi_version():
    assert gpr_amd.lib().gprx_abi_version() == 2


def test_struct_layouts_match_header():
    # gprx_knode: int32 op, int32 pad, double p[3] -> 32 bytes; desc: 8 + 32*32
    assert ctypes.sizeof(gprx.KNode) == 32
    assert ctypes.sizeof(gprx.KernelDesc) == 8 + 32 * gprx.MAX_KNODES
    assert ctypes.sizeof(gprx.FitInfo) == 8 * 2 + 4 * 2 + 8 * 3 + 8 * 2 + 4 * 2
    assert ctypes.sizeof(gprx.KStat) == 32 + 8 * 4


def test_no_device_fails_loudly():
    """The product path has no CPU fallback: without a GPU every context creation fails."""
    if gpr_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(gpr_amd.GprxError) as e:
        gpr_amd.Context(0)
    assert "no HIP device" in str(e.value)


def _runtime_in_subprocess(torch_first):
    import json
    import subprocess
    import sys
    code = ("import json, sys\nsys.path.insert(0, %r)\n" % ROOT
            + ("import torch\n" if torch_first else "")
            + "import gpr_amd\ngpr_amd.lib()\nprint(json.dumps(gpr_amd.runtime_info()))\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, check=True)
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_runtime_binding_library_first():
    """libgprx loaded with no PyTorch in the process (bench.py at every N, the two-process tests'
    socket-bootstrapped ranks) binds /opt/rocm's HIP runtime, HSA runtime and RCCL, one copy each."""
    info = _runtime_in_subprocess(False)
    assert info["single_copy"] and not info["torch_loaded_first"], info
    for k in ("libamdhip64", "librccl", "libhsa-runtime64"):
        assert len(info[k]) == 1 and info[k][0].startswith("/opt/rocm"), info


def test_runtime_binding_torch_first():
    """With the PyTorch wheel imported first, libgprx shares the runtime and RCCL torch bundles
    (the loader resolves libgprx's sonames to the objects torch loaded): still ONE copy each."""
    pytest.importorskip("torch")
    info = _runtime_in_subprocess(True)
    assert info["single_copy"] and info["torch_loaded_first"], info
    assert len(info["libamdhip64"]) == 1 and "/torch/lib/" in info["libamdhip64"][0], info


_HC_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
from gpr_amd.hostcoll import SocketGroup
import ctypes
rank, world, port = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
g = SocketGroup(rank, world, port=port, timeout=60)
parts = g.allgather(bytes([rank]) * (rank + 3))
assert parts == [bytes([r]) * (r + 3) for r in range(world)], parts
assert g.max(rank * 1.5) == (world - 1) * 1.5 and g.min(rank) == 0
assert g.broadcast(b"uid" if rank == 0 else None) == b"uid"
fn = g.allgather_fn()
send = (ctypes.c_double * 2)(rank, -rank)
recv = (ctypes.c_double * (2 * world))()
assert fn(None, ctypes.addressof(send), 16, ctypes.addressof(recv)) == 0
assert list(recv) == [v for r in range(world) for v in (float(r), float(-r))]
big = bytes(range(256)) * 40000 if rank == world - 1 else b"x"
assert g.allgather(big)[world - 1] == bytes(range(256)) * 40000
g.barrier()
g.close()
print("ok", rank)
"""


def test_hostcoll_socket_group(tmp_path):
    """gpr_amd.hostcoll (bench.py's and the two-process tests' host collectives): all-gather of
    ragged and 10 MB payloads, max/min, broadcast and the C all-gather callback over 3 processes."""
    import socket
    import subprocess
    import sys
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = str(so.getsockname()[1])
    script = tmp_path / "hc.py"
    script.write_text(_HC_SCRIPT)
    procs = [subprocess.Popen([sys.executable, str(script), ROOT, str(r), "3", port], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(3)]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs


def test_hostcoll_admission_drops_strays():
    """Rank 0 of a SocketGroup drops connections that announce a wrong token, a rank outside
    1..world-1, a rank that already joined, or nothing at all, and keeps waiting for the real
    ranks (a stray connection must not take a slot or hang the group)."""
    import socket
    import struct
    import threading
    from gpr_amd.hostcoll import SocketGroup
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    res = {}

    def hub():
        g = SocketGroup(0, 3, port=port, timeout=60, token="tok")
        res["parts"] = g.allgather(b"zero")
        g.close()

    th = threading.Thread(target=hub)
    th.start()

    def stray(rank, tok, announce=True):
        import time
        for _ in range(200):
            try:
                s = socket.create_connection(("127.0.0.1", port), timeout=5)
                break
            except OSError:
                time.sleep(0.02)
        if announce:
            t = tok.encode()
            s.sendall(struct.pack("<ii", rank, len(t)) + t)
        return s

    strays = [stray(1, "bad"), stray(7, "tok"), stray(-1, "tok"), stray(0, "tok")]
    r1 = SocketGroup(1, 3, port=port, timeout=60, token="tok")
    strays.append(stray(1, "tok"))  # a duplicate of a rank that has joined
    r2 = {}

    def join2():
        g = SocketGroup(2, 3, port=port, timeout=60, token="tok")
        r2["parts"] = g.allgather(b"two")
        g.close()

    t2 = threading.Thread(target=join2)
    t2.start()
    p1 = r1.allgather(b"one")
    t2.join(60)
    th.join(60)
    r1.close()
    for s in strays:
        s.close()
    assert res["parts"] == [b"zero", b"one", b"two"] == p1 == r2["parts"]
