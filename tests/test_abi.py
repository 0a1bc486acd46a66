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
