"""gpr_amd — MI355X-native Gaussian-process regression core (agiger/GPR hot path).

The numerics live in libgprx (gpr_amd/lib/libgprx.so, hand-written gfx950 HIP kernels
behind the C ABI of include/gprx.h).  This package holds the Python binding used by the
tests and bench.py; the C++ host API mirroring the reference classes is in include/gpr/.
"""
from . import kernels
from .kernels import (Gaussian, GaussianExp, White, RationalQuadratic, Periodic, Sum, Product, parse_kernel,
                      general_kernel)
from .gprx import (Context, DeviceArray, Model, GprxError, lib, device_count, unique_id, query_shard, LIB_PATH,
                   runtime_info)

__all__ = ["DeviceArray", "kernels", "Gaussian", "GaussianExp", "White", "RationalQuadratic", "Periodic", "Sum", "Product",
           "parse_kernel", "general_kernel", "Context", "Model", "GprxError", "lib", "device_count", "unique_id", "LIB_PATH",
           "runtime_info"]
