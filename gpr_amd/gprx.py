"""ctypes binding of libgprx (include/gprx.h) — the Python face of the drop-in boundary.

This module is the binding a Python caller (tests, bench.py) uses; the C++ host API in
include/gpr/ binds the same symbols natively.  There is no CPU fallback: if the HIP
library or a GPU is missing every compute call raises GprxError.
"""
import ctypes
import os

import numpy as np

from .kernels import as_node

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPRX_LIB_OVERRIDE") or os.path.join(_HERE, "lib", "libgprx.so")  # override: dev experiments only

GPRX_F32 = 0
GPRX_F64 = 1
MAX_KNODES = 32
MAX_KPARAMS = 48
UNIQUE_ID_BYTES = 128

FIT_DEFAULT = 0
FIT_NO_LU_FALLBACK = 1
FIT_DISTRIBUTED = 2
FIT_FORCE_LU = 8
FIT_F32_NO_REFINE = 4
LML_GRAD = 1
LML_COMPAT = 2
LML_DISTRIBUTED = 4
LML_FORCE_LU = 8

STATUS = {0: "OK", 1: "NONFINITE", 2: "NOT_SPD", 3: "SINGULAR", 4: "DIM", 5: "HIP", 6: "RCCL", 7: "OOM",
          8: "ARG", 9: "STATE", 10: "NO_DEVICE"}

# Every symbol include/gprx.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "gprx_abi_version", "gprx_device_count", "gprx_ctx_create", "gprx_dist_unique_id", "gprx_ctx_create_dist",
    "gprx_ctx_create_peer",
    "gprx_ctx_destroy", "gprx_last_error", "gprx_model_create", "gprx_model_destroy", "gprx_model_set_data",
    "gprx_model_set_kernel", "gprx_model_set_noise", "gprx_model_fit", "gprx_model_get_alpha",
    "gprx_model_set_alpha",
    "gprx_model_predict", "gprx_model_posterior_cov", "gprx_model_core_matrix", "gprx_model_lml",
    "gprx_kernel_matrix", "gprx_cross_matrix", "gprx_deriv_matrix", "gprx_cholesky", "gprx_spd_inverse",
    "gprx_sparse_fit", "gprx_ctx_set_stats", "gprx_ctx_get_stats",
    "gprx_model_set_kernel_matrix", "gprx_model_predict_kx", "gprx_model_posterior_cov_kx", "gprx_model_lml_dk",
    "gprx_model_set_sparse_cov", "gprx_sparse_lml",
    "gprx_device_alloc", "gprx_device_free", "gprx_device_upload", "gprx_device_download",
]


class GprxError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"[{STATUS.get(status, status)}] {msg}")
        self.status = status
        self.msg = msg


class KNode(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("pad", ctypes.c_int32), ("p", ctypes.c_double * 3)]


class KernelDesc(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("pad", ctypes.c_int32), ("node", KNode * MAX_KNODES)]


class KStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int64), ("ms", ctypes.c_double),
                ("flops", ctypes.c_double), ("bytes", ctypes.c_double)]


class FitInfo(ctypes.Structure):
    _fields_ = [("logdet", ctypes.c_double), ("datafit", ctypes.c_double), ("info", ctypes.c_int32),
                ("method", ctypes.c_int32), ("ms_build", ctypes.c_double), ("ms_factor", ctypes.c_double),
                ("ms_solve", ctypes.c_double), ("ms_refine", ctypes.c_double), ("refine_delta", ctypes.c_double),
                ("refine_steps", ctypes.c_int32), ("pad", ctypes.c_int32)]


_lib = None

# gprx_allgather_fn (include/gprx.h): int fn(void* user, const void* send, size_t bytes, void* recv)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def torch_allgather(group=None):
    """A gprx_allgather_fn over torch.distributed (any backend: gloo on the host here): the
    caller-side collective gprx_ctx_create_peer bootstraps with."""
    import torch
    import torch.distributed as dist

    def fn(user, send, nbytes, recv):
        try:
            world = dist.get_world_size(group)
            mine = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=torch.uint8) if nbytes else \
                torch.empty(0, dtype=torch.uint8)
            out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(out, mine, group=group)
            if nbytes:
                ctypes.memmove(recv, b"".join(o.numpy().tobytes() for o in out), nbytes * world)
            return 0
        except Exception:  # reported to the library as a failed collective
            return 1
    return fn


def lib():
    """Load libgprx.so (built in-tree by `make` / __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GprxError(5, f"libgprx.so not built ({LIB_PATH}); run `make`")
        L = ctypes.CDLL(LIB_PATH)
        L.gprx_last_error.restype = ctypes.c_char_p
        L.gprx_last_error.argtypes = [ctypes.c_void_p]
        L.gprx_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.gprx_device_alloc.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]
        L.gprx_device_free.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_device_upload.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.gprx_device_download.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.gprx_ctx_create_dist.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_void_p)]
        L.gprx_ctx_create_peer.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ALLGATHER_FN, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_void_p)]
        L.gprx_dev_dist_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
        L.gprx_dev_ctx_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
        L.gprx_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.gprx_model_create.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.gprx_model_destroy.argtypes = [ctypes.c_void_p]
        L.gprx_model_set_data.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int32, ctypes.c_int32]
        L.gprx_model_set_kernel.argtypes = [ctypes.c_void_p, ctypes.POINTER(KernelDesc)]
        L.gprx_model_set_noise.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.gprx_model_fit.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(FitInfo)]
        L.gprx_model_get_alpha.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_model_set_alpha.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_model_predict.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_void_p]
        L.gprx_model_posterior_cov.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                               ctypes.c_void_p]
        L.gprx_model_core_matrix.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_model_lml.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                     ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]
        L.gprx_model_set_kernel_matrix.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_model_set_sparse_cov.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_model_predict_kx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_model_posterior_cov_kx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_int64, ctypes.c_void_p]
        L.gprx_model_lml_dk.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_double), ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_double)]
        for f in ("gprx_kernel_matrix", "gprx_deriv_matrix"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(KernelDesc), ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
        L.gprx_cross_matrix.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(KernelDesc), ctypes.c_void_p,
                                        ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.c_void_p]
        for f in ("gprx_cholesky", "gprx_spd_inverse"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.POINTER(ctypes.c_int32)]
        L.gprx_sparse_fit.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(KernelDesc), ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.gprx_sparse_lml.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(KernelDesc), ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]
        L.gprx_dist_unique_id.argtypes = [ctypes.c_void_p]
        L.gprx_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.gprx_ctx_set_stats.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.gprx_ctx_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(KStat), ctypes.c_int32,
                                         ctypes.POINTER(ctypes.c_int32)]
        # developer / parity hooks (include/gprx_dev.h)
        L.gprx_ctx_create_virtual.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.gprx_dev_build_matrix.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(KernelDesc),
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                            ctypes.c_int32, ctypes.c_void_p]
        L.gprx_dev_build_time.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(KernelDesc),
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def _check(st, ctx=None):
    if st != 0:
        raise GprxError(st, lib().gprx_last_error(ctx).decode())


def kernel_desc(kernel) -> KernelDesc:
    node = as_node(kernel)
    prog = node.postorder()
    if len(prog) > MAX_KNODES:
        raise GprxError(8, "kernel has too many nodes")
    d = KernelDesc()
    d.n_nodes = len(prog)
    for i, (op, ps) in enumerate(prog):
        d.node[i].op = op
        for j, p in enumerate(ps):
            d.node[i].p[j] = p
    return d


def _dt(dtype):
    dtype = np.dtype(dtype)
    if dtype == np.float64:
        return GPRX_F64
    if dtype == np.float32:
        return GPRX_F32
    raise TypeError(f"unsupported dtype {dtype}")


def _ptr(a):
    """Address of an input: a numpy array (host), or any object with data_ptr() -- e.g. a
    torch CUDA tensor, device memory the library reads without a PCIe copy (gprx.h)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


def _input(a, dtype):
    """A contiguous input of `dtype`: numpy arrays are converted, device tensors are taken as they are
    (they must already be contiguous and of the model's dtype)."""
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous() or str(a.dtype).replace("torch.", "") != np.dtype(dtype).name:
            raise TypeError("device inputs must be contiguous and of the model's dtype")
        return a
    return np.ascontiguousarray(a, dtype)


def runtime_info():
    """The HIP runtime, HSA runtime and RCCL this process has mapped (from /proc/self/maps), and
    whether more than one copy of any is mapped.

    libgprx asks for them by soname (libamdhip64.so.7, librccl.so.1; RUNPATH /opt/rocm/lib).
    The dynamic loader resolves a soname to an object already loaded under that soname first,
    so the binding is set by whichever comes first in the process: loading libgprx first binds
    /opt/rocm's (ROCm 7.2, what it is compiled with, and what bench.py and the tests use); importing
    the PyTorch wheel first binds the copies it bundles (torch/lib), which libgprx then shares.
    Either way there is ONE runtime per process."""
    found = {"libamdhip64": set(), "librccl": set(), "libhsa-runtime64": set()}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) < 6:
                    continue
                path = parts[5]
                base = os.path.basename(path)
                for k in found:
                    if base.startswith(k + ".so"):
                        found[k].add(os.path.realpath(path))
    except OSError:
        pass
    out = {k: sorted(v) for k, v in found.items()}
    out["single_copy"] = all(len(v) <= 1 for v in found.values())
    out["torch_loaded_first"] = any("/torch/lib/" in p for v in found.values() for p in v)
    return out


def device_count():
    c = ctypes.c_int()
    _check(lib().gprx_device_count(ctypes.byref(c)))
    return c.value


def unique_id():
    """RCCL unique id (bytes) for gprx_ctx_create_dist; call on rank 0 and share it."""
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check(lib().gprx_dist_unique_id(buf))
    return buf.raw


def query_shard(q, rank, world):
    """Rows [lo, hi) of Q queries that `rank` of `world` predicts (SURVEY.md 8(e) "Predict:
    shard queries; replicate X, alpha"): contiguous, sizes differing by at most one."""
    if world < 1 or not (0 <= rank < world) or q < 0:
        raise ValueError("query_shard: need 0 <= rank < world and q >= 0")
    return (q * rank) // world, (q * (rank + 1)) // world


class DeviceArray:
    """A copy of a host array in the context's device memory (gprx_device_alloc): inputs that stay
    resident in HBM across calls.  Passes wherever the API takes device inputs (data_ptr()).
    (A framework's CUDA tensors cannot serve once this library owns the device when the framework
    bundles its own HIP runtime, as the PyTorch wheel does.)"""

    def __init__(self, ctx, a=None, *, _base=None, _shape=None, _empty=None):
        if _base is not None:  # a reshaped view of _base's buffer
            self.ctx, self.p, self.dtype, self._base = _base.ctx, _base.p, _base.dtype, _base
            self.shape = tuple(_shape)
            return
        if _empty is not None:  # (shape, dtype): allocated, not initialised
            self.ctx, self.shape, self.dtype, self._base = ctx, tuple(_empty[0]), np.dtype(_empty[1]), None
            p = ctypes.c_void_p()
            ctx._c(lib().gprx_device_alloc(ctx.h, self.nbytes, ctypes.byref(p)))
            self.p = p.value
            return
        a = np.ascontiguousarray(a)
        self.ctx, self.dtype, self.shape, self._base = ctx, a.dtype, a.shape, None
        p = ctypes.c_void_p()
        ctx._c(lib().gprx_device_alloc(ctx.h, a.nbytes, ctypes.byref(p)))
        self.p = p.value
        ctx._c(lib().gprx_device_upload(ctx.h, ctypes.c_void_p(self.p), a.ctypes.data_as(ctypes.c_void_p),
                                        a.nbytes))

    @classmethod
    def empty(cls, ctx, shape, dtype=np.float64):
        """Uninitialised device memory of the given shape (a destination, e.g. sparse_fit's out)."""
        return cls(ctx, _empty=(shape, dtype))

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def nbytes(self):
        return int(np.prod(self.shape)) * self.dtype.itemsize

    def data_ptr(self):
        return self.p or 0

    def is_contiguous(self):
        return True

    def reshape(self, *shape):
        shape = shape[0] if len(shape) == 1 and isinstance(shape[0], tuple) else shape
        shape = list(shape)
        if -1 in shape:
            k = shape.index(-1)
            shape[k] = int(np.prod(self.shape)) // int(np.prod([s for s in shape if s != -1]))
        if int(np.prod(shape)) != int(np.prod(self.shape)):
            raise ValueError("cannot reshape")
        return DeviceArray(None, _base=self._base or self, _shape=shape)

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        self.ctx._c(lib().gprx_device_download(self.ctx.h, out.ctypes.data_as(ctypes.c_void_p),
                                               ctypes.c_void_p(self.p), out.nbytes))
        return out

    def free(self):
        if self._base is None and self.p and self.ctx.h:
            lib().gprx_device_free(self.ctx.h, ctypes.c_void_p(self.p))
        self.p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    """One per process per GPU (gprx_ctx)."""

    def __init__(self, device=0, dist=None, virtual=0, peer=None):
        """dist = (rank, world, unique_id): one RCCL rank per process; virtual = g: g virtual
        ranks of the distributed fit in this process on one GPU (gprx_ctx_create_virtual);
        peer = (rank, world, fn): one rank per process bootstrapped by the caller's all-gather
        fn(send_bytes) -> list of every rank's bytes (gprx_ctx_create_peer), e.g.
        torch_allgather() over a gloo process group."""
        h = ctypes.c_void_p()
        self._cb = None
        if virtual:
            _check(lib().gprx_ctx_create_virtual(device, int(virtual), ctypes.byref(h)))
        elif peer is not None:
            rank, world, fn = peer
            self._cb = ALLGATHER_FN(fn)  # kept alive as long as the context
            _check(lib().gprx_ctx_create_peer(device, rank, world, self._cb, None, ctypes.byref(h)))
        elif dist is None:
            _check(lib().gprx_ctx_create(device, ctypes.byref(h)))
        else:
            rank, world, uid = dist
            buf = ctypes.create_string_buffer(bytes(uid), UNIQUE_ID_BYTES)
            _check(lib().gprx_ctx_create_dist(device, rank, world, buf, ctypes.byref(h)))
        self.h = h

    TRANSPORTS = {0: "single", 1: "rccl", 2: "peer", 3: "virtual"}

    def info(self):
        """Identity of this context (gprx_dev_ctx_info, local): rank, world, HIP device, transport,
        the RCCL communicator's own rank count and rank (ncclCommCount / ncclCommUserRank, -1 with
        no communicator), the device's PCI domain:bus:device and the shared-GPU CU share."""
        v = (ctypes.c_int64 * 10)()
        _check(lib().gprx_dev_ctx_info(self.h, v, 10))
        v = list(v)
        return {"rank": v[0], "world": v[1], "device": v[2], "transport": self.TRANSPORTS.get(v[3], str(v[3])),
                "rccl_count": v[4], "rccl_rank": v[5], "pci": f"{v[6]:04x}:{v[7]:02x}:{v[8]:02x}", "cu_slot": v[9]}

    def close(self):
        if self.h:
            lib().gprx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, st):
        _check(st, self.h)

    def device_array(self, a):
        """`a` copied into this context's device memory (DeviceArray)."""
        return DeviceArray(self, a)

    def set_stats(self, enable=True):
        """Per-kernel HIP-event timing of the library's launches (gprx_ctx_set_stats)."""
        self._c(lib().gprx_ctx_set_stats(self.h, 1 if enable else 0))

    def stats(self):
        arr = (KStat * 16)()
        cnt = ctypes.c_int32()
        self._c(lib().gprx_ctx_get_stats(self.h, arr, 16, ctypes.byref(cnt)))
        return {arr[i].name.decode(): dict(launches=arr[i].launches, ms=arr[i].ms, flops=arr[i].flops,
                                           bytes=arr[i].bytes) for i in range(min(cnt.value, 16))}

    def kernel_matrix(self, kernel, X, dtype=np.float64):
        X = np.ascontiguousarray(X, dtype)
        n, d = X.shape
        K = np.empty((n, n), dtype)
        self._c(lib().gprx_kernel_matrix(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(X), n, d,
                                         _ptr(K)))
        return K

    def deriv_matrix(self, kernel, X, dtype=np.float64):
        X = np.ascontiguousarray(X, dtype)
        n, d = X.shape
        P = as_node(kernel).num_params()
        D = np.empty((P, n, n), dtype)
        self._c(lib().gprx_deriv_matrix(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(X), n, d,
                                        _ptr(D)))
        return D

    def cross_matrix(self, kernel, A, B, dtype=np.float64):
        A = np.ascontiguousarray(A, dtype)
        B = np.ascontiguousarray(B, dtype)
        K = np.empty((A.shape[0], B.shape[0]), dtype)
        self._c(lib().gprx_cross_matrix(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(A), A.shape[0],
                                        _ptr(B), B.shape[0], A.shape[1], _ptr(K)))
        return K

    def build_matrix(self, kernel, X, sigma, path=0, dtype=np.float64):
        """K(X, X) + sigma^2 I exactly as the fit's MFMA pair-statistics build writes it
        (gprx_dev_build_matrix: path 0 = the fused BUILD tasks of the tile factorisation,
        path 1 = the stand-alone kbuild_mma_kernel)."""
        X = np.ascontiguousarray(X, dtype)
        n, d = X.shape
        K = np.empty((n, n), dtype)
        self._c(lib().gprx_dev_build_matrix(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(X), n, d,
                                            float(sigma), path, _ptr(K)))
        return K

    def build_time(self, kernel, X, sigma, path=0, iters=5, dtype=np.float64):
        """Mean device ms of that build alone, features resident (gprx_dev_build_time)."""
        X = np.ascontiguousarray(X, dtype)
        n, d = X.shape
        ms = ctypes.c_double(0)
        self._c(lib().gprx_dev_build_time(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(X), n, d,
                                          float(sigma), path, iters, ctypes.byref(ms)))
        return ms.value

    def cholesky(self, A):
        A = np.array(A, copy=True, order="C")
        info = ctypes.c_int32()
        st = lib().gprx_cholesky(self.h, _dt(A.dtype), _ptr(A), A.shape[0], ctypes.byref(info))
        if st not in (0, 2):
            self._c(st)
        return A, info.value

    def spd_inverse(self, A):
        A = np.array(A, copy=True, order="C")
        info = ctypes.c_int32()
        self._c(lib().gprx_spd_inverse(self.h, _dt(A.dtype), _ptr(A), A.shape[0], ctypes.byref(info)))
        return A

    def sparse_fit(self, kernel, X, Y, Xm, sigma, jitter, dtype=np.float64, out=None):
        """SparseGaussianProcess::Initialize; X, Y may be device arrays (read in HBM, no copy).
        out = (Kinv, RV, RM): caller-owned destinations, host arrays or DeviceArrays (results
        kept in HBM, no PCIe copy); by default new host arrays."""
        X = _input(X, dtype)
        Y = _input(Y, dtype)
        if Y.ndim == 1:
            Y = Y[:, None] if not hasattr(Y, "data_ptr") else Y.reshape(-1, 1)
        Xm = np.ascontiguousarray(Xm, dtype)
        n, d = X.shape
        m = Y.shape[1]
        M = Xm.shape[0]
        if out is None:
            Kinv, RV, RM = np.empty((M, M), dtype), np.empty((M, m), dtype), np.empty((M, M), dtype)
        else:
            Kinv, RV, RM = out
            for a, shp in ((Kinv, (M, M)), (RV, (M, m)), (RM, (M, M))):
                if a is not None and (tuple(a.shape) != shp or np.dtype(a.dtype) != np.dtype(dtype)):
                    raise ValueError(f"sparse_fit: output of shape {tuple(a.shape)} / {a.dtype}, need {shp} / {np.dtype(dtype)}")
        self._c(lib().gprx_sparse_fit(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(X), _ptr(Y), n, d,
                                      m, _ptr(Xm), M, sigma, jitter, _ptr(Kinv), _ptr(RV), _ptr(RM)))
        return Kinv, RV, RM

    def sparse_lml(self, kernel, X, Y, Xm, sigma, jitter, dtype=np.float64, grad=True, compat=False):
        """SparseGaussianLogLikelihood (include/SparseLikelihood.h:231-344) -> (value, grad, logdet)."""
        X = np.ascontiguousarray(X, dtype)
        Y = np.ascontiguousarray(Y, dtype)
        if Y.ndim == 1:
            Y = Y[:, None]
        Xm = np.ascontiguousarray(Xm, dtype)
        n, d = X.shape
        m = Y.shape[1]
        M = Xm.shape[0]
        flags = (LML_GRAD if grad else 0) | (LML_COMPAT if compat else 0)
        v = ctypes.c_double()
        ld = ctypes.c_double()
        npar = ctypes.c_int32()
        g = np.zeros(3 * MAX_KNODES, np.float64)
        self._c(lib().gprx_sparse_lml(self.h, _dt(dtype), ctypes.byref(kernel_desc(kernel)), _ptr(X), _ptr(Y), n, d,
                                      m, _ptr(Xm), M, sigma, jitter, flags, ctypes.byref(v), _ptr(g),
                                      ctypes.byref(npar), ctypes.byref(ld)))
        return v.value, (g[:npar.value].copy() if grad else None), ld.value


class Model:
    """A resident dense GP (gprx_model): GaussianProcess<T> state on the GPU."""

    def __init__(self, ctx: Context, dtype=np.float64):
        self.ctx = ctx
        self.dtype = np.dtype(dtype)
        h = ctypes.c_void_p()
        ctx._c(lib().gprx_model_create(ctx.h, _dt(dtype), ctypes.byref(h)))
        self.h = h
        self.n = self.d = self.m = 0
        self.kernel = None
        self._Xh = None

    def close(self):
        if self.h:
            lib().gprx_model_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, st):
        _check(st, self.ctx.h)

    def set_data(self, X, Y):
        """X (n x d), Y (n x m): host arrays, or DeviceArrays of this context (read in HBM,
        gprx_model_set_data takes host or device memory; a kernel with no device form then needs
        host arrays)."""
        if isinstance(X, DeviceArray) or isinstance(Y, DeviceArray):
            if not (isinstance(X, DeviceArray) and isinstance(Y, DeviceArray)) or X.dtype != self.dtype \
                    or Y.dtype != self.dtype:
                raise TypeError("set_data: X and Y both DeviceArrays of the model's dtype, or both host arrays")
            n, d = X.shape
            m = Y.shape[1] if len(Y.shape) > 1 else 1
            self._c(lib().gprx_model_set_data(self.h, ctypes.c_void_p(X.p), ctypes.c_void_p(Y.p), n, d, m))
            self.n, self.d, self.m = n, d, m
            self._Xh = None
            return
        X = np.ascontiguousarray(X, self.dtype)
        Y = np.ascontiguousarray(Y, self.dtype)
        if Y.ndim == 1:
            Y = Y[:, None]
        n, d = X.shape
        self._c(lib().gprx_model_set_data(self.h, _ptr(X), _ptr(Y), n, d, Y.shape[1]))
        self.n, self.d, self.m = n, d, Y.shape[1]
        self._Xh = X  # host copy: a kernel with no device form is evaluated against it
        if self._host_kernel():
            self._set_host_kernel()

    def set_kernel(self, kernel):
        """A kernel string / node (evaluated on the device), or an object with no device form:
        callable k(Xa, Xb) -> na x nb matrix, optionally with .gradient(Xa, Xb) -> P x na x nb
        (the reference's virtual Kernel::operator() / GetDerivative, include/Kernel.h:52-59).
        The latter is evaluated here on the host; the factorisation and solves stay on the
        device (gprx_model_set_kernel_matrix and the *_kx entry points)."""
        if callable(kernel) and not isinstance(kernel, str) and not hasattr(kernel, "op"):
            self.kernel = kernel
            if self._Xh is not None:  # else set_data evaluates it
                self._set_host_kernel()
            return
        self.kernel = as_node(kernel)
        self._c(lib().gprx_model_set_kernel(self.h, ctypes.byref(kernel_desc(self.kernel))))

    def _host_kernel(self):
        return self.kernel is not None and callable(self.kernel) and not hasattr(self.kernel, "op")

    def _set_host_kernel(self):
        K = np.ascontiguousarray(self.kernel(self._Xh, self._Xh), self.dtype)
        self._c(lib().gprx_model_set_kernel_matrix(self.h, _ptr(K)))

    def set_noise(self, sigma):
        self._c(lib().gprx_model_set_noise(self.h, float(sigma)))

    def fit(self, flags=FIT_DEFAULT):
        info = FitInfo()
        self._c(lib().gprx_model_fit(self.h, flags, ctypes.byref(info)))
        return info

    def dist_info(self):
        """Layout and memory of the last distributed fit (gprx_dev_dist_info): per-rank device
        bytes of the engine and of the packed storage, row-block group, window panels, update
        chunk width, workgroups per rank, simulated makespan (us)."""
        keys = ["bytes_rank", "bytes_storage", "gb", "ww", "chunk_w", "P", "est_us", "world", "dense_factor",
                "posterior_chunks", "posterior_bytes_rank", "push_linv", "push_tiles", "push_bytes", "push_rank"]
        v = (ctypes.c_int64 * len(keys))()
        self._c(lib().gprx_dev_dist_info(self.h, v, len(keys)))
        return dict(zip(keys, list(v)))

    def alpha(self):
        a = np.empty((self.n, self.m), self.dtype)
        self._c(lib().gprx_model_get_alpha(self.h, _ptr(a)))
        return a

    def set_alpha(self, alpha):
        a = np.ascontiguousarray(alpha, self.dtype).reshape(self.n, self.m)
        self._c(lib().gprx_model_set_alpha(self.h, _ptr(a)))

    def predict(self, Xq, deriv=False):
        Xq = np.ascontiguousarray(Xq, self.dtype)
        q = Xq.shape[0]
        mean = np.empty((q, self.m), self.dtype)
        D = np.empty((q, self.d, self.m), self.dtype) if deriv else None
        if self._host_kernel():
            Kx = np.ascontiguousarray(self.kernel(Xq, self._Xh), self.dtype)
            self._c(lib().gprx_model_predict_kx(self.h, _ptr(Kx), _ptr(Xq), q, _ptr(mean), _ptr(D)))
        else:
            self._c(lib().gprx_model_predict(self.h, _ptr(Xq), q, _ptr(mean), _ptr(D)))
        return (mean, D) if deriv else mean

    def posterior_cov(self, Xa, Xb):
        Xa = np.ascontiguousarray(Xa, self.dtype)
        Xb = np.ascontiguousarray(Xb, self.dtype)
        out = np.empty(Xa.shape[0], self.dtype)
        if self._host_kernel():
            Ka = np.ascontiguousarray(self.kernel(Xa, self._Xh), self.dtype)
            Kb = np.ascontiguousarray(self.kernel(Xb, self._Xh), self.dtype)
            kab = np.ascontiguousarray([self.kernel(Xa[i:i + 1], Xb[i:i + 1])[0, 0] for i in range(Xa.shape[0])],
                                       self.dtype)
            self._c(lib().gprx_model_posterior_cov_kx(self.h, _ptr(Ka), _ptr(Kb), _ptr(kab), Xa.shape[0], _ptr(out)))
        else:
            self._c(lib().gprx_model_posterior_cov(self.h, _ptr(Xa), _ptr(Xb), Xa.shape[0], _ptr(out)))
        return out

    def set_sparse_cov(self, W):
        """Make W = Kmm^{-1} - RM resident: posterior_cov then gives the sparse GP's operator()
        (include/SparseGaussianProcess.h:94-106); the model's data are the inducing points."""
        W = np.ascontiguousarray(W, self.dtype)
        self._c(lib().gprx_model_set_sparse_cov(self.h, _ptr(W)))

    def credible_interval(self, Xq):
        """GetCredibleInterval (lib/GaussianProcess.cpp:102-114): 2 sqrt(max(0, gp(x,x)))."""
        c = self.posterior_cov(Xq, Xq)
        return 2 * np.sqrt(np.maximum(c, 0))

    def core_matrix(self):
        C = np.empty((self.n, self.n), self.dtype)
        self._c(lib().gprx_model_core_matrix(self.h, _ptr(C)))
        return C

    def lml(self, grad=True, compat=False, distributed=False, force_lu=False):
        flags = ((LML_GRAD if grad else 0) | (LML_COMPAT if compat else 0) | (LML_DISTRIBUTED if distributed else 0)
                 | (LML_FORCE_LU if force_lu else 0))
        if self._host_kernel():
            dK = np.ascontiguousarray(self.kernel.gradient(self._Xh, self._Xh), self.dtype) if grad else None
            P = dK.shape[0] if grad else 0
            v, ld = ctypes.c_double(), ctypes.c_double()
            g = np.zeros(max(P, 1), np.float64)
            self._c(lib().gprx_model_lml_dk(self.h, flags & ~LML_GRAD, _ptr(dK), P, ctypes.byref(v),
                                            _ptr(g) if grad else None, ctypes.byref(ld)))
            return v.value, (g[:P].copy() if grad else None), ld.value
        v = ctypes.c_double()
        g = np.zeros(MAX_KPARAMS, np.float64)
        npar = ctypes.c_int32()
        ld = ctypes.c_double()
        self._c(lib().gprx_model_lml(self.h, flags, ctypes.byref(v), _ptr(g), ctypes.byref(npar), ctypes.byref(ld)))
        return v.value, (g[:npar.value].copy() if grad else None), ld.value
