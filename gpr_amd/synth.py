"""Deterministic synthetic GP workloads.

SplitMix64, seed 0x47505231 ("GPR1"): X[i,k] = u(i*d+k) with u = (splitmix64(seed+idx)>>11) 2^-53;
labels Y = sin(2 pi x0) + 0.5 cos(2 pi x_{1 mod d}) + 0.1 (2u'-1) with u' from stream seed+0x9E37;
queries from stream seed+0x51.  Identical on CPU, GPU and in the committed fixtures.
"""
import numpy as np

SEED = 0x47505231
_M64 = (1 << 64) - 1

# BASELINE.json configs (the bench and parity tests use exactly these shapes/kernels)
C3_KERNEL = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
C3 = dict(n=16384, d=32, m=1, sigma=1.0, kernel=C3_KERNEL, dtype="f64")
C2 = dict(n=4096, d=16, m=1, sigma=0.1, kernel="GaussianKernel(1,1,)", dtype="f64")
C4 = dict(n=32768, d=32, m=1, sigma=1.0, kernel="RationalQuadraticKernel(1,0.3,1,)", dtype="f32")


def splitmix64(idx):
    z = (np.asarray(idx, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(stream_seed, count):
    idx = np.arange(count, dtype=np.uint64) + np.uint64(stream_seed)
    return (splitmix64(idx) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def make_data(n, d, m=1, seed=SEED, dtype=np.float64):
    X = uniform(seed, n * d).reshape(n, d)
    noise = uniform(seed + 0x9E37, n * m).reshape(n, m)
    base = np.sin(2 * np.pi * X[:, 0]) + 0.5 * np.cos(2 * np.pi * X[:, 1 % d])
    Y = base[:, None] + 0.1 * (2 * noise - 1)
    return X.astype(dtype), Y.astype(dtype)


def make_queries(q, d, seed=SEED, dtype=np.float64):
    return uniform(seed + 0x51, q * d).reshape(q, d).astype(dtype)
