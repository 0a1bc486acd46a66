#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle (oracle/).

The oracle restates the reference's algorithm (kernel pair loop, LAPACK dgetrf+dgetri LU
inverse in fp64, alpha = C Y, predict / derivative / posterior formulas, LML with the
long-double determinant) and is itself pinned to the reference's own known-answer tests
(tests/test_oracle_kats.py).  The fixtures freeze its outputs on small inputs so the GPU
parity tests (tests/test_golden.py) compare the HIP path with committed vectors, and the
CPU suite detects any drift of the oracle.

Inputs:
* synthetic cases: SplitMix64 data (gpr_amd/synth.py), n = 64, d = 3, m = 2 (m = 1 for
  the likelihood), one case per kernel family and scalar type;
* breathing1D: the reference's own test data file tests/data/breathing1D.mat (copied
  verbatim here; MatrixIO format, 1 x 3773 fp64), first 200 samples as a 1-D regression.

    python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from gpr_amd.synth import make_data, make_queries  # noqa: E402

KERNELS = {
    "gauss": "GaussianKernel(0.7,1.3,)",
    "periodic": "PeriodicKernel(0.9,2.5,0.8,)",
    "rq": "RationalQuadraticKernel(1.1,0.6,1.5,)",
    "gaussexp": "GaussianExpKernel(-0.3,0.1,)",
    "sum_c3": "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))",
    "product": "ProductKernel(GaussianKernel(1.5,1,),PeriodicKernel(1,1.3,0.9,))",
    "white_sum": "SumKernel(GaussianKernel(0.8,1,),WhiteKernel(0.3,))",
}
N, D, M, Q, SIGMA = 64, 3, 2, 16, 0.5


def read_matrixio(path):
    """The reference's matrix file format (lib/MatrixIO.cpp:38-100): 'rows cols\\n' + raw
    row-major fp64."""
    raw = open(path, "rb").read()
    nl = raw.index(b"\n")
    r, c = (int(v) for v in raw[:nl].split())
    return np.frombuffer(raw[nl + 1:nl + 1 + 8 * r * c], dtype=np.float64).reshape(r, c)


def synthetic_case(name, ks, dtype):
    X, Y = make_data(N, D, M)
    X, Y = X.astype(dtype), Y.astype(dtype)
    Xq = make_queries(Q, D).astype(dtype)
    K = O.kernel_matrix(ks, X, dtype)
    alpha, C = O.fit(ks, X, Y, SIGMA, dtype)
    mean, Dm = O.predict(ks, X, alpha, Xq, dtype, with_deriv=True)
    cov = O.posterior_cov(ks, X, C, Xq, Xq[::-1].copy(), dtype)
    val, grad, det, logdet = O.lml(ks, X, Y[:, :1], SIGMA, dtype)
    return dict(kernel=np.array(ks), sigma=np.array(SIGMA), X=X, Y=Y, Xq=Xq, K=K, alpha=alpha, C=C, mean=mean,
                D=Dm, cov=cov, lml=np.array(val, dtype=np.float64), lml_grad=np.asarray(grad, dtype=np.float64),
                logdet=np.array(logdet))


def breathing_case():
    y = read_matrixio(os.path.join(HERE, "breathing1D.mat"))[0, :200]
    X = (np.arange(200, dtype=np.float64) / 200.0)[:, None]
    Y = y[:, None].copy()
    ks = "GaussianKernel(0.05,0.2,)"
    sigma = 0.01
    Xq = ((np.arange(50, dtype=np.float64) + 0.5) / 50.0)[:, None]
    alpha, C = O.fit(ks, X, Y, sigma)
    mean, Dm = O.predict(ks, X, alpha, Xq, with_deriv=True)
    val, grad, det, logdet = O.lml(ks, X, Y, sigma)
    return dict(kernel=np.array(ks), sigma=np.array(sigma), X=X, Y=Y, Xq=Xq, alpha=alpha, mean=mean, D=Dm,
                lml=np.array(val), lml_grad=np.asarray(grad), logdet=np.array(logdet))


def main():
    for name, ks in KERNELS.items():
        for dtype, tag in ((np.float64, "f64"), (np.float32, "f32")):
            np.savez_compressed(os.path.join(HERE, f"{name}_{tag}.npz"), **synthetic_case(name, ks, dtype))
    np.savez_compressed(os.path.join(HERE, "breathing1D_f64.npz"), **breathing_case())
    print("wrote", len(KERNELS) * 2 + 1, "fixtures")


if __name__ == "__main__":
    main()
