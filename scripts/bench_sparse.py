#!/usr/bin/env python3
"""Sparse GP fit throughput (BASELINE.json configs[4]: M=2048 inducing, N=1e6, d=64, fp64,
GaussianKernel(3,1), sigma=0.1, jitter=1e-4), one process per GPU.

Dense rows are sharded over ranks (rank r holds rows r*N/W ..); each rank streams its
Knm blocks into the (M+1) x M normal-equation block, RCCL all-reduces it (the path's one
exchange), then every rank factors the M x M system.  `--n` shrinks N for quick runs.

    python scripts/bench_sparse.py --n 131072
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/bench_sparse.py
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--M", type=int, default=2048)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--lml", type=int, default=1, help="also time the sparse log likelihood + gradient")
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import gpr_amd
    from gpr_amd.synth import make_data
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = tdist
        uid = [gpr_amd.unique_id() if rank == 0 else None]
        tdist.broadcast_object_list(uid, src=0)
        ctx = gpr_amd.Context(local, dist=(rank, world, uid[0]))
    else:
        ctx = gpr_amd.Context(local)
    n, M, d = args.n, args.M, args.d
    ks = "GaussianKernel(3,1,)"
    rows = np.array_split(np.arange(n), world)[rank]
    X, Y = make_data(n, d, 1)
    Xm = X[:: n // M][:M].copy()
    Xl, Yl = X[rows].copy(), Y[rows].copy()
    del X, Y
    for _ in range(args.warmup):
        ctx.sparse_fit(ks, Xl, Yl, Xm, 0.1, 1e-4)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.sparse_fit(ks, Xl, Yl, Xm, 0.1, 1e-4)
    dt = (time.perf_counter() - t0) / args.steps
    if dist:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    flops = 2.0 * n * M * d + n * M * (M + 1) + 2.0 * M ** 3
    if rank == 0:
        print(json.dumps({"metric": "sparse GP fit (M inducing, N dense)", "n": n, "M": M, "d": d, "n_gpus": world,
                          "ms_per_fit": dt * 1e3, "fits_per_s": 1.0 / dt, "tflops_effective": flops / dt / 1e12,
                          "note": "wall time incl. host->device upload of the rank's rows and host outputs"}))
    if args.lml:  # SparseGaussianLogLikelihood value + gradient (gprx_sparse_lml)
        ctx.sparse_lml(ks, Xl, Yl, Xm, 0.1, 1e-4)
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            v, g, ld = ctx.sparse_lml(ks, Xl, Yl, Xm, 0.1, 1e-4)
        dt = (time.perf_counter() - t0) / args.steps
        if dist:
            import torch
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t[0])
        # fit's normal equations + the gradient pass's GEMM K(Xc, Xm) Sigma (2 N M^2) + M^3 inverses
        lflops = flops + 2.0 * n * M * M + 2.0 * M ** 3
        if rank == 0:
            print(json.dumps({"metric": "sparse GP log likelihood + gradient", "n": n, "M": M, "d": d,
                              "n_gpus": world, "ms_per_eval": dt * 1e3, "value": v, "grad": list(g),
                              "tflops_effective": lflops / dt / 1e12,
                              "note": "wall time incl. host->device upload of the rank's rows"}))
    ctx.close()


if __name__ == "__main__":
    main()
