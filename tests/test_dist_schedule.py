"""World-size-2/3 gloo test of the storage-sharded multi-GPU fit (tests/dist_schedule.py restates
gprx_dist.cpp / potrf_tiles_kernel<T, true> / k_dsolve.hip): each rank stores only the lower
tiles of its row blocks, the diagonal inverses are pushed to every rank and the factored tiles
into bounded, flow-controlled windows; the back substitution sums the ranks' partials at each
block's owner.  Every rank ends with alpha, log det and data fit equal to a single-process solve;
in LML mode the C tiles each rank accumulated give its gradient partial, and the partials
all-reduce to the full gradient."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gauss(X, sig, sc):
    r2 = np.sum((X[:, None, :] - X[None, :, :]) ** 2, axis=-1)
    e = np.exp(-0.5 * r2 / sig ** 2)
    K = sc * sc * e
    # d/d sigma, d/d scale (include/Kernel.h:471-479 order)
    return K, [sc * sc * r2 / sig ** 3 * e, 2.0 * sc * e]


def _worker(rank, world, port, n, B, gb, ww, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from tests.dist_schedule import forward_substitution, back_substitution, grad_partial_tiles, sharded_fit
    from gpr_amd.synth import make_data
    X, Y = make_data(n, 3, 2)
    K, dK = _gauss(X, 0.9, 1.1)

    def bcast(buf, root):
        t = torch.from_numpy(buf)
        dist.broadcast(t, src=root)
        buf[:] = t.numpy()

    def allgather_obj(obj):
        res = [None] * world
        dist.all_gather_object(res, obj)
        return res

    def allreduce_sum(a):
        t = torch.from_numpy(np.array(a, dtype=np.float64, copy=True))  # all_reduce is in place
        dist.all_reduce(t)
        return t.numpy()

    r = sharded_fit(K, Y, 0.5, n, B, rank, world, gb, ww, bcast, allgather_obj, allreduce_sum, inv=True)
    part = grad_partial_tiles(r["alpha"][:, :1], r["C"], dK, n, B)
    grad = 0.5 * allreduce_sum(part)
    # the refinement's correction solve through the sharded factor: (L L^T)^{-1} rhs
    nc = -(-n // B)
    rhs = np.zeros((nc * B, 2))
    rhs[:n] = Y
    z = forward_substitution(r["T"], r["Linv"], rhs, nc, B, rank, world, gb, allgather_obj)
    sol = back_substitution(r["T"], r["Linv"], {k: z[k * B:(k + 1) * B] for k in range(nc)}, nc, B, 2, rank, world,
                            gb, allgather_obj)
    np.savez(out + f"_{rank}.npz", alpha=r["alpha"], logdet=r["logdet"], datafit=r["datafit"], grad=grad, part=part,
             stored=r["stored"], window_max=r["window_max"], sol=sol[:n])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,B,gb,ww", [(2, 300, 64, 1, 2), (2, 513, 64, 2, 3), (3, 400, 32, 3, 4),
                                              (3, 700, 64, 1, 16)])
def test_sharded_fit_gloo(tmp_path, world, n, B, gb, ww):
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(world, _free_port(), n, B, gb, ww, out), nprocs=world, join=True)
    from gpr_amd.synth import make_data
    X, Y = make_data(n, 3, 2)
    K, dK = _gauss(X, 0.9, 1.1)
    Kn = K + 0.25 * np.eye(n)
    aref = np.linalg.solve(Kn, Y)
    ldref = np.linalg.slogdet(Kn)[1]
    dfref = float(np.sum(Y * aref))
    C = np.linalg.inv(Kn)
    a1 = aref[:, 0]
    gref = np.array([0.5 * np.trace((np.outer(a1, a1) - C) @ D) for D in dK])
    parts, stored = [], 0
    nc = -(-n // B)
    for r in range(world):
        z = np.load(out + f"_{r}.npz")
        assert np.max(np.abs(z["alpha"] - aref)) <= 1e-10 * np.max(np.abs(aref))
        assert np.max(np.abs(z["sol"] - aref)) <= 1e-10 * np.max(np.abs(aref))
        assert abs(float(z["logdet"]) - ldref) <= 1e-10 * abs(ldref)
        assert abs(float(z["datafit"]) - dfref) <= 1e-10 * abs(dfref)
        assert np.max(np.abs(z["grad"] - gref)) <= 1e-9 * np.max(np.abs(gref))
        assert int(z["window_max"]) <= ww
        parts.append(z["part"])
        stored += int(z["stored"])
    # each rank's partial covers only its row blocks; together they are the gradient
    assert np.max(np.abs(parts[0] - parts[1])) > 0
    assert np.max(np.abs(0.5 * sum(parts) - gref)) <= 1e-9 * np.max(np.abs(gref))
    # the ranks together store the lower factor once (+ label, U and C tiles), never N^2 each
    lower = nc * (nc + 1) // 2 + nc + nc * (nc + 1) // 2 + nc * (nc + 1) // 2
    assert stored == lower * B * B
