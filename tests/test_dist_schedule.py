"""World-size-2 gloo test of the storage-sharded multi-GPU fit and of the distributed LML
gradient reduction (tests/dist_schedule.py restates gprx_dist.cpp / potrf_tiles_kernel<T,
true> and model_lml on a distributed context): each rank stores only its row blocks, the
diagonal inverses are broadcast and the panels exchanged, and every rank ends with alpha,
log det and data fit equal to a single-process solve; the per-rank gradient partials
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


def _worker(rank, world, port, n, B, gb, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from tests.dist_schedule import assemble_L, grad_partial, sharded_fit
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

    alpha, logdet, datafit, tiles, Linv, np_ = sharded_fit(K, Y, 0.5, n, B, rank, world, gb, bcast,
                                                           allgather_obj, allreduce_sum)
    L = assemble_L(tiles, Linv, np_ // B, B)
    Wi = np.linalg.inv(L)
    C = Wi.T @ Wi
    part = grad_partial(alpha[:, :1], C, dK, n, B, rank, world, gb)
    grad = 0.5 * allreduce_sum(part)
    np.savez(out + f"_{rank}.npz", alpha=alpha, logdet=logdet, datafit=datafit, grad=grad, part=part)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,B,gb", [(300, 64, 1), (513, 64, 2), (400, 32, 3)])
def test_sharded_fit_world2(tmp_path, n, B, gb):
    world = 2
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(world, _free_port(), n, B, gb, out), nprocs=world, join=True)
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
    parts = []
    for r in range(world):
        z = np.load(out + f"_{r}.npz")
        assert np.max(np.abs(z["alpha"] - aref)) <= 1e-10 * np.max(np.abs(aref))
        assert abs(float(z["logdet"]) - ldref) <= 1e-10 * abs(ldref)
        assert abs(float(z["datafit"]) - dfref) <= 1e-10 * abs(dfref)
        assert np.max(np.abs(z["grad"] - gref)) <= 1e-9 * np.max(np.abs(gref))
        parts.append(z["part"])
    # each rank's partial covers only its row blocks: the two differ and sum to the gradient
    assert np.max(np.abs(parts[0] - parts[1])) > 0
    assert np.max(np.abs(0.5 * (parts[0] + parts[1]) - gref)) <= 1e-9 * np.max(np.abs(gref))
