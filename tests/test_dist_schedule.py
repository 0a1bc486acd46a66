"""World-size-2 gloo test of the multi-GPU fit schedule (tests/dist_schedule.py restates
potrf_dist / the sharded build): every rank ends with the full factor and the forward-solved
label rows, identical to a single-process Cholesky."""
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


def _worker(rank, world, port, n, NBO, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from tests.dist_schedule import build_owned, potrf_dist
    from oracle import oracle as O
    from gpr_amd.synth import make_data
    ks = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
    X, Y = make_data(n, 4, 2)
    Kfull = O.kernel_matrix(ks, X)
    np_ = -(-n // NBO) * NBO
    ld = np_ + 128
    A = build_owned(Kfull, Y, 0.5, n, np_, ld, NBO, rank, world)

    def bcast(buf, root):
        t = torch.from_numpy(buf)
        dist.broadcast(t, src=root)
        buf[:] = t.numpy()

    A = potrf_dist(A, np_, NBO, rank, world, bcast)
    L = np.tril(A[:n, :n])
    Z = A[np_:np_ + 2, :n]
    np.save(out + f"_L{rank}.npy", L)
    np.save(out + f"_Z{rank}.npy", Z)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,NBO", [(300, 64), (513, 128)])
def test_panel_cyclic_factor_world2(tmp_path, n, NBO):
    world = 2
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(world, _free_port(), n, NBO, out), nprocs=world, join=True)
    from oracle import oracle as O
    from gpr_amd.synth import make_data
    ks = "SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"
    X, Y = make_data(n, 4, 2)
    K = O.kernel_matrix(ks, X) + 0.25 * np.eye(n)
    Lref = np.linalg.cholesky(K)
    Zref = np.linalg.solve(Lref, Y).T
    for r in range(world):
        L = np.load(out + f"_L{r}.npy")
        Z = np.load(out + f"_Z{r}.npy")
        assert np.max(np.abs(L - Lref)) <= 1e-10 * np.max(np.abs(Lref))
        assert np.max(np.abs(Z - Zref)) <= 1e-10 * np.max(np.abs(Zref))
