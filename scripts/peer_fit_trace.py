"""Multi-process sharded C3 fits with every rank on ONE GPU (GPRX_DIST_SHARED_GPU, peer context
over gpr_amd.hostcoll sockets), per-rank tile timelines dumped (GPRX_DIST_TRACE_FILE) for the last
fit: python scripts/peer_fit_trace.py <rank> <world> <port> <N> <fits> <trace prefix>"""
import os
import sys
import time

import numpy as np

rank, world, port, n, nfit, pref = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]),
                                    int(sys.argv[5]), sys.argv[6])
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPRX_DIST_SHARED_GPU"] = "1"
import gpr_amd  # noqa: E402
from gpr_amd.hostcoll import SocketGroup  # noqa: E402
from gpr_amd.synth import C3, make_data  # noqa: E402

grp = SocketGroup(rank, world, port=port)
ctx = gpr_amd.Context(0, peer=(rank, world, grp.allgather_fn()))
X, Y = make_data(n, C3["d"], C3["m"])
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel(C3["kernel"])
M.set_noise(C3["sigma"])
for i in range(nfit):
    if i == nfit - 1:
        os.environ["GPRX_DIST_TRACE_FILE"] = pref
    t0 = time.perf_counter()
    info = M.fit(gpr_amd.gprx.FIT_DISTRIBUTED)
    print(f"rank {rank} fit {i}: {1e3 * (time.perf_counter() - t0):.1f} ms wall, factor {info.ms_factor:.1f} ms",
          flush=True)
print("dist_info", rank, M.dist_info(), flush=True)
M.close()
ctx.close()
grp.barrier()
grp.close()
