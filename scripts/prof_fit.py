"""Two C3 fits (N = 16384 default, d = 32, the C3 kernel tree) for rocprofv3 PMC passes:
small, no torch import, no benchmark loop around it."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import gpr_amd  # noqa: E402
from tests.helpers import make_data  # noqa: E402
N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ctx = gpr_amd.Context(0)
X, Y = make_data(N, 32)
M = gpr_amd.Model(ctx, np.float64)
M.set_data(X, Y)
M.set_kernel("SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))")
M.set_noise(1.0)
for it in range(2):
    info = M.fit()
    print('build %.3f factor %.3f solve %.3f' % (info.ms_build, info.ms_factor, info.ms_solve), flush=True)
