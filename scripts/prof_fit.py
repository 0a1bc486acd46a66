import sys, time
sys.path.insert(0, '.')
import numpy as np, gpr_amd
from tests.helpers import make_data
N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ctx = gpr_amd.Context(0)
X, Y = make_data(N, 32)
M = gpr_amd.Model(ctx, np.float64); M.set_data(X, Y)
M.set_kernel("SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))"); M.set_noise(1.0)
for it in range(2):
    info = M.fit()
    print('build %.3f factor %.3f solve %.3f' % (info.ms_build, info.ms_factor, info.ms_solve), flush=True)
