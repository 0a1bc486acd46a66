import sys, time
sys.path.insert(0, '.')
import numpy as np, gpr_amd
from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr
ctx = gpr_amd.Context(0)
ks = "PeriodicKernel(0.9,2.5,0.8,)"
for (n, d, m, dt, deriv) in [(200,2,1,np.float64,True),(200,2,1,np.float64,False),(200,8,1,np.float64,True),(517,2,3,np.float64,True),(200,2,1,np.float32,True)]:
    X, Y = make_data(n, d, m)
    M = gpr_amd.Model(ctx, dt); M.set_data(X.astype(dt), Y.astype(dt)); M.set_kernel(ks); M.set_noise(0.5); M.fit()
    a = M.alpha()
    Xq = make_queries(61, d)
    r = M.predict(Xq.astype(dt), deriv=deriv)
    mean = r[0] if deriv else r
    mr = O.predict(ks, X, a.astype(np.float64), Xq)
    print(n, d, m, dt.__name__, deriv, 'mean err', relerr(mean, mr), mean[:3,0], mr[:3,0])
# timing of the north-star fit
for ks2, N, d in [("GaussianKernel(2,1,)", 4096, 16), ("SumKernel(GaussianKernel(2,0.15,),PeriodicKernel(0.1,3.141592653589793,1,))", 16384, 32)]:
    X, Y = make_data(N, d)
    M = gpr_amd.Model(ctx, np.float64); M.set_data(X, Y); M.set_kernel(ks2); M.set_noise(1.0 if N > 5000 else 0.1)
    for it in range(3):
        t0 = time.perf_counter(); info = M.fit(); t1 = time.perf_counter()
        print(N, 'fit wall %.2f ms  build %.3f factor %.3f solve %.3f logdet %.4f' % ((t1-t0)*1e3, info.ms_build, info.ms_factor, info.ms_solve, info.logdet))
