import sys
sys.path.insert(0, '.')
import numpy as np, gpr_amd
from oracle import oracle as O
from tests.helpers import make_data, make_queries, relerr
ctx = gpr_amd.Context(0)
bad = 0
for rep in range(40):
    for ks in ["GaussianKernel(0.7,1.3,)", "PeriodicKernel(0.9,2.5,0.8,)"]:
        X, Y = make_data(200, 2)
        M = gpr_amd.Model(ctx, np.float64); M.set_data(X, Y); M.set_kernel(ks); M.set_noise(0.5); M.fit()
        a = M.alpha(); Xq = make_queries(61, 2)
        mean, D = M.predict(Xq, deriv=True)
        e = relerr(mean, O.predict(ks, X, a, Xq))
        if e > 1e-9:
            bad += 1; print('BAD', rep, ks, e, mean[:3, 0])
print('bad', bad)
