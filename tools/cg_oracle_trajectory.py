"""CPU: scipy CG driven by the oracle (the reference's GPR:107-141 SMLII, n x n)
on day-fixture cell 37, recording every evaluated hyper-vector and nlZ
(profiles/r04/t3/cell37_oracle_trajectory.npz, read by
tools/cg_trajectory_check.py on the GPU box).  Run from the repo root."""
import numpy as np, time, sys
sys.path.insert(0, '.')
from oracle import gp_oracle as O
from scipy.optimize import minimize
d=np.load('tests/golden/day_ref_fits.npz')
c=37; a,b=d['offs'][c],d['offs'][c+1]
x=d['x'].reshape(-1,3)[a:b]; y=d['y'][a:b]; mean=float(d['mean'])
mX=np.full(len(y),mean)
rec=[]
def f(h):
    v,g=O.neg_log_ml(h,x,y,mX)
    v=float(np.asarray(v).ravel()[0])
    rec.append((h.copy(),v))
    return v,np.asarray(g,float).ravel()
t=time.time()
r=minimize(f, np.array(O.X0_PRODUCTION), jac=True, method='CG')
print('nfev',r.nfev,'status',r.status, 'fun', r.fun, time.time()-t)
vals=np.array([v for _,v in rec]); print('inf evals', np.sum(~np.isfinite(vals)))
np.savez('profiles/r04/t3/cell37_oracle_trajectory.npz', H=np.array([h for h,_ in rec]), F=vals)
