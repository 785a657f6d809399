"""Extended-precision (numpy longdouble, 80-bit) recomputation of SMLII
(GPR_CS2S3.py:107-141) on the smallest cells of tests/golden/day_ref_fits.npz,
to compare the GPU's objective (a tests/test_gpu_day_t1.py dump, OI_T1_DUMP)
and the reference's 5 observation orders (tests/golden/day_ref_t1.npz) with
the exact value.  Build container only; slow (pure-numpy O(n^3)).
Usage: python tools/t1_extended_precision.py NCELLS [x]   (x: also the GPU-like
float64 emulation with pairwise / exact sums)."""
import numpy as np, sys
sys.path.insert(0,'/root/repo')
fx=np.load('/root/repo/tests/golden/day_ref_fits.npz'); t1=np.load('/root/repo/tests/golden/day_ref_t1.npz')
f=np.load('/root/repo/profiles/r06/t1/gpu_day_t1_dedup1.npz'); gpu,ref=f['gpu'],f['ref']
LD=np.longdouble
def smlii_ld(h,x,y,mean):
    h=np.asarray(h,LD); ell=np.exp(h[:3]); sf2=np.exp(h[3]); sn2=np.exp(h[4])
    xl=np.asarray(x,LD); n=len(y)
    s=np.sqrt(LD(3))*xl/ell
    D=s[:,None,:]-s[None,:,:]; Q=np.sqrt((D**2).sum(-1)); e=np.exp(-Q)
    K=sf2*(1+Q)*e; dK=[sf2*(D[:,:,d]**2)*e for d in range(3)]
    A=K+np.eye(n,dtype=LD)*sn2
    L=np.zeros((n,n),LD)
    for j in range(n):
        v=A[j:,j]-L[j:,:j]@L[j,:j]
        L[j,j]=np.sqrt(v[0]); L[j+1:,j]=v[1:]/L[j,j]
    W=np.zeros((n,n),LD)  # L^-1 by forward substitution on identity
    for i in range(n):
        W[i,:i+1]=(np.eye(n,dtype=LD)[i,:i+1]-L[i,:i]@W[:i,:i+1])/L[i,i]
    Kinv=W.T@W
    r=np.asarray(y,LD)-LD(mean); a=Kinv@r
    nlz=r@a/2+np.log(np.diag(L)).sum()+n*np.log(2*np.pi*LD(1))/2
    Qm=Kinv-np.outer(a,a)
    g=[(Qm*dK[d]).sum()/2 for d in range(3)]+[(Qm*2*K).sum()/2, sn2*np.trace(Qm)]
    return np.array([nlz]+g,LD)
sizes=fx['sizes']; idx=[k for k in np.argsort(sizes) if sizes[k]<=420][:int(sys.argv[1])]
for p in (0,1):
  eg=[];er=[]
  for k in idx:
    a,b=fx['offs'][k],fx['offs'][k+1]
    tr=smlii_ld(t1['hyp'][k,p],fx['x'].reshape(-1,3)[a:b],fx['y'][a:b],float(fx['mean']))
    eg.append(np.abs(gpu[k,p]-tr.astype(float)).astype(float))
    er.append(np.abs(ref[k,p]-tr[None,:]).astype(float))  # orders x q
  eg=np.array(eg); er=np.array(er)
  print('point',p,'cells',len(idx))
  for q,nm in enumerate(['nlZ','g_lx','g_ly','g_lt','g_sf2','g_sn2']):
    print(f"  {nm:6s} median |gpu-truth| {np.median(eg[:,q]):.2e}  median |ref_k-truth| (all orders) {np.median(er[:,:,q]):.2e}  run0 {np.median(er[:,0,q]):.2e}")

def gpu_like(h,x,y,mean,exact):
    import math
    from scipy.linalg import solve_triangular
    ell=np.exp(h[:3]); sf2=np.exp(h[3]); sn2=np.exp(h[4]); n=len(y)
    u=(np.sqrt(3.)*x)/ell
    D=u[:,None,:]-u[None,:,:]; Q=np.sqrt((D**2).sum(-1)); e=np.exp(-Q); K=sf2*((1+Q)*e)
    L=np.linalg.cholesky(K+np.eye(n)*sn2); W=solve_triangular(L,np.eye(n),lower=True); Kinv=W.T@W
    r=y-mean; z=solve_triangular(L,r,lower=True); a=W.T@z
    w0=Kinv-np.outer(a,a)
    il=np.tril_indices(n)
    wgt=np.where(il[0]==il[1],1.0,2.0)
    terms=[wgt*(w0[il]*(sf2*((D[:,:,d]**2)*e)[il])) for d in range(3)]+[wgt*(w0[il]*(2*K[il]))]
    S=(lambda t: math.fsum(t)) if exact else (lambda t: float(np.sum(t)))
    g=[S(t)/2 for t in terms]+[sn2*S(np.diag(w0))]
    return np.array(g)
if len(sys.argv)>2:
  for p in (0,1):
    e0=[];e1=[];er=[]
    for k in idx:
      a,b=fx['offs'][k],fx['offs'][k+1]; x=fx['x'].reshape(-1,3)[a:b]; y=fx['y'][a:b]
      tr=smlii_ld(t1['hyp'][k,p],x,y,float(fx['mean']))[1:].astype(float)
      e0.append(np.abs(gpu_like(t1['hyp'][k,p],x,y,float(fx['mean']),False)-tr))
      e1.append(np.abs(gpu_like(t1['hyp'][k,p],x,y,float(fx['mean']),True)-tr))
      er.append(np.abs(ref[k,p,0,1:]-tr))
    print('point',p,'pairwise-sum W^TW', np.median(e0,0), '\n  exact-sum W^TW', np.median(e1,0), '\n  ref run0', np.median(er,0))
