import sys, numpy as np, scipy.sparse as sp, scipy.sparse.linalg as spla
sys.path[:0]=['/root/repo/tests']
from amg_ref import AMGRef, power_lambda

class AMGNE(AMGRef):
    """smoother on the normal equations: x += D^-1 A^T (b - A x) scaled (Cimmino / Chebyshev)"""
    def __init__(self, A, mode="jacobi", **kw):
        super().__init__(A, **kw)
        self.mode=mode
        for L in self.levels:
            A_=L["A"]; At=A_.T.tocsr()
            dn=np.asarray(A_.multiply(A_).sum(axis=0)).ravel()   # diag(A^T A) = column norms^2
            L["At"]=At; L["dninv"]=np.where(dn>0,1/np.where(dn>0,dn,1),1)
            # lambda of D^-1 A^T A (SPD-ish: power iteration is fine)
            n=A_.shape[0]; x=np.ones(n)/np.sqrt(n); lam=0
            for _ in range(30):
                y=L["dninv"]*(At@(A_@x)); lam=np.linalg.norm(y); x=y/lam
            L["lamn"]=lam
    def _sm(self, L, f, x):
        s=max(1,self.sweeps)
        A_,At,dn,lam=L["A"],L["At"],L["dninv"],L["lamn"]
        if self.mode=="jacobi":
            om=1.0/lam
            for _ in range(s):
                r=f-(A_@x if x is not None else 0)
                z=om*dn*(At@r)
                x=z if x is None else x+z
            return x
        # Chebyshev on D^-1 A^T A over [lam/alpha, 1.1 lam]
        b=1.1*lam; a=b/self.alpha; th,de=0.5*(b+a),0.5*(b-a); sg=th/de; rho=1/sg
        if x is None:
            x=np.zeros_like(f); d=dn*(At@f)/th
        else:
            d=dn*(At@(f-A_@x))/th
        for _ in range(s):
            rn=1/(2*sg-rho); t=dn*(At@(f-A_@(x+d))); x=x+d; d=rn*rho*d+2*rn/de*t; rho=rn
        return x+d
    def _vcycle(self, l, f):
        L=self.levels[l]
        if l+1==len(self.levels):
            return self.inv@f if self.inv is not None else self._sm(L,f,None)
        x=self._sm(L,f,None); r=f-L["A"]@x
        x=x+L["P"]@self._vcycle(l+1,L["R"]@r)
        return self._sm(L,f,x)

A=sp.csr_matrix(np.load('/tmp/A_input_turek_2D_Re20_stat.npy')); n=A.shape[0]
prm={'block_size': 3, 'threshold': 1e-14, 'smoother_sweeps': 2, 'coarse_max_size': 100, 'elliptic': False, 'max_levels': 10}
b=np.random.default_rng(3).standard_normal(n)
for mode in ("jacobi","cheb"):
    for sw in (2,4):
        ref=AMGNE(A,mode=mode,**dict(prm,smoother_sweeps=sw))
        res=[]
        x,info=spla.gmres(A,b,M=spla.LinearOperator((n,n),matvec=ref.vmult),rtol=1e-4,restart=28,maxiter=300,callback=lambda r: res.append(r),callback_type='pr_norm')
        print(mode,"sweeps",sw,"sizes",[L["A"].shape[0] for L in ref.levels],"gmres info",info,"its",len(res), "true rel res %.2e"%(np.linalg.norm(b-A@x)/np.linalg.norm(b)))
# plain GMRES for comparison, and smoother only (no coarse)
res=[]; x,info=spla.gmres(A,b,rtol=1e-4,restart=28,maxiter=300,callback=lambda r: res.append(r),callback_type='pr_norm'); print("no preconditioner: info",info,"its",len(res))
