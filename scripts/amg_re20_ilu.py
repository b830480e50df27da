import sys, numpy as np, scipy.sparse as sp, scipy.sparse.linalg as spla
sys.path[:0]=['/root/repo/tests']
from amg_ref import AMGRef

def iluk(A, k):
    """ILU(k) on the pattern of level-of-fill <= k (dense work on small n; test)"""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    # symbolic: levels
    lev = {}
    rows=[]
    for i in range(n):
        cols = A.indices[A.indptr[i]:A.indptr[i+1]]
        row = {int(c):0 for c in cols}
        # elimination
        ks = sorted(c for c in row if c < i)
        done=set()
        while ks:
            kk = ks.pop(0)
            if kk in done: continue
            done.add(kk)
            lk = row[kk]
            for j,lj in rows[kk].items():
                if j > kk:
                    nl = lk + lj + 1
                    if nl <= k:
                        if j not in row or row[j] > nl:
                            new = j not in row
                            row[j] = nl if j not in row else min(row[j], nl)
                            if new and j < i:
                                ks.append(j); ks.sort()
        rows.append(row)
    # numeric (IKJ) on the pattern
    pat=[sorted(r) for r in rows]
    L=np.zeros((n,n)); U=np.zeros((n,n))
    W=A.toarray().copy()
    LU=np.zeros((n,n))
    for i in range(n):
        w = {j:W[i,j] for j in pat[i]}
        for kk in sorted(j for j in pat[i] if j < i):
            w[kk] = w[kk] / LU[kk,kk]
            for j in pat[kk]:
                if j > kk and j in w:
                    w[j] -= w[kk]*LU[kk,j]
        for j,v in w.items(): LU[i,j]=v
    Lm = np.tril(LU,-1)+np.eye(n); Um=np.triu(LU)
    return sp.csr_matrix(Lm), sp.csr_matrix(Um)

class AMGILU(AMGRef):
    def __init__(self, A, fill=0, **kw):
        super().__init__(A, **kw)
        for L in self.levels[:-1] if self.inv is not None else self.levels:
            L["L"], L["U"] = iluk(L["A"], fill)
    def _smooth(self, L, f, x):
        for _ in range(max(1,self.sweeps)):
            r = f - (L["A"] @ x if x is not None else 0)
            y = spla.spsolve_triangular(L["L"], r, lower=True)
            z = spla.spsolve_triangular(L["U"], y, lower=False)
            x = z if x is None else x + z
        return x
    def _vcycle(self, l, f):
        L = self.levels[l]
        if l + 1 == len(self.levels):
            return self.inv @ f if self.inv is not None else self._smooth(L, f, None)
        x = self._smooth(L, f, None)
        r = f - L["A"] @ x
        xc = self._vcycle(l + 1, L["R"] @ r)
        x = x + L["P"] @ xc
        return self._smooth(L, f, x)

A = sp.csr_matrix(np.load('/tmp/A_input_turek_2D_Re20_stat.npy'))
n=A.shape[0]
prm={'block_size': 3, 'threshold': 1e-14, 'smoother_sweeps': 2, 'coarse_max_size': 100, 'elliptic': False, 'max_levels': 10}
for fill in ():
    ref=AMGILU(A, fill=fill, **prm)
    b=np.random.default_rng(3).standard_normal(n)
    res=[]
    x,info=spla.gmres(A,b,M=spla.LinearOperator((n,n),matvec=ref.vmult),rtol=1e-4,restart=28,maxiter=200,callback=lambda r: res.append(r),callback_type='pr_norm')
    E=np.eye(n)-np.array([ref.vmult(A@np.eye(n)[:,j]) for j in range(n)]).T
    print("ILU(%d): sizes"%fill,[L["A"].shape[0] for L in ref.levels],"gmres info",info,"its",len(res),"rho(I-MA) %.3g"%max(abs(np.linalg.eigvals(E))))

print("--- single-level ILU(k) preconditioner (the reference's Re20 coarse: ML one level, coarse type ILU fill 1)")
for fill in (0,1):
    L,U=iluk(A,fill)
    M=spla.LinearOperator((n,n),matvec=lambda v: spla.spsolve_triangular(U,spla.spsolve_triangular(L,v,lower=True),lower=False))
    b=np.random.default_rng(3).standard_normal(n)
    res=[]
    x,info=spla.gmres(A,b,M=M,rtol=1e-4,restart=28,maxiter=300,callback=lambda r: res.append(r),callback_type='pr_norm')
    print("ILU(%d) alone: gmres info"%fill,info,"its",len(res),"true rel res %.2e"%(np.linalg.norm(b-A@x)/np.linalg.norm(b)), "min |U_ii| %.2e"%abs(U.diagonal()).min())
