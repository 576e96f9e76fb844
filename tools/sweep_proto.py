#!/usr/bin/env python3
"""Dev prototype (numpy): accuracy of a tile-wise block sweep inverse + block LDL^T against the tiled
Cholesky of the dense kernel, on IPM-like condensed Hessians.  Not part of the product."""
import numpy as np
rng=np.random.default_rng(1)
def sweep_tile_mfma(S, amask=31):
    """kernel formulation: zero pivot rows/cols, one rank-3 'MFMA' per pivot; returns Minv"""
    S=S.copy(); swept=np.zeros(16,bool)
    for blk in range(5):
        if not (amask>>blk)&1: continue
        o=3*blk; pr=range(o,o+3)
        P=S[o:o+3,o:o+3].copy(); t=S[o:o+3,:].copy()   # pivot rows (LDS)
        # Pinv by adjugate
        a,b,c,d,e,f=P[0,0],P[0,1],P[0,2],P[1,1],P[1,2],P[2,2]
        C00=d*f-e*e; C01=c*e-b*f; C02=b*e-c*d; C11=a*f-c*c; C12=b*c-a*e; C22=a*d-b*b
        det=a*C00+b*C01+c*C02; idt=1/det
        Pinv=np.array([[C00,C01,C02],[C01,C11,C12],[C02,C12,C22]])*idt
        A=np.zeros((16,4)); B=np.zeros((4,16))
        for m in range(16):
            A[m,:3]= -np.eye(3)[m-o] if m in pr else t[:,m]
        for n in range(16):
            B[:3,n]= -Pinv[:,n-o] if n in pr else Pinv@t[:,n]
        S[o:o+3,:]=0; S[:,o:o+3]=0
        S=S-A@B
        swept[o:o+3]=True
    Minv=-S
    for r in range(16):
        if not swept[r]: Minv[r,r]=1.0
    return Minv
def tiled_ldl_solve(M, rhs):
    T=[[M[16*i:16*i+16,16*j:16*j+16].copy() for j in range(4)] for i in range(4)]
    Minv=[None]*4; Z=[[None]*4 for _ in range(4)]
    for b in range(4):
        Minv[b]=sweep_tile_mfma(T[b][b])
        for c in range(b+1,4): Z[b][c]=Minv[b]@T[b][c]
        for c in range(b+1,4):
            for d in range(c,4): T[c][d]=T[c][d]-T[b][c].T@Z[b][d]
    y=[rhs[16*b:16*b+16].copy() for b in range(4)]
    for b in range(4):
        for a in range(b): y[b]-=Z[a][b].T@y[a]
    x=[Minv[b]@y[b] for b in range(4)]
    for b in range(3,-1,-1):
        for c in range(b+1,4): x[b]-=Z[b][c]@x[c]
    return np.concatenate(x)
# condensed-like H: semi-separable from random dynamics
N=60
G=rng.normal(size=(120,60))*np.repeat(np.triu(np.ones((10,10)))[:, :], 1, axis=0).repeat(12,0)[:, :].repeat(6,1)[:, :60] 
H=G.T@G*50+1e-4*np.eye(60)
for trial in range(5):
    D=np.zeros((60,60))
    for bb in range(20):
        Gc=rng.normal(size=(3,5)); w=10**rng.uniform(-6,9,5)
        D[3*bb:3*bb+3,3*bb:3*bb+3]=(Gc*w)@Gc.T
    Mc=H+D
    # pad to 4 tiles of 15 + identity slot
    M=np.eye(64)
    idx=[16*(b//5)+3*(b%5)+a for b in range(20) for a in range(3)]
    M[np.ix_(idx,idx)]=Mc
    x=rng.normal(size=64); r=M@x
    xs=tiled_ldl_solve(M,r)
    print("cond %.1e tiled-sweep-ldl err %.2e  np.solve err %.2e"%(np.linalg.cond(Mc), np.abs(xs-x).max()/np.abs(x).max(), np.abs(np.linalg.solve(M,r)-x).max()/np.abs(x).max()))
def tiled_generic(M, rhs, inv):
    T=[[M[16*i:16*i+16,16*j:16*j+16].copy() for j in range(4)] for i in range(4)]
    Minv=[None]*4; Z=[[None]*4 for _ in range(4)]
    for b in range(4):
        Minv[b]=inv(T[b][b])
        for c in range(b+1,4): Z[b][c]=Minv[b]@T[b][c]
        for c in range(b+1,4):
            for d in range(c,4): T[c][d]=T[c][d]-T[b][c].T@Z[b][d]
    y=[rhs[16*b:16*b+16].copy() for b in range(4)]
    for b in range(4):
        for a in range(b): y[b]-=Z[a][b].T@y[a]
    x=[Minv[b]@y[b] for b in range(4)]
    for b in range(3,-1,-1):
        for c in range(b+1,4): x[b]-=Z[b][c]@x[c]
    return np.concatenate(x)
def tiled_chol(M, rhs):
    T=[[M[16*i:16*i+16,16*j:16*j+16].copy() for j in range(4)] for i in range(4)]
    Ui=[None]*4; U=[[None]*4 for _ in range(4)]
    for b in range(4):
        L=np.linalg.cholesky(T[b][b]); Li=np.linalg.inv(L)  # U_bb^-T = L^-1
        Ui[b]=Li
        for c in range(b+1,4): U[b][c]=Li@T[b][c]
        for c in range(b+1,4):
            for d in range(c,4): T[c][d]=T[c][d]-U[b][c].T@U[b][d]
    y=[rhs[16*b:16*b+16].copy() for b in range(4)]
    for b in range(4):
        acc=y[b]
        for a in range(b): acc=acc-U[a][b].T@y[a]
        y[b]=Ui[b]@acc
    x=[None]*4
    for b in range(3,-1,-1):
        acc=y[b]
        for c in range(b+1,4): acc=acc-U[b][c]@x[c]
        x[b]=Ui[b].T@acc
    return np.concatenate(x)
rng=np.random.default_rng(1)
for trial in range(5):
    D=np.zeros((60,60))
    for bb in range(20):
        Gc=rng.normal(size=(3,5)); w=10**rng.uniform(-6,9,5)
        D[3*bb:3*bb+3,3*bb:3*bb+3]=(Gc*w)@Gc.T
    Mc=H+D
    M=np.eye(64); M[np.ix_(idx,idx)]=Mc
    x=rng.normal(size=64); r=M@x
    e=lambda xs: np.abs(xs-x).max()/np.abs(x).max()
    print("cond %.1e ldl-sweep %.2e ldl-npinv %.2e tiled-chol %.2e np %.2e"%(np.linalg.cond(Mc), e(tiled_ldl_solve(M,r)), e(tiled_generic(M,r,np.linalg.inv)), e(tiled_chol(M,r)), e(np.linalg.solve(M,r))))
