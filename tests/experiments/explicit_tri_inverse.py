"""Numerical experiment behind the triangular-GEMM TRSM: W_q with
U = L^{-1} Yhat from a triangular solve vs from the explicit triangular inverse
L^{-1} = solve(L, I) applied as a GEMM, both against the gelsy oracle.  CPU only.

  python tests/experiments/explicit_tri_inverse.py toy331_fr
"""
import sys, os
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'fft-isdf-scratch_amd'), os.path.dirname(HERE)]
import numpy as np, scipy.linalg as sl
from cases import inputs, oracle
from oracle import isdf_ref as R
name=sys.argv[1]
cell,kmesh,m0,c0,x0,coords,chi,dm = inputs(name)
o = oracle(name)
kpts=R.get_kpts(cell.a,kmesh); phase=R.get_phase(cell.a,kpts,kmesh)
mesh=cell.mesh; vol=abs(np.linalg.det(cell.a)); N=coords.shape[0]; Gv=R.get_Gv(cell.a,mesh)
res={}
for mode in ("trsm","inv"):
    ws=[]
    for q,vq in enumerate(kpts):
        x4=o["x4"][q]; y=o["y"][q]
        fq=np.exp(-1j*coords@vq)
        yh=R.fft(y.T*fq,mesh)
        cg=R.get_coulG(cell.a,vq,mesh,Gv=Gv)*vol/N/N
        L=np.linalg.cholesky(x4)
        if mode=="trsm": Z=sl.solve_triangular(L,yh,lower=True)
        else:
            Li=sl.solve_triangular(L,np.eye(len(L)),lower=True)
            Z=Li@yh
        Zs=Z*np.sqrt(cg)
        Mz=Zs@Zs.conj().T
        W=sl.solve_triangular(L.conj().T,sl.solve_triangular(L.conj().T,Mz,lower=False).conj().T,lower=False).conj().T
        ws.append(W)
    w=np.asarray(ws)
    vj=R.get_j_kpts(o["xip"],w[0],dm,kpts_band_is_zero=bool(abs(kpts).max()<1e-9))
    vk=R.get_k_kpts(o["xip"],w,dm,phase)
    print(name,mode,"dJ %.2e dK %.2e"%(abs(vj-o["vj"]).max(),abs(vk-o["vk"]).max()))
