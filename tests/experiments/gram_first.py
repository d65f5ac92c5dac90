"""Numerical experiment behind DESIGN.md §3.4 "Rejected: Gram-first": W_q from
x4^-1 (Yhat D Yhat^H) x4^-1 vs the TRSM-first order L^-H (Z D Z^H) L^-1 (Z = L^-1 Yhat),
both against the gelsy oracle, on the oracle's own x4/y.  CPU only (numpy).

  python tests/experiments/gram_first.py toy331_fr toy333_fr si_small
"""
import sys, time
import os
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'fft-isdf-scratch_amd'), os.path.dirname(HERE)]
import numpy as np, scipy.linalg as sl
from cases import inputs, oracle
from oracle import isdf_ref as R
for name in sys.argv[1:]:
    cell,kmesh,m0,c0,x0,coords,chi,dm = inputs(name)
    o = oracle(name)
    kpts=R.get_kpts(cell.a,kmesh); phase=R.get_phase(cell.a,kpts,kmesh)
    mesh=cell.mesh; vol=abs(np.linalg.det(cell.a)); N=coords.shape[0]; Gv=R.get_Gv(cell.a,mesh)
    wq=[]; wz=[]
    for q,vq in enumerate(kpts):
        x4=o["x4"][q]; y=o["y"][q]   # y (N, nip)
        fq=np.exp(-1j*coords@vq)
        # gram first: M = Y^T K conj(Y), K = e^{-i q r} conv e^{+i q r}
        yt=y.T*fq
        yh=R.fft(yt,mesh)
        cg=R.get_coulG(cell.a,vq,mesh,Gv=Gv)*vol/N
        # zeta = ifft(fft(z fq) cg) fq^*; W = zeta z^H = sum_r ... Parseval: = (1/N) fft(z fq) cg fft(z fq)^H
        M=(yh*cg)@yh.conj().T/N
        L=np.linalg.cholesky(x4)
        A=sl.solve_triangular(L,M,lower=True)
        A=sl.solve_triangular(L.conj().T,A,lower=False)  # x4^{-1} M
        B=sl.solve_triangular(L,A.conj().T,lower=True)
        B=sl.solve_triangular(L.conj().T,B,lower=False)  # x4^{-1} (x4^{-1}M)^H = x4^-1 M x4^-1
        W=B.conj().T
        # TRSM first (current GPU order)
        Zh=sl.solve_triangular(L,yh,lower=True)
        Mz=(Zh*cg)@Zh.conj().T/N
        Wz=sl.solve_triangular(L.conj().T,sl.solve_triangular(L.conj().T,Mz,lower=False).conj().T,lower=False).conj().T
        wq.append(W); wz.append(Wz)
        ev=np.linalg.eigvalsh(x4)
        if q<3: print(name,q,"cond %.2e"%(ev[-1]/ev[0]),"dW gram %.2e trsm %.2e |W| %.2e"%(abs(W-o["wq"][q]).max(),abs(Wz-o["wq"][q]).max(),abs(o["wq"][q]).max()))
    for lab,w in (("gram",wq),("trsm",wz)):
        w=np.asarray(w)
        vj=R.get_j_kpts(o["xip"],w[0],dm,kpts_band_is_zero=bool(abs(kpts).max()<1e-9))
        vk=R.get_k_kpts(o["xip"],w,dm,phase)
        print(name,lab,"dJ %.2e dK %.2e"%(abs(vj-o["vj"]).max(),abs(vk-o["vk"]).max()))
