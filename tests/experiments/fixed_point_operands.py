"""Numerical experiment behind DESIGN.md §3.4 (int8 / Ozaki emulation): the J/K error when
the TRSM and/or HERK operands are rounded to t-bit fixed point (per-row scale), i.e. the
accuracy an exact integer-GEMM emulation with t-bit operands would reach.  CPU only.

  python tests/experiments/fixed_point_operands.py toy331_fr 30 36 42 48
"""
import sys
import os
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'fft-isdf-scratch_amd'), os.path.dirname(HERE)]
import numpy as np, scipy.linalg as sl
from cases import inputs, oracle
from oracle import isdf_ref as R
def trunc_rows(A,t):
    m=np.maximum(abs(A.real).max(1,keepdims=True),abs(A.imag).max(1,keepdims=True))
    e=2.0**np.ceil(np.log2(m+1e-300))
    s=2.0**t/e
    return (np.round(A.real*s)+1j*np.round(A.imag*s))/s
name=sys.argv[1]; ts=[int(x) for x in sys.argv[2:]]
cell,kmesh,m0,c0,x0,coords,chi,dm = inputs(name)
o = oracle(name)
kpts=R.get_kpts(cell.a,kmesh); phase=R.get_phase(cell.a,kpts,kmesh)
mesh=cell.mesh; vol=abs(np.linalg.det(cell.a)); N=coords.shape[0]; Gv=R.get_Gv(cell.a,mesh)
pre=[]
for q,vq in enumerate(kpts):
    x4=o["x4"][q]; y=o["y"][q]
    fq=np.exp(-1j*coords@vq)
    yh=R.fft(y.T*fq,mesh)
    cg=R.get_coulG(cell.a,vq,mesh,Gv=Gv)*vol/N/N
    L=np.linalg.cholesky(x4); Li=sl.solve_triangular(L,np.eye(len(L)),lower=True)
    pre.append((yh,cg,L,Li))
def run(mode,t):
    ws=[]
    for yh,cg,L,Li in pre:
        if mode in("trsm","both"):
            Z=trunc_rows(Li,t)@trunc_rows(yh.T,t).T   # B truncated per column
        else:
            Z=sl.solve_triangular(L,yh,lower=True)
        Zs=Z*np.sqrt(cg)
        if mode in("herk","both"):
            Zs=trunc_rows(Zs,t)
        Mz=Zs@Zs.conj().T
        W=sl.solve_triangular(L.conj().T,sl.solve_triangular(L.conj().T,Mz,lower=False).conj().T,lower=False).conj().T
        ws.append(W)
    w=np.asarray(ws)
    vj=R.get_j_kpts(o["xip"],w[0],dm,kpts_band_is_zero=bool(abs(kpts).max()<1e-9))
    vk=R.get_k_kpts(o["xip"],w,dm,phase)
    return abs(vj-o["vj"]).max(),abs(vk-o["vk"]).max()
print(name,"fp64",run("none",0))
for t in ts:
    for mode in ("herk","trsm","both"):
        print(name,mode,t,"dJ %.2e dK %.2e"%run(mode,t))
