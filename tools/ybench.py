"""y-build microbenchmark at C3 shape (nk 64, ngrid 36^3, nao 26, nip 600, the 36 time-reversal
representatives): ms per fisdf_build_y_qs call on synthetic inputs.
  python tools/ybench.py [--reps 5]     (FISDF_LIB_VARIANT / FISDF_Y_PIPE / FISDF_YBLK_MB apply)"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fft-isdf-scratch_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fisdf import _lib as L  # noqa: E402
from fisdf import kshard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--nip", type=int, default=600)
args = ap.parse_args()
kmesh, ngrid, nao, nip = (4, 4, 4), 36 ** 3, 26, args.nip
nk = 64
g = torch.Generator(device="cuda").manual_seed(1)
f = torch.randn((nk, ngrid, nao), dtype=torch.complex128, device="cuda", generator=g)
X = torch.randn((nk, nip, nao), dtype=torch.complex128, device="cuda", generator=g)
reps, _, _ = kshard.time_reversal_reps(kmesh)
qs = np.ascontiguousarray(reps, dtype=np.int32)
yT = torch.empty((len(qs), nip, ngrid), dtype=torch.complex128, device="cuda")
ctx = L.Context(0, torch.cuda.current_stream().cuda_stream)
km, kmp = L.iarr(kmesh)
a, ap_ = L.darr(np.eye(3).ravel() * 6.74)
ctx.call("fisdf_set_time_reversal", 1)


def run():
    ctx.call("fisdf_build_y_qs", L.ptr(f), ngrid * nao, 0, ngrid, ngrid, L.ptr(X), nip, nao, kmp,
             ap_, qs.ctypes.data_as(L._ip), len(qs), L.ptr(yT))


run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(args.reps):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / args.reps
gb = (len(qs) * 3) * nip * ngrid * 16 / 1e9
print(f"y build [{os.environ.get('FISDF_LIB_VARIANT', '')}] nq {len(qs)}: {ms:.3f} ms/call "
      f"(fx written + read + y written at 36 slots: {gb:.1f} GB -> {gb / ms:.2f} TB/s)", flush=True)
