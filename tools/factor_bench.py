"""x4_q factorisation chain alone (fisdf_factor_x4_async + _wait: unpivoted blocked Cholesky,
block-row operator, L^-1) on synthetic Hermitian positive-definite 600 x 600 matrices, for the
batch of one rank at 1 GPU (36 q at C3) and at 8 ranks (4-5 q): ms per call.
  python tools/factor_bench.py [--nip 600] [--batches 36 5 1] [--reps 5]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fft-isdf-scratch_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fisdf import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nip", type=int, default=600)
ap.add_argument("--batches", type=int, nargs="+", default=[36, 5, 1])
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
ctx = L.Context(0, torch.cuda.current_stream().cuda_stream)
g = torch.Generator(device="cuda").manual_seed(3)
for nb in a.batches:
    B = torch.randn((nb, a.nip, 2 * a.nip), dtype=torch.complex128, device="cuda", generator=g)
    x4 = (B @ B.conj().transpose(1, 2)).contiguous()      # Hermitian positive definite
    qs = np.arange(nb, dtype=np.int32)
    ranks = np.zeros(nb, np.int32)

    def run():
        ctx.call("fisdf_factor_x4_async", L.ptr(x4), qs.ctypes.data_as(L._ip), nb, a.nip, 1e-14, None)
        ctx.call("fisdf_factor_x4_wait", ranks.ctypes.data_as(L._ip))
        torch.cuda.synchronize()

    run()
    t = time.perf_counter()
    for _ in range(a.reps):
        run()
    ms = (time.perf_counter() - t) / a.reps * 1e3
    print(f"factor nip {a.nip} batch {nb}: {ms:.3f} ms per call (ranks {ranks.min()}-{ranks.max()})",
          flush=True)
