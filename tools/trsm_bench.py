"""Isolated timing of the fit's big NN products at C3 shapes through fisdf_zgemm_mode:
U = L^-1 Yhat (A lower triangular, complex and real-A modes) and a full NN GEMM.
  python tools/trsm_bench.py        (FISDF_GEMM_WIDE=0 for the 64 x 64 kernel)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from fisdf import _lib as L  # noqa: E402

dev = torch.device("cuda", 0)
ctx = L.Context(0, torch.cuda.current_stream(dev).cuda_stream)
one = (C.c_double * 2)(1.0, 0.0)
zero = (C.c_double * 2)(0.0, 0.0)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


r, N = 600, 46656
Lm = torch.tril(torch.randn(r, r, dtype=torch.complex128, device=dev))
Y = torch.randn(r, N, dtype=torch.complex128, device=dev)
U = torch.empty_like(Y)
tag = "wide" if os.environ.get("FISDF_GEMM_WIDE", "1") != "0" else "64x64"
for mode, name, n_cols, flop in ((0, "NN full", N, 8.0 * r * r * N), (4, "TRSM (A lower)", N, 4.0 * r * r * N),
                                 (5, "TRSM real A, half grid", 24624, 2.0 * r * r * 24624)):
    ms = timeit(lambda: ctx.call("fisdf_zgemm_mode", 0, 0, r, n_cols, r, one, L.ptr(Lm), r, 0,
                                 L.ptr(Y), N, 0, zero, L.ptr(U), N, 0, 1, mode))
    print(f"{tag:6s} {name:24s} {ms:.3f} ms  {flop / ms / 1e9:.1f} TF/s (algorithmic)", flush=True)
