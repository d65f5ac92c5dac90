"""Time the library's FP64-MFMA ZGEMM / HERK at the hot-path shapes (C3) through the C-ABI.
  python tools/gemm_bench.py"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]
import torch  # noqa: E402
from fisdf import _lib as L  # noqa: E402

dev = torch.device("cuda", 0)
ctx = L.Context(0, torch.cuda.current_stream(dev).cuda_stream)
one = (C.c_double * 2)(1.0, 0.0)
mone = (C.c_double * 2)(-1.0, 0.0)
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


def rnd(*shape):
    return torch.randn(*shape, dtype=torch.complex128, device=dev)


QUICK = "--quick" in sys.argv
r, N = 600, 46656
A = rnd(r, N)
Cm = rnd(r, r)
for ks in ((13, 41) if QUICK else (8, 13, 16, 32, 41)):
    ms = timeit(lambda: ctx.call("fisdf_herk", r, N, 1.0, L.ptr(A), N, L.ptr(Cm), r, ks))
    print(f"herk n={r} K={N} ksplit={ks}: {ms:.3f} ms  {4.0 * r * r * N / ms / 1e9:.1f} TF/s", flush=True)
# TRSM-like block GEMMs: C(64 x N) -= L(64 x K) X(K x N)
X = rnd(r, N)
Bm = rnd(r, N)
Lm = rnd(r, r)
for K in (() if QUICK else (64, 128, 256, 512)):
    ms = timeit(lambda: ctx.call("fisdf_zgemm", 0, 0, 64, N, K, mone, L.ptr(Lm), r, 0, L.ptr(X), N, 0,
                                 one, L.ptr(Bm), N, 0, 1, 1))
    print(f"zgemm NN M=64 N={N} K={K}: {ms:.3f} ms  {8.0 * 64 * N * K / ms / 1e9:.1f} TF/s", flush=True)
for M, K in (((600, 600),) if QUICK else ((300, 300), (256, 256), (600, 600), (128, 128))):
    ms = timeit(lambda: ctx.call("fisdf_zgemm", 0, 0, M, N, K, mone, L.ptr(Lm), r, 0, L.ptr(X), N, 0,
                                 one, L.ptr(Bm), N, 0, 1, 1))
    print(f"zgemm NN M={M} N={N} K={K}: {ms:.3f} ms  {8.0 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)
if "--herk-shapes" in sys.argv:
    # tile-waste study: HERK at multiples of 64 vs 600, and the same product as a full GEMM
    for n in (512, 576, 600, 640):
        An = rnd(n, N)
        Cn = rnd(n, n)
        for ks in (13, 32):
            ms = timeit(lambda: ctx.call("fisdf_herk", n, N, 1.0, L.ptr(An), N, L.ptr(Cn), n, ks))
            print(f"herk n={n} ks={ks}: {ms:.3f} ms  {4.0 * n * n * N / ms / 1e9:.1f} TF/s (lower-half flops)", flush=True)
        for ks in (4, 8):
            ms = timeit(lambda: ctx.call("fisdf_zgemm", 0, 3, n, n, N, one, L.ptr(An), N, 0, L.ptr(An), N, 0,
                                         zero, L.ptr(Cn), n, 0, 1, ks))
            print(f"zgemm NC n={n} K={N} ks={ks}: {ms:.3f} ms  {8.0 * n * n * N / ms / 1e9:.1f} TF/s", flush=True)
if "--fx" in sys.argv:
    # the y build's fx GEMM: FX[k] (nip x gb) = X_k (nip x nao) f_k^H, 48 k of a 4x4x4 mesh
    nip, nao, gb, nks = 600, 26, 2330, 48
    Xk = rnd(nks, nip, nao)
    fk = rnd(nks, gb, nao)
    FX = torch.empty(nks, nip, gb, dtype=torch.complex128, device=dev)
    ms = timeit(lambda: ctx.call("fisdf_zgemm", 0, 3, nip, gb, nao, one, L.ptr(Xk), nao, nip * nao,
                                 L.ptr(fk), nao, gb * nao, zero, L.ptr(FX), gb, nip * gb, nks, 1))
    print(f"fx gemm nip={nip} gb={gb} nao={nao} batch={nks}: {ms:.3f} ms  "
          f"{FX.numel() * 16 / ms / 1e6:.0f} GB/s written", flush=True)
